"""Models of the reference's bundled payloads, rebuilt on the fused HIP ops.

* :class:`MnistMLP` -- dist_mnist.py:166-192 (784 -> 100 ReLU -> 10, 79,510
  params) and mnist_with_summaries.py:76-106 (784 -> 500 ReLU -> dropout ->
  10, 397,510 params): every dense layer is one MFMA ``gemm_bias_act`` launch.
* :class:`KerasCNN` -- multi_worker_strategy-with-keras.py:45-56 (3x Conv3x3
  + 2x MaxPool + Dense64 + Dense10, 93,322 params): convolutions are MIOpen
  (library conv, not a fused op in the reference), dense layers fused HIP.
* :class:`EstimatorDNN` -- keras_model_to_estimator.py:47-52 (10 -> 16 ReLU
  -> 1 sigmoid, 193 params).
* :func:`resnet50` -- BASELINE.json config #2 (ResNet-50, 25.6M params),
  channels-last bf16 convs through MIOpen, BatchNorm + ReLU (+ residual)
  as one fused HIP pass (ops/bn.py), fused dense head.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..ops.bn import FusedBatchNorm2d
from ..ops.mlp import DenseAct


class MnistMLP(torch.nn.Module):
    def __init__(self, hidden=100, keep_prob=1.0, dtype=torch.bfloat16, device=None):
        super().__init__()
        self.hid = DenseAct(784, hidden, "relu", dtype, device, keep_prob=keep_prob)
        self.sm = DenseAct(hidden, 10, "none", dtype, device)
        # dropout draws a fresh host seed per call: a captured graph would freeze it
        self.graph_safe = keep_prob >= 1.0

    def forward(self, x):
        return self.sm(self.hid(x.reshape(x.shape[0], -1)))


class KerasCNN(torch.nn.Module):
    def __init__(self, dtype=torch.bfloat16, device=None):
        super().__init__()
        kw = dict(dtype=dtype, device=device)
        self.c1 = torch.nn.Conv2d(1, 32, 3, **kw)
        self.c2 = torch.nn.Conv2d(32, 64, 3, **kw)
        self.c3 = torch.nn.Conv2d(64, 64, 3, **kw)
        self.d1 = DenseAct(3 * 3 * 64, 64, "relu", dtype, device)
        self.d2 = DenseAct(64, 10, "none", dtype, device)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.c1(x)), 2)
        x = F.max_pool2d(F.relu(self.c2(x)), 2)
        x = F.relu(self.c3(x))
        return self.d2(self.d1(x.flatten(1)))


class EstimatorDNN(torch.nn.Module):
    def __init__(self, dtype=torch.float32, device=None):
        super().__init__()
        self.d1 = DenseAct(10, 16, "relu", torch.bfloat16, device)
        self.d2 = DenseAct(16, 1, "none", torch.bfloat16, device)

    def forward(self, x):
        return self.d2(self.d1(x.to(torch.bfloat16))).float().squeeze(-1)


# ---------------------------------------------------------------------------
# ResNet-50 (He et al. 2015), bottleneck v1.5 (stride on the 3x3)
# ---------------------------------------------------------------------------
class Bottleneck(torch.nn.Module):
    """BatchNorm + ReLU (and, after conv3, the residual add) are one fused
    HIP pass each (ops/bn.py, csrc/hip/bn.hip); convolutions are MIOpen."""

    expansion = 4

    def __init__(self, cin, width, stride=1, downsample=None, **kw):
        super().__init__()
        self.conv1 = torch.nn.Conv2d(cin, width, 1, bias=False, **kw)
        self.bn1 = FusedBatchNorm2d(width, relu=True, **kw)
        self.conv2 = torch.nn.Conv2d(width, width, 3, stride, 1, bias=False, **kw)
        self.bn2 = FusedBatchNorm2d(width, relu=True, **kw)
        self.conv3 = torch.nn.Conv2d(width, width * 4, 1, bias=False, **kw)
        self.bn3 = FusedBatchNorm2d(width * 4, relu=True, **kw)  # relu(bn3(conv3(y)) + identity)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = self.bn1(self.conv1(x))
        y = self.bn2(self.conv2(y))
        return self.bn3(self.conv3(y), residual=idt)


class ResNet(torch.nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes=1000, dtype=torch.bfloat16, device=None):
        super().__init__()
        kw = dict(dtype=dtype, device=device)
        self.stem = torch.nn.Sequential(torch.nn.Conv2d(3, 64, 7, 2, 3, bias=False, **kw),
                                        FusedBatchNorm2d(64, relu=True, **kw), torch.nn.MaxPool2d(3, 2, 1))
        cin = 64
        stages = []
        for i, (n, width) in enumerate(zip(layers, (64, 128, 256, 512))):
            blocks = []
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                ds = None
                if j == 0:
                    ds = torch.nn.Sequential(torch.nn.Conv2d(cin, width * 4, 1, stride, bias=False, **kw),
                                             FusedBatchNorm2d(width * 4, relu=False, **kw))
                blocks.append(Bottleneck(cin, width, stride, ds, **kw))
                cin = width * 4
            stages.append(torch.nn.Sequential(*blocks))
        self.stages = torch.nn.Sequential(*stages)
        self.fc = DenseAct(2048, num_classes, "none", dtype, device)

    def forward(self, x):
        x = self.stages(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def resnet50(num_classes=1000, dtype=torch.bfloat16, device=None):
    return ResNet((3, 4, 6, 3), num_classes, dtype, device)


def num_params(m):
    return sum(p.numel() for p in m.parameters())
