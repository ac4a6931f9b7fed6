"""tf_operator_amd -- an MI355X-native distributed-training operator.

Control plane: TFJob / PyTorchJob / MXJob / XGBoostJob CRDs reconciled by a
pure C++17 core (:mod:`tf_operator_amd.core`) driven by an asyncio
Kubernetes I/O shell (:mod:`tf_operator_amd.operator`), with a Python SDK
(:mod:`tf_operator_amd.sdk`), an in-process fake API server and a local
kubelet for cluster-free end-to-end tests.

Data plane: PyTorch-ROCm trainers (:mod:`tf_operator_amd.train`,
:mod:`tf_operator_amd.models`) on hand-written gfx950 HIP kernels
(:mod:`tf_operator_amd.ops`) and RCCL collectives over xGMI
(:mod:`tf_operator_amd.parallel`).
"""
from .version import __version__, GIT_SHA, info  # noqa: F401
