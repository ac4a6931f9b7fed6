#!/bin/bash
# HIP-graph step for the small payloads: tests + throughput with / without graphs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/graph; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -q -x --timeout 120 --timeout-method thread -k "graph or device_step or adamw or fp32_accumulate or bias_act or dense" > $O/pytest.log 2>&1 &&
timeout -k 10 300 python -m tf_operator_amd.examples.dist_mnist --train_steps 5000 --log_every 1000 > $O/mnist_graph.log 2>&1 &&
TOA_HIP_GRAPH=0 timeout -k 10 300 python -m tf_operator_amd.examples.dist_mnist --train_steps 5000 --log_every 1000 > $O/mnist_eager.log 2>&1 &&
timeout -k 10 300 python -m tf_operator_amd.examples.keras_cnn --epochs 4 --steps_per_epoch 200 --saved_model_dir /tmp/kc1 > $O/cnn_graph.log 2>&1 &&
TOA_HIP_GRAPH=0 timeout -k 10 300 python -m tf_operator_amd.examples.keras_cnn --epochs 4 --steps_per_epoch 200 --saved_model_dir /tmp/kc2 > $O/cnn_eager.log 2>&1
