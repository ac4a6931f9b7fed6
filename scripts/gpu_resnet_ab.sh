#!/bin/bash
# ResNet-50 payload: fused HIP BatchNorm vs PyTorch batch_norm (TOA_BN=torch),
# one process each, same box; plus a rocprofv3 per-step kernel table of the
# fused build.  Output: gpurun_out/$1/
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:?out}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -m tf_operator_amd.examples.resnet_train --steps 20 --warmup 8 --batch 256 > "$O/resnet_hipbn.log" 2>&1 &&
TOA_BN=torch timeout -k 10 300 python -m tf_operator_amd.examples.resnet_train --steps 20 --warmup 8 --batch 256 > "$O/resnet_torchbn.log" 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$O/prof" -o run -- python3 -m tf_operator_amd.examples.resnet_train --steps 4 --warmup 6 --batch 256 > "$O/resnet_prof.log" 2>&1 &&
timeout -k 10 120 python3 scripts/step_breakdown.py "$O/prof" adamw > "$O/step_breakdown.txt" 2>&1
rc=$?
find "$O/prof" -name "*kernel_trace.csv" -delete
exit $rc
