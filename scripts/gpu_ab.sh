#!/bin/bash
# A/B: torch.matmul GEMMs vs the tuned hipBLASLt layer, same box, back to back
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab; mkdir -p $O
for i in 1 2; do
TOA_GEMM=torch timeout -k 10 300 python bench.py > $O/torch_$i.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/tuned_$i.log 2>&1 || exit $?
done
