#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/blasab; mkdir -p $O
for i in 1 2; do
timeout -k 10 300 python bench.py > $O/lt_$i.log 2>&1 || exit $?
TORCH_BLAS_PREFER_HIPBLASLT=0 timeout -k 10 300 python bench.py > $O/rocblas_$i.log 2>&1 || exit $?
done
