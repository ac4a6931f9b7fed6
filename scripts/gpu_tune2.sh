#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tune2; mkdir -p $O
timeout -k 10 900 python scripts/tune_gemm.py --out $O/gemm_tuning_gfx950.json > $O/tune.log 2>&1 || exit $?
cp $O/gemm_tuning_gfx950.json tf_operator_amd/ops/gemm_tuning_gfx950.json
TOA_GEMM=torch timeout -k 10 300 python bench.py > $O/torch.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/tuned.log 2>&1
