#!/bin/bash
# Round-4 assembly GEMM session on one MI355X (run through gpurun):
#   1. the plain kernel's A/B arms (gemm_gen.py PLAIN_VARIANTS) against the
#      product kernel and hipBLASLt at the Llama forms;
#   2. the Llama-3-8B step, TOA_GEMM=asm vs nosk, alternating runs.
# Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_asm_ab}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 420 python -u scripts/asm_gemm_bench.py --rounds 3 --reps 4 --mlp 0 --variants 1,2,3,4,5 \
  --forms qkv.fwd,o.fwd,down.fwd,gate_up.fwd,qkv.dgrad_wt > "$O/variants.log" 2>&1 || exit $?
echo "variants done"
bash scripts/gpu_ab_env.sh "${1:-r4_asm_ab}/inmodel" 2 "TOA_GEMM=asm" "TOA_GEMM=nosk" --steps 8 --warmup 3 || exit $?
