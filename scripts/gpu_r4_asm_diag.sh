#!/bin/bash
# Assembly GEMM diagnosis on one MI355X (run through gpurun):
#   1. wait-cycle breakdown (timing kernel) at every Llama form;
#   2. all forms vs hipBLASLt with the A/B arms;
#   3. optionally (PMC=1) counters at the down-projection forward (K = 14336);
#   4. optionally (INMODEL=1) the Llama step, TOA_GEMM=asm vs nosk, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_diag}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 240 python -u scripts/asm_gemm_bench.py --timing > "$O/timing.log" 2>&1 || exit $?
echo "timing done"
timeout -k 10 480 python -u scripts/asm_gemm_bench.py --rounds 3 --reps 3 --mlp 1 --variants 1,2,3,4,5 > "$O/forms.log" 2>&1 || exit $?
echo "forms done"
if [ "${PMC:-0}" = 1 ]; then
  ASM_PMC_SHAPE=24576,4096,14336 bash scripts/gpu_asm_pmc.sh "${1:-r4_diag}/pmc_down" > "$O/pmc.log" 2>&1 || exit $?
  echo "pmc done"
fi
if [ "${INMODEL:-0}" = 1 ]; then
  bash scripts/gpu_ab_env.sh "${1:-r4_diag}/inmodel" 2 "TOA_GEMM=asm" "TOA_GEMM=nosk" --steps 8 --warmup 3 || exit $?
fi
