#!/bin/bash
# Counters, second set: the assembly TN GEMM and hipBLASLt called alternately
# (same thermal state) at the down projection; the assembly NT weight
# gradient against the HIP one at the gate|up form.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-r4_pmc2}
ASM_PMC_ORDER=interleave ASM_PMC_SHAPE=24576,4096,14336 bash scripts/gpu_asm_pmc.sh "$O/asm_down_il" > "gpurun_out/$O.il.log" 2>&1 || { tail -5 "gpurun_out/$O.il.log"; exit 1; }
cat "gpurun_out/$O/asm_down_il/summary.md"
ASM_PMC_WGRAD=1 ASM_PMC_SHAPE=24576,28672,4096 PMC_KERNELS="toa_wgrad_nt_asm wgrad_nt_kernel" bash scripts/gpu_asm_pmc.sh "$O/wgrad_gate_up" > "gpurun_out/$O.wg.log" 2>&1 || { tail -5 "gpurun_out/$O.wg.log"; exit 1; }
cat "gpurun_out/$O/wgrad_gate_up/summary.md"
