#!/bin/bash
# Round-4 counters: the assembly GEMM vs hipBLASLt at the down-projection
# forward (K = 14336) and the attention kernels at the bench shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=${1:-r4_pmc}
ASM_PMC_SHAPE=24576,4096,14336 bash scripts/gpu_asm_pmc.sh "$O/asm_down" > "gpurun_out/$O.asm.log" 2>&1 || { tail -5 "gpurun_out/$O.asm.log"; exit 1; }
cat "gpurun_out/$O/asm_down/summary.md"
bash scripts/gpu_attn_pmc.sh > "gpurun_out/$O.attn.log" 2>&1 || { tail -5 "gpurun_out/$O.attn.log"; exit 1; }
mkdir -p "gpurun_out/$O/attn" && cp gpurun_out/attnpmc/summary.md "gpurun_out/$O/attn/summary.md"
cat "gpurun_out/$O/attn/summary.md"
