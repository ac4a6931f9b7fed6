#!/bin/bash
# MFMA-pipe busy fraction of every hot kernel of the Llama-3-8B step, in
# the model (one counter pass over bench.py --direct, 2 timed steps).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r5_step_pmc}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -s KILL 600 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY \
  -d "$O/p1" -o p1 -- python3 bench.py --direct --steps 2 --warmup 1 > "$O/bench.log" 2>&1 || { tail -5 "$O/bench.log"; exit 1; }
python3 scripts/pmc_summary.py "$O" toa_gemm_tn_asm_plain toa_gemm_tn_asm_swiglu_fwd toa_gemm_tn_asm_swiglu_bwd toa_wgrad_nt_asm toa_attn_dkdv_asm toa_attn_fwd_asm attn_bwd_dqg adamw rms_bwd rms_fwd > "$O/summary.md" || exit 1
find "$O/p1" -name '*.db' -size +30M -delete
cat "$O/summary.md"
