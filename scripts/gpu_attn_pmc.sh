#!/bin/bash
# LDS / MFMA counters of the attention kernels (scripts/probes/attn_pmc.py):
# two --pmc passes; summary via scripts/pmc_summary.py into gpurun_out/attnpmc/.
set -e
export TMPDIR=/tmp
O=${1:-gpurun_out/attnpmc}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT -d $O/p1 -o p1 -- python3 scripts/probes/attn_pmc.py
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU -d $O/p2 -o p2 -- python3 scripts/probes/attn_pmc.py
python3 scripts/pmc_summary.py $O attn_fwd_gl toa_attn_fwd_asm attn_bwd_dkdv_ds toa_attn_dkdv_asm attn_bwd_dqg attn_delta > $O/summary.md
