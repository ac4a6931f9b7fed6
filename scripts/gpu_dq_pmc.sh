#!/bin/bash
# HBM traffic of the attention kernels at the bench shape (scripts/probes/attn_pmc.py):
# FETCH_SIZE in one pass, WRITE_SIZE + L2 hit / miss in another; summary via scripts/pmc_summary.py.
set -e
export TMPDIR=/tmp
O=${1:-gpurun_out/dqpmc}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/p1 -o p1 -- python3 scripts/probes/attn_pmc.py
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $O/p2 -o p2 -- python3 scripts/probes/attn_pmc.py
python3 scripts/pmc_summary.py $O attn_fwd_gl toa_attn_fwd_asm attn_bwd_dkdv_ds toa_attn_dkdv_asm attn_bwd_dqg attn_delta > $O/summary.md
