#!/bin/bash
# PMC counters for the attention kernels (own run: --pmc with kernel-trace only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/attnpmc; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace --output-format csv -d $O/a -o run -- python3 scripts/attn_bench.py > $O/log_a.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAVES --kernel-trace --output-format csv -d $O/b -o run -- python3 scripts/attn_bench.py > $O/log_b.txt 2>&1
