#!/bin/bash
# PMC counters for the attention kernels (own runs: --pmc with kernel-trace only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/attnpmc2; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d $O/a -o run -- python3 scripts/attn_bench.py > $O/log_a.txt 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/b -o run -- python3 scripts/attn_bench.py > $O/log_b.txt 2>&1
rc=$?
find $O -name '*kernel_trace.csv' -size +20M -delete
exit $rc
