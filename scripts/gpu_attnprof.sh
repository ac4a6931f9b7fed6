#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/attnprof; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 scripts/attn_bench.py > $O/log.txt 2>&1; echo "rc=$?" >> $O/log.txt
rm -f $O/run_kernel_trace.csv
