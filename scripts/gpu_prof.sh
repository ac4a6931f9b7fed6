#!/bin/bash
# rocprofv3 kernel trace + stats of the flagship bench (short run)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
MODEL=${1:-llama3-8b}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --model $MODEL --steps 2 --warmup 1 > gpurun_out/prof/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc" >> gpurun_out/prof/bench.log
find gpurun_out/prof -name '*stats*' | head
# keep only summaries (kernel trace csv can be large)
find gpurun_out/prof -name '*kernel_trace.csv' -size +30M -delete
exit $rc
