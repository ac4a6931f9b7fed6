#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/attn
export TMPDIR=/tmp
O=gpurun_out/attn
timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -q -x -k "flash" > $O/pytest_flash.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_flash.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -q > $O/pytest_all.log 2>&1; echo "rc=$?" >> $O/pytest_all.log
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > $O/bench_hipattn.log 2>&1; echo "rc=$?" >> $O/bench_hipattn.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 > $O/prof.log 2>&1; echo "rc=$?" >> $O/prof.log
find $O/prof -name '*kernel_trace.csv' -delete
exit 0
