#!/bin/bash
# GPU tests + bench + kernel stats (short)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/quick; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python scripts/attn_bench.py > $O/attn.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 > $O/prof.log 2>&1
rm -f $O/prof/run_kernel_trace.csv
