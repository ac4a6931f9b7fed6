#!/bin/bash
# GPU pass after W^T + ZeRO-1: GPU tests, smoke, bench, rocprof stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/round2; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc" >> $O/$name.log
  echo "$name rc=$rc" >&2; return $rc; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
step bench 600 python bench.py &&
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1
rc=$?
find $O/prof -name '*kernel_trace.csv' -size +30M -delete 2>/dev/null
exit $rc
