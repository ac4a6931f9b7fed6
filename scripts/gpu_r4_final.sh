#!/bin/bash
# Round-end validation on a fresh box (run through gpurun):
#   1. bench.py first (the driver's command; its latency probes are the box's
#      first GPU processes);
#   2. the whole GPU test suite;
#   3. __graft_entry__.smoke();
#   4. one N=1 step under rocprofv3 --kernel-trace, per-kernel table.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_final}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 420 python bench.py --steps 8 --warmup 3 > "$O/bench.json" 2> "$O/bench.err" || exit $?
echo "bench: $(grep '^{' "$O/bench.json" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["submit_to_first_step"]["samples_s"])')"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 660 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 || { tail -20 "$O/pytest_gpu.log"; exit 1; }
  tail -1 "$O/pytest_gpu.log"
  timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
  tail -1 "$O/smoke.log"
fi
if [ "${PROF:-1}" = 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/n1" -o run -- \
    python3 bench.py --direct --steps 2 --warmup 1 > "$O/n1.json" 2> "$O/n1.err" || exit $?
  python scripts/step_breakdown.py "$O/n1" xent_fwd > "$O/n1_breakdown.txt" || exit $?
  find "$O/n1" -name '*kernel_trace.csv' -size +20M -delete
  head -25 "$O/n1_breakdown.txt"
fi
