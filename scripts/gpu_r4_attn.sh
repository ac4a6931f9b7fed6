#!/bin/bash
# Attention A/B at the bench shape: backward forms (with the dK/dV kernel's
# issue-vs-wait timing) and forward forms, then a kernel trace of the same run.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_attn}; mkdir -p "$O"
export TMPDIR=/tmp
V=${VARIANTS:-split,ds}
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "attention or rope" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
  tail -2 "$O/tests.log"
fi
timeout -k 10 300 python scripts/attn_bwd_ab.py --variants "$V" --timing --rounds 6 > "$O/ab.log" 2>&1 || exit $?
tail -1 "$O/ab.log"
timeout -k 10 200 python scripts/attn_fwd_ab.py --forms ${FWD:-reg,gl} > "$O/fwd_ab.log" 2>&1 || exit $?
tail -1 "$O/fwd_ab.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 scripts/attn_bwd_ab.py --variants "$V" --rounds 2 --reps 3 > "$O/prof.log" 2>&1 || exit $?
find "$O/prof" -name '*kernel_stats.csv' -exec cp {} "$O/kernel_stats.csv" \;
head -12 "$O/kernel_stats.csv"
