#!/bin/bash
# rocprofv3 kernel traces of one N=1 step and of rank 0's emulated world-8
# ZeRO-1 step without traffic; per-step kernel tables (scripts/step_breakdown.py).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3_prof_pair}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/n1" -o run -- \
  python3 bench.py --direct --steps 2 --warmup 1 > "$O/n1.json" 2> "$O/n1.err" || exit $?
python scripts/step_breakdown.py "$O/n1" xent_fwd > "$O/n1_breakdown.txt" || exit $?
find "$O/n1" -name '*kernel_trace.csv' -size +20M -delete
export TOA_EMULATE_WORLD=8 TOA_EMULATE_BYTES=0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/e8q" -o run -- \
  python3 bench.py --direct --zero 1 --steps 2 --warmup 1 > "$O/e8q.json" 2> "$O/e8q.err" || exit $?
python scripts/step_breakdown.py "$O/e8q" xent_fwd > "$O/e8q_breakdown.txt" || exit $?
find "$O/e8q" -name '*kernel_trace.csv' -size +20M -delete
echo ok
