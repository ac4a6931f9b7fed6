#!/bin/bash
# World-8 ZeRO-1 overlap emulation in steady state: 20 timed steps (the final
# all-gather of the window, which nothing overlaps, amortised as in the
# driver's 20-step runs), 350 and 200 GB/s, pipelined tail on / off.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_overlap3}; mkdir -p "$O"
export TMPDIR=/tmp
for g in 350 200; do
  timeout -k 10 540 python scripts/overlap_emulation.py --out "$O/s20_$g" --gbps $g --steps 20 --warmup 2 \
    --policies "nosk,nosk+TOA_ZERO_PIPE=0" --timeout 400 > "$O/s20_$g.log" 2>&1 || exit $?
  tail -1 "$O/s20_$g.log"
done
