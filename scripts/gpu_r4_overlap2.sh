#!/bin/bash
# World-8 ZeRO-1 overlap emulation at 8 and 16 collective channels (RCCL ring
# workgroups), 350 and 200 GB/s, pipelined tail (run through gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_overlap2}; mkdir -p "$O"
export TMPDIR=/tmp
for c in 8 16; do
  for g in 350 200; do
    timeout -k 10 400 python scripts/overlap_emulation.py --out "$O/c${c}_$g" --gbps $g --channels $c --steps 6 \
      --warmup 2 --policies nosk > "$O/c${c}_$g.log" 2>&1 || exit $?
    tail -1 "$O/c${c}_$g.log"
  done
done
