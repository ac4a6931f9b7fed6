#!/bin/bash
# Round-5 world-8 ZeRO-1 overlap emulation: ring collectives vs copy-engine
# all-gather vs copy-engine all-gather + reduce-scatter (the reduction fused
# into the optimizer), at 350 and 200 GB/s (parallel/emulate.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_overlap2}
mkdir -p "$O"
P="asm,asm+TOA_EMULATE_AG=sdma,asm+TOA_EMULATE_AG=sdma+TOA_EMULATE_RS=sdma"
timeout -k 10 420 python scripts/overlap_emulation.py --out "$O/g350" --gbps 350 --steps 20 --warmup 3 \
  --policies "$P" > "$O/g350.log" 2>&1 || exit $?
timeout -k 10 420 python scripts/overlap_emulation.py --out "$O/g200" --gbps 200 --steps 20 --warmup 3 \
  --policies "$P" > "$O/g200.log" 2>&1
