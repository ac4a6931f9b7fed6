#!/bin/bash
# Fresh-box bench (latency probes are the box's first GPU processes) and the
# world-8 ZeRO-1 overlap emulation with and without the pipelined tail, at
# 350 and 200 GB/s (run through gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_overlap}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 420 python bench.py --steps 6 --warmup 2 > "$O/bench.json" 2> "$O/bench.err" || exit $?
echo "bench: $(grep '^{' "$O/bench.json" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("submit_to_first_step",{}).get("samples_s"))')"
for g in 350 200; do
  timeout -k 10 600 python scripts/overlap_emulation.py --out "$O/$g" --gbps $g --steps 6 --warmup 2 \
    --policies "nosk,nosk+TOA_ZERO_PIPE=0" > "$O/$g.log" 2>&1 || exit $?
  tail -1 "$O/$g.log"
done
