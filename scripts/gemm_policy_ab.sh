#!/bin/bash
# GEMM policy on one MI355X (run through gpurun):
#   1. N=1 step, hipBLASLt heuristic (stream-K) vs the non-stream-K table,
#      alternating runs in one call (same box);
#   2. rocprofv3 kernel traces of the world-8 ZeRO-1 step with emulated
#      collective traffic (parallel/emulate.py) under both policies, and the
#      interleaving summary (scripts/overlap_trace.py).
# Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3_gemm_policy}; mkdir -p "$O"
export TMPDIR=/tmp
for i in 1 2; do
  for pol in torch nosk; do
    TOA_GEMM=$pol timeout -k 10 240 python bench.py --direct --steps 10 --warmup 3 > "$O/n1_${pol}_$i.json" 2> "$O/n1_${pol}_$i.err" || exit $?
    echo "n1 $pol $i: $(python -c "import json;print(json.load(open('$O/n1_${pol}_$i.json'))['ms_per_step'])")"
  done
done
export TOA_EMULATE_WORLD=8 TOA_EMULATE_GBPS=350
for pol in torch nosk; do
  export TOA_GEMM=$pol
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/trace_$pol" -o run -- \
    python3 bench.py --direct --zero 1 --steps 2 --warmup 1 > "$O/trace_$pol.json" 2> "$O/trace_$pol.err" || exit $?
  python scripts/overlap_trace.py "$O/trace_$pol" --out "$O/overlap_$pol.json" > /dev/null || exit $?
  find "$O/trace_$pol" -name '*kernel_trace.csv' -size +20M -delete
  echo "traced $pol"
done
