#!/bin/bash
# Fresh-box session (run through gpurun; each call gets a fresh box):
#   1. bench.py first, so its latency probes are the box's first GPU
#      processes (the driver's round-end bench sees the same);
#   2. the assembly GEMM's numerics and its A/B arms (gemm_gen.py PLAIN_VARIANTS);
#   3. optionally (INMODEL=1) the Llama step, TOA_GEMM=asm vs nosk, alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_fresh}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 420 python bench.py --steps 6 --warmup 2 > "$O/bench.json" 2> "$O/bench.err" || exit $?
echo "bench: $(grep '^{' "$O/bench.json" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("submit_to_first_step"))')"
timeout -k 10 200 python -u scripts/asm_gemm_bench.py --check > "$O/check.log" 2>&1 || exit $?
timeout -k 10 420 python -u scripts/asm_gemm_bench.py --rounds 3 --reps 4 --mlp 1 --variants 1,2,3,4,5 \
  --forms qkv.fwd,o.fwd,down.fwd,gate_up.fwd,qkv.dgrad_wt > "$O/variants.log" 2>&1 || exit $?
echo "variants done"
if [ "${INMODEL:-0}" = 1 ]; then
  bash scripts/gpu_ab_env.sh "${1:-r4_fresh}/inmodel" 2 "TOA_GEMM=asm" "TOA_GEMM=nosk" --steps 8 --warmup 3 || exit $?
fi
