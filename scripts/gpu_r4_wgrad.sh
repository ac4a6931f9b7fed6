#!/bin/bash
# Assembly NT weight gradient on one MI355X (run through gpurun): GPU tests,
# then the Llama wgrad forms against the HIP kernel and hipBLASLt.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_wgrad}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py \
  -k "wgrad_asm or gemm_asm" > "$O/tests.log" 2>&1 || exit $?
echo "tests ok"
timeout -k 10 400 python -u scripts/asm_gemm_bench.py --wgrad --rounds 3 --reps 3 > "$O/wgrad.log" 2>&1 || exit $?
echo "wgrad bench done"
