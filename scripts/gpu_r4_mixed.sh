#!/bin/bash
# GEMM policy 'mixed' (assembly kernel for the fused MLP and the wide data
# gradients): routing test, one-process in-model A/B against nosk, then the
# assembly forms with every PLAIN_VARIANTS arm (the persistent one included).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_mixed}; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "mixed_policy or first_step" > "$O/tests.log" 2>&1 || { tail -20 "$O/tests.log"; exit 1; }
tail -1 "$O/tests.log"
timeout -k 10 600 python -u scripts/wgrad_inmodel_ab.py --rounds 4 --steps 4 --arms "gemm=nosk,gemm=mixed" > "$O/inmodel_ab.log" 2>&1 || exit $?
tail -1 "$O/inmodel_ab.log"
if [ "${FORMS:-1}" = 1 ]; then
  timeout -k 10 480 python -u scripts/asm_gemm_bench.py --rounds 3 --reps 3 --mlp 1 --variants 1,2,3,4,5 > "$O/forms.log" 2>&1 || exit $?
  echo "forms done"
fi
