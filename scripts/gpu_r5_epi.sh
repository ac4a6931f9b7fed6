#!/bin/bash
# Round 5: the software-pipelined SwiGLU epilogues -- GPU numerics, the fused
# MLP against hipBLASLt + the SwiGLU pass, and the in-model A/B against the
# round-4 epilogues (one process, ABBA).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_epi}; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "swiglu or gemm_asm or mlp" > "$O/tests.log" 2>&1 || { tail -20 "$O/tests.log"; exit 1; }
timeout -k 10 400 python scripts/asm_gemm_bench.py --rounds 4 > "$O/forms.log" 2>&1 || { tail -5 "$O/forms.log"; exit 1; }
timeout -k 10 600 python scripts/wgrad_inmodel_ab.py --arms epi=r4,epi=pipe --rounds 8 --steps 4 > "$O/inmodel.log" 2>&1
