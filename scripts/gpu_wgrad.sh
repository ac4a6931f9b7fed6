#!/bin/bash
# hand-written NT wgrad GEMM: numerics + timing vs hipBLASLt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/wgrad; mkdir -p $O
export TMPDIR=/tmp
PYTHONPATH=. timeout -k 10 600 python scripts/wgrad_nt_bench.py "$@" > $O/bench.log 2>&1
