#!/bin/bash
# W^T data-gradient path: kernel tests, isolated GEMM A/B, full-step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/dgrad; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -q -x --timeout 120 --timeout-method thread -k "transpose or dgrad or overlapped" > $O/pytest.log 2>&1 &&
timeout -k 10 300 python scripts/dgrad_bench.py > $O/dgrad_bench.log 2>&1 &&
timeout -k 10 400 python bench.py > $O/bench_wt.log 2>&1 &&
TOA_DGRAD_WT=0 timeout -k 10 400 python bench.py > $O/bench_nowt.log 2>&1
