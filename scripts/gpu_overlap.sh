#!/bin/bash
# overlapped-optimizer check: numerics test, then serial vs overlapped bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/overlap; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -q -x -k "trainer or embedding" > $O/pytest.log 2>&1 || exit $?
TOA_OPT_OVERLAP=0 timeout -k 10 400 python bench.py --steps 8 --warmup 3 > $O/bench_serial.log 2>&1 || exit $?
TOA_OPT_OVERLAP=1 timeout -k 10 400 python bench.py --steps 8 --warmup 3 > $O/bench_overlap.log 2>&1 || exit $?
TOA_OPT_OVERLAP=0 timeout -k 10 400 python bench.py --steps 8 --warmup 3 > $O/bench_serial2.log 2>&1 || exit $?
TOA_OPT_OVERLAP=1 timeout -k 10 400 python bench.py --steps 8 --warmup 3 > $O/bench_overlap2.log 2>&1
