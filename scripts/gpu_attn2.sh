#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/attn2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -q -x -k "flash" > $O/pytest_flash.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_flash.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/attn_bench.py > $O/attn_bench.log 2>&1; echo "rc=$?" >> $O/attn_bench.log
exit 0
