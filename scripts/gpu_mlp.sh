#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/mlp; mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -q -x -k "dense or accuracy" > $O/pytest.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest.log
exit $rc
