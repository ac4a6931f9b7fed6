#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/comm; mkdir -p $O
timeout -k 10 280 python -m pytest tests/test_comm_gpu.py -q -x > $O/pytest.log 2>&1; rc=$?
echo "rc=$rc" >> $O/pytest.log
exit $rc
