#!/bin/bash
# Round 5: the ZeRO-1 gradient reduce-scatter by copy-engine pulls -- the
# two-process transport test and the two-rank trainer with both collectives
# on the copy engines (gloo process group carrying only the norm).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_rs}; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_comm_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "pull or copy_engine" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
