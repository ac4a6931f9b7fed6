#!/bin/bash
# One-process in-model A/B (scripts/wgrad_inmodel_ab.py), then the GPU test
# suite (run through gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r4_inmodel}; mkdir -p "$O"
export TMPDIR=/tmp
if [ "${AB:-1}" = 1 ]; then
  timeout -k 10 480 python -u scripts/wgrad_inmodel_ab.py --rounds 3 --steps 4 ${ARMS:+--arms $ARMS} > "$O/ab.log" 2>&1 || exit $?
  tail -1 "$O/ab.log"
fi
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 660 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > "$O/pytest_gpu.log" 2>&1 || exit $?
  tail -1 "$O/pytest_gpu.log"
fi
