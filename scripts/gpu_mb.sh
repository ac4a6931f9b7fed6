#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/mb; mkdir -p $O
for mb in 4 5 6; do
timeout -k 10 400 python bench.py --micro-batch $mb --steps 6 --warmup 2 > $O/mb$mb.log 2>&1 || exit $?
done
