#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/attnscale; mkdir -p $O
for xs in 1 0.1; do for gs in 1 0.0001; do
XS=$xs GS=$gs timeout -k 10 120 python scripts/attn_bench.py >> $O/log.txt 2>&1 || exit $?
done; done
