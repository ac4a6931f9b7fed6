#!/bin/bash
# Round 5: the AdamW that writes the W^T copies itself (toa_adamw_wt) --
# GPU numerics (bit-identical to the flat AdamW + transpose refresh; the
# trainer's W^T and overlap tests) and the in-model A/B against the separate
# refresh (one process, ABBA), then a kernel trace of the step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r5_adamwt}; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "adamw or transposed or overlapped_optimizer or trainer" > "$O/tests.log" 2>&1 || { tail -20 "$O/tests.log"; exit 1; }
timeout -k 10 600 python scripts/wgrad_inmodel_ab.py --arms adamwt=0,adamwt=1 --rounds 8 --steps 4 > "$O/inmodel.log" 2>&1 \
  || { tail -5 "$O/inmodel.log"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --steps 2 --warmup 2 --direct \
  > "$O/prof.log" 2>&1 || { tail -5 "$O/prof.log"; exit 1; }
