#!/bin/bash
# One call for several round-4 checks (the pool's queue is long): attention
# tests + A/B with timing, assembly NT weight-gradient tests + forms, counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
P=${1:-r4_batch}
TESTS=1 VARIANTS=split,ds bash scripts/gpu_r4_attn.sh "$P/attn" || exit $?
bash scripts/gpu_r4_wgrad.sh "$P/wgrad" || exit $?
tail -8 "gpurun_out/$P/wgrad/wgrad.log"
if [ "${PMC:-1}" = 1 ]; then
  bash scripts/gpu_r4_pmc.sh "$P/pmc" || exit $?
fi
