set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r5s2_arms; mkdir -p $O
timeout -k 10 300 python scripts/attn_dkdv_arms.py --rounds 5 > $O/arms.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/attn_bwd_ab.py --variants dship+ds --rounds 2 --reps 2 > $O/prof.log 2>&1
echo rc=$?
