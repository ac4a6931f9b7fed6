#!/bin/bash
# Same-box A/B of bench.py --direct under two environments, alternating runs:
#   scripts/gpu_ab_env.sh <out> <rounds> "<env A>" "<env B>" [bench args...]
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; R=$2; A=$3; B=$4; shift 4
mkdir -p "$O"
export TMPDIR=/tmp
for i in $(seq 1 "$R"); do
  for arm in A B; do
    if [ $arm = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python bench.py --direct "$@" > "$O/${arm}_$i.out" 2> "$O/${arm}_$i.err" || exit $?
    echo "$arm $i [$E]: $(grep '^{' "$O/${arm}_$i.out" | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
