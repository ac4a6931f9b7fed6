#!/bin/bash
# One GPU pass: GPU tests, graft smoke, payload examples, flagship bench, rocprof stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/round; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name" >&2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc=$rc" >> $O/$name.log
  echo "$name rc=$rc" >&2; return $rc; }
step pytest_gpu 600 python -m pytest tests -m gpu -q -x &&
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
step ex_smoke 120 python -m tf_operator_amd.examples.smoke &&
step ex_mnist 300 python -m tf_operator_amd.examples.dist_mnist --train_steps 500 &&
step ex_summaries 300 python -m tf_operator_amd.examples.mnist_with_summaries &&
step ex_resnet 300 python -m tf_operator_amd.examples.resnet_train --steps 20 --warmup 5 --batch 256 &&
step bench 600 python bench.py &&
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1
rc=$?
find $O/prof -name '*kernel_trace.csv' -size +30M -delete 2>/dev/null
exit $rc
