#!/bin/bash
# profiling launcher + FULL_TRACE analog on the GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/proflaunch; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -m tf_operator_amd.utils.profiling --mode stats --out $O/mnist -- python3 -m tf_operator_amd.examples.dist_mnist --train_steps 2000 --log_every 1000 > $O/launcher.log 2>&1 &&
timeout -k 10 300 python -m tf_operator_amd.examples.mnist_with_summaries --max_steps 200 --log_dir $O/mws > $O/mws.log 2>&1
rc=$?
ls -la $O/mws/train >> $O/mws.log 2>&1
find $O -name '*kernel_trace.csv' -delete
exit $rc
