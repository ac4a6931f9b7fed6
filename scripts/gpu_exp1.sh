#!/bin/bash
# perf experiments: micro-batch, TunableOp GEMM tuning
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/exp1
export TMPDIR=/tmp
O=gpurun_out/exp1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --micro-batch 6 > $O/mb6.log 2>&1; echo "rc=$?" >> $O/mb6.log
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=40 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=10
timeout -k 10 600 python bench.py --steps 3 --warmup 2 --micro-batch 4 > $O/tune.log 2>&1; echo "rc=$?" >> $O/tune.log
export PYTORCH_TUNABLEOP_TUNING=0
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --micro-batch 4 > $O/tuned.log 2>&1; echo "rc=$?" >> $O/tuned.log
ls -la $O
exit 0
