#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abprof; mkdir -p $O
export TMPDIR=/tmp
export TOA_GEMM=torch
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/torch -o run -- python3 bench.py --steps 2 --warmup 1 > $O/torch.log 2>&1 || exit $?
export TOA_GEMM=auto
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tuned -o run -- python3 bench.py --steps 2 --warmup 1 > $O/tuned.log 2>&1
rm -f $O/*/run_kernel_trace.csv
