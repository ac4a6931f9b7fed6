#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lat; mkdir -p $O
timeout -k 10 300 python scripts/gemm_bench.py 16384 cublaslt cublas > $O/gemm.log 2>&1; echo "rc=$?" >> $O/gemm.log
timeout -k 10 600 python benchmarks/submit_latency.py --workers 1 --payload llama --model llama3-8b --repeats 3 > $O/lat_llama.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/submit_latency.py --workers 1 --payload mnist --repeats 5 > $O/lat_mnist.log 2>&1
