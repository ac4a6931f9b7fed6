#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lat2; mkdir -p $O
timeout -k 10 900 python benchmarks/submit_latency.py --workers 1 --payload llama --model llama3-8b --repeats 4 > $O/lat_llama.log 2>&1 || exit $?
timeout -k 10 300 python benchmarks/submit_latency.py --workers 1 --payload mnist --repeats 5 > $O/lat_mnist.log 2>&1
