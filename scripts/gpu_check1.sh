#!/bin/bash
# first GPU check: kernel numerics, tiny smoke, bench (1B then 8B), rocprof stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showmeminfo vram > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py -q > gpurun_out/pytest_ops.log 2>&1; echo "pytest rc=$?" | tee -a gpurun_out/pytest_ops.log
timeout -k 10 200 python __graft_entry__.py > gpurun_out/build.log 2>&1 || true
timeout -k 10 300 python bench.py --model llama3-1b --steps 3 --warmup 2 --micro-batch 4 > gpurun_out/bench_1b.log 2>&1; echo "bench1b rc=$?" >> gpurun_out/bench_1b.log
timeout -k 10 500 python bench.py --steps 4 --warmup 2 > gpurun_out/bench_8b.log 2>&1; rc=$?; echo "bench8b rc=$rc" >> gpurun_out/bench_8b.log
exit 0
