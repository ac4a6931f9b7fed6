#!/bin/bash
# Round-3 kernel validation + A/B on one MI355X (run through gpurun):
# new-kernel GPU tests, attention-backward A/B, TN GEMM vs hipBLASLt, and the
# world-8 overlap emulation at 10 steps.  A step that fails its checks does
# not stop the benchmarks; a fault, abort or time limit ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${1:-r3_kernels}; mkdir -p "$O"
export TMPDIR=/tmp
step() {  # step <name> <seconds> cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$O/$n.log" 2>&1
  local rc=$?
  echo "$n rc=$rc"
  case $rc in 0|1|2) return 0 ;; *) echo "stopping after $n (rc=$rc)"; exit $rc ;; esac
}
step tests 600 python -u -m pytest tests/test_ops_gpu.py tests/test_comm_gpu.py -x -v --timeout 180 \
  --timeout-method thread -k "flash_attention or gemm_tn or fused_mlp or operator_env or momentum_none"
step attn_bwd_ab 300 python scripts/attn_bwd_ab.py
step gemm_tn_bench 600 python scripts/gemm_tn_bench.py
step overlap 600 python scripts/overlap_emulation.py --out "$O/overlap" --steps 10 --warmup 2
