#!/bin/bash
# Submit -> first-step latency on one MI355X, cold process starts vs the
# local kubelet's warm fork server (benchmarks/submit_latency.py --warm).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/warm
run() {  # label seconds args...
  timeout -k 10 "$2" python -u benchmarks/submit_latency.py "${@:3}" > "gpurun_out/warm/$1.json" 2> "gpurun_out/warm/$1.log"
}
timeout -k 10 300 python -u -m pytest tests/test_forkserver.py -x -v --timeout 150 --timeout-method thread > gpurun_out/warm/pytest.log 2>&1 &&
run mnist_cold 300 --payload mnist --repeats 5 &&
run mnist_warm 300 --payload mnist --repeats 5 --warm &&
run llama_cold 420 --payload llama --repeats 3 &&
run llama_warm 420 --payload llama --repeats 3 --warm
rc=$?
tail -3 gpurun_out/warm/pytest.log
cat gpurun_out/warm/*.json
exit $rc
