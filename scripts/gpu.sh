#!/bin/bash
# One parametrised GPU-box runner (used through gpurun):
#
#   scripts/gpu.sh <out-name> <step> [<step> ...]
#
# Each step runs under its own time limit; the first failing step ends the
# call (no retries).  Logs land in gpurun_out/<out-name>/<step>.log.
#
# steps:
#   tests            pytest -m gpu (one process, per-test timeout)
#   tests:<expr>     pytest -m gpu -k <expr>
#   smoke            __graft_entry__.smoke()
#   bench            python bench.py (through the operator, N=1, driver defaults)
#   bench:<args>     python bench.py <args, comma separated>
#   direct:<args>    python bench.py --direct <args> (no operator)
#   prof             rocprofv3 --kernel-trace --stats of bench.py --direct (2 timed steps)
#   pmc:<script>:<counters>  rocprofv3 --pmc <counters> --kernel-trace of python3 <script>
#   py:<module>:<args>       python -m <module> <args, comma separated>
#   examples         the bundled payloads (smoke, mnist, summaries, resnet)
#   resnet           the ResNet-50 payload twice (fresh box: MIOpen find-db path), batch 256
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
NAME=${1:?out name}; shift
O=gpurun_out/$NAME; mkdir -p "$O"
export TMPDIR=/tmp

run() {  # run <log> <seconds> cmd...
  local log=$1 t=$2; shift 2
  echo "== $log: $*" >&2
  timeout -k 10 "$t" "$@" > "$O/$log.log" 2>&1
  local rc=$?
  echo "rc=$rc" >> "$O/$log.log"
  echo "$log rc=$rc" >&2
  tail -n 3 "$O/$log.log" >&2
  return $rc
}

for st in "$@"; do
  case "$st" in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $? ;;
    tests:*) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${st#tests:}" || exit $? ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench) run bench 900 python bench.py || exit $? ;;
    bench:*) IFS=, read -ra A <<< "${st#bench:}"; run bench 1100 python bench.py "${A[@]}" || exit $? ;;
    direct:*) IFS=, read -ra A <<< "${st#direct:}"; run direct 900 python bench.py --direct "${A[@]}" || exit $? ;;
    prof)
      run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
        python3 bench.py --direct --steps 2 --warmup 1 || exit $?
      find "$O/prof" -name '*kernel_trace.csv' -size +30M -delete ;;
    pmc:*)
      rest=${st#pmc:}; script=${rest%%:*}; ctrs=${rest#*:}
      run "pmc_$(basename "$script" .py)" 300 rocprofv3 --pmc ${ctrs//,/ } --kernel-trace --output-format csv \
        -d "$O/pmc" -o run -- python3 "$script" || exit $? ;;
    py:*)
      rest=${st#py:}; mod=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
      IFS=, read -ra A <<< "$args"
      run "py_${mod##*.}" 900 python -m "$mod" "${A[@]}" || exit $? ;;
    examples)
      run ex_smoke 120 python -m tf_operator_amd.examples.smoke &&
      run ex_mnist 300 python -m tf_operator_amd.examples.dist_mnist --train_steps 500 &&
      run ex_summaries 300 python -m tf_operator_amd.examples.mnist_with_summaries &&
      run ex_resnet 300 python -m tf_operator_amd.examples.resnet_train --steps 20 --warmup 5 --batch 256 || exit $? ;;
    resnet)
      run resnet1 300 python -m tf_operator_amd.examples.resnet_train --steps 40 --warmup 8 --batch 256 &&
      run resnet2 300 python -m tf_operator_amd.examples.resnet_train --steps 40 --warmup 8 --batch 256 || exit $? ;;
    *) echo "unknown step $st" >&2; exit 2 ;;
  esac
done
