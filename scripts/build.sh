#!/bin/bash
# Build everything (gfx950 HIP library + C++ core), regenerate the CRDs, run the CPU test tiers.
#   scripts/build.sh            build + CRDs + CPU tests
#   scripts/build.sh --no-test  build + CRDs
#   scripts/build.sh --images   also docker build the operator / trainer images
set -euo pipefail
cd "$(dirname "$0")/.."
python -m tf_operator_amd._build
python -m tf_operator_amd.api.schema --out manifests/base
if [[ " $* " != *" --no-test "* ]]; then
  python -m pytest tests -q -m "not gpu"
fi
if [[ " $* " == *" --images "* ]]; then
  docker build -f docker/operator.Dockerfile -t tf-operator-amd/training-operator:v0.1.0 .
  docker build -f docker/trainer.Dockerfile -t tf-operator-amd/trainer:v0.1.0 .
fi
