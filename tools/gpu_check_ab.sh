#!/bin/bash
# GPU box: op + model tests (-k filter), then a config-2 A/B of the baseline tree against this one
#   tools/gpu_check_ab.sh TAG "PYTEST_K" [env assignments for the second variant run ...]
set -o pipefail
TAG=$1; K=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/$TAG"
cd "$R" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ops.py \
  tests/test_gpu_model.py tests/test_gpu_custom_ops.py -k "$K" > "$R/gpurun_out/$TAG/tests.log" 2>&1 \
  || { tail -30 "$R/gpurun_out/$TAG/tests.log"; exit 1; }
tail -1 "$R/gpurun_out/$TAG/tests.log"
bash tools/ab.sh "$TAG" 2 basetree default basetree default
