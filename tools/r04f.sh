#!/bin/bash
# model + op tests of the tree, then the measurement pass (tools/final_pass.sh TAG measure)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
TAG=${1:-r04f}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ops.py -x -v --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
bash tools/final_pass.sh $TAG measure
