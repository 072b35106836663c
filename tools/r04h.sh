#!/bin/bash
# GPU suite without the full-size tests, full-size parity at config 2, then the measurement pass
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
TAG=${1:-r04h}
O=gpurun_out/$TAG
mkdir -p $O
rm -f gpurun_out/parity.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu --deselect tests/test_gpu_fullsize.py -x -v --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest "tests/test_gpu_fullsize.py::test_training_step_at_baseline_size[2]" -x -v \
  --timeout 380 --timeout-method thread > $O/fullsize2.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/fullsize2.log | tail -3
[ $rc -eq 0 ] || exit $rc
cp gpurun_out/parity.jsonl $O/parity.jsonl
bash tools/final_pass.sh $TAG measure
