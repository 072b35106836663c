#!/bin/bash
# GPU suite without the full-size tests, then the full-size parity at configs 2 and 3 with the fp32 oracle
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=gpurun_out/r04d
mkdir -p $O
rm -f gpurun_out/parity.jsonl
timeout -k 10 500 python -u -m pytest tests -m gpu --deselect tests/test_gpu_fullsize.py -v --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
cp gpurun_out/parity.jsonl $O/parity_model.jsonl 2>/dev/null
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash tools/r04_parity.sh r04d "2 3"
