#!/bin/bash
# round-4 GPU pass b: gather probes, the GPU suite without the full-size tests (margins logged), SQ counters
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 120 tools/membench2 > $O/membench2.jsonl 2>&1 || { tail -5 $O/membench2.jsonl; exit 1; }
cat $O/membench2.jsonl
rm -f gpurun_out/parity.jsonl
timeout -k 10 700 python -u -m pytest tests -m gpu --deselect tests/test_gpu_fullsize.py -v --timeout 400 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
cp gpurun_out/parity.jsonl $O/parity_model.jsonl 2>/dev/null
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/sq_pass.sh r04b
