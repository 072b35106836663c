#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 120 tools/membench2 > $O/membench2.jsonl 2>&1 || { tail -5 $O/membench2.jsonl; exit 1; }
cat $O/membench2.jsonl
timeout -k 10 300 python tools/grad_err_golden.py batch2_div_s10 > $O/grad_err.txt 2>&1 || { tail -5 $O/grad_err.txt; exit 1; }
cat $O/grad_err.txt
PDG_LIB=variants/unb/libpdivgnn_hip.so timeout -k 10 300 python tools/grad_err_golden.py batch2_div_s10 > $O/grad_err_unb.txt 2>&1 || { tail -5 $O/grad_err_unb.txt; exit 1; }
cat $O/grad_err_unb.txt
PDG_LIB=variants/x6c/libpdivgnn_hip.so timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py -k "node_net or node_pq" \
  -q --timeout 150 --timeout-method thread > $O/x6c_ops.log 2>&1; tail -3 $O/x6c_ops.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -v --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/ab.sh r04c 2 default old unb x6c unbc default old unb x6c unbc
