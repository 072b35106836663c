#!/bin/bash
# column-sum tail: op test, then same-box A/B of the tail against the separate ln_colsum_nodes launch
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "node_bwd_coop or mlp2_bwd_coop or decoder_bwd_coop" -x -v \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -4
[ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh r04j "PDG_COLSUM_TAIL=1" "PDG_COLSUM_TAIL=0"
