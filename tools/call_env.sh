#!/bin/bash
# One GPU call: GPU tests (optional -k filter), bitwise gradient check of engine variant settings
# against the defaults, and a config-2 timing A/B of them.
#   tools/call_env.sh TAG "PYTEST_K|-" "ENV=VAL ..." ...
set -o pipefail
TAG=$1; K=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
if [ "$K" != "-" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" \
    > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
  tail -1 "$O/tests.log"
fi
timeout -k 10 120 python tools/grads_dump.py "$O/g_default.pt" || exit 1
i=0
for e in "$@"; do
  i=$((i + 1))
  env PDG_AB=1 $e timeout -k 10 120 python tools/grads_dump.py "$O/g_$i.pt" || exit 1
  echo "[$e]"; python tools/grads_dump.py --compare "$O/g_$i.pt" "$O/g_default.pt" | tail -3
done
bash tools/ab_env.sh "$TAG" "PDG_NONE=1" "$@"
