#!/bin/bash
# One GPU call: GPU tests (optional -k filter), the default bench line, bitwise gradient check and
# config-2 A/B of library variants.   tools/call_ab.sh TAG "PYTEST_K|-" variant...
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
timeout -k 10 300 python bench.py --no-cpu-baseline > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
python - "$O/bench.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("bench", d["value"], d["ms_per_step"], "tree", d["tree"])
print({k: round(v, 4) for k, v in d["kernel_ms"].items()})
PY
timeout -k 10 120 python tools/grads_dump.py "$O/g_default.pt" || exit 1
for v in "$@"; do
  PDG_LIB=$R/variants/$v/libpdivgnn_hip.so timeout -k 10 120 python tools/grads_dump.py "$O/g_$v.pt" || exit 1
  python tools/grads_dump.py --compare "$O/g_$v.pt" "$O/g_default.pt" | tail -3
done
bash tools/ab.sh "$TAG" 2 default "$@" default "$@"
