#!/bin/bash
# Full-size parity with the fp32 oracle forced on (PDG_PARITY_FP32=1): the reference fp32 CPU path's own
# distance to fp64 beside the GPU's, per gradient tensor, at the given BASELINE config(s).
#   tools/r04_parity.sh TAG "2 3"      (config 4 alone takes ~11 min of host CPU: run it in its own call)
set -o pipefail
TAG=$1; CFGS=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out/$TAG
IDS=$(for c in $CFGS; do printf "tests/test_gpu_fullsize.py::test_training_step_at_baseline_size[%s] " "$c"; done)
PDG_PARITY_FP32=1 PDG_PARITY_LOG=$R/gpurun_out/$TAG/parity.jsonl timeout -k 10 1120 python -u -m pytest \
  $IDS -x -v --timeout 1100 --timeout-method thread > gpurun_out/$TAG/parity.log 2>&1
rc=$?
tail -8 gpurun_out/$TAG/parity.log
python - "$R/gpurun_out/$TAG/parity.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d.get("config"), "pred", d.get("pred_vs_f64"), "worst", d.get("worst_grad"), "oracle_s", d.get("oracle_s"))
PY
exit $rc
