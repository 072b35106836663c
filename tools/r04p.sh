#!/bin/bash
# gz1e from gC - gz1m: op / model tests, then a same-box A/B of the step
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/r04p"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_model.py \
  -k "pq_scatter or gz1e or fused_edge or golden" > "$R/gpurun_out/r04p/t.log" 2>&1 || { tail -30 "$R/gpurun_out/r04p/t.log"; exit 1; }
tail -3 "$R/gpurun_out/r04p/t.log"
bash "$R/tools/ab_env.sh" r04p "PDG_GZ1E_FROM_GC=1" "PDG_GZ1E_FROM_GC=0"
