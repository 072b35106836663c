#!/bin/bash
# GPU check of the fused message sums: op + model tests, then config-2 and config-5 A/B (PDG_SEG_SUMS).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/seg
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ops.py \
  -k "seg_sums or coop or segment_sum" > "$O/ops.log" 2>&1 || { tail -30 "$O/ops.log"; exit 1; }
tail -2 "$O/ops.log"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_model.py \
  > "$O/model.log" 2>&1 || { tail -30 "$O/model.log"; exit 1; }
tail -2 "$O/model.log"
for c in 2 5; do
for e in PDG_SEG_SUMS_TRAIN=0 PDG_SEG_SUMS_TRAIN=1 PDG_SEG_SUMS=0 PDG_SEG_SUMS=1; do
  env PDG_AB=1 $e timeout -k 10 300 python "$R/bench.py" --no-cpu-baseline --no-extras --steps 30 --config $c > "$O/x.log" 2>&1 || { echo "$e failed"; tail -5 "$O/x.log"; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$O/x.log') if l.startswith('{')][-1])
print('cfg $c %-16s %10.0f nodes/s %8.3f ms  '%('$e',d['value'],d['ms_per_step'])+' '.join('%s=%.4f'%(k,v) for k,v in d['kernel_ms'].items()))"
done; done
