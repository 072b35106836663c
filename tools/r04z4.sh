#!/bin/bash
# inference (config 5): message sums inside the edge forward (seg_sums, default) vs the deferred +
# XCD-interleaved edge forward with pdg_segment_sum, same box, three pairs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04z4
mkdir -p "$O"
cd "$R" || exit 1
for rep in 1 2 3; do
  for e in "PDG_SEG_SUMS=1" "PDG_SEG_SUMS=0"; do
    env PDG_AB=1 $e timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline --no-extras > "$O/x.log" 2>&1 \
      || { echo "$e failed"; tail -5 "$O/x.log"; exit 1; }
    python -c "
import json
d=json.loads([l for l in open('$O/x.log') if l.startswith('{')][-1])
print('%-16s %10.0f nodes/s %8.3f ms  '%('$e',d['value'],d['ms_per_step'])+' '.join('%s=%.4f'%(k,v) for k,v in d['kernel_ms'].items()))"
  done
done
