#!/bin/bash
# A/B of engine env flags: tools-style, run on the GPU box.  usage: ab_env.sh TAG "ENV1" "ENV2" ...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/$TAG"
for rep in 1 2; do
for e in "$@"; do
  env PDG_AB=1 $e timeout -k 10 300 python "$R/bench.py" --no-cpu-baseline --no-extras --steps 30 > "$R/gpurun_out/$TAG/x.log" 2>&1 || { echo "$e failed"; tail -5 "$R/gpurun_out/$TAG/x.log"; exit 1; }
  python -c "
import json,sys
d=json.loads([l for l in open('$R/gpurun_out/$TAG/x.log') if l.startswith('{')][-1])
print('%-28s %10.0f nodes/s %8.3f ms  '%('$e',d['value'],d['ms_per_step'])+' '.join('%s=%.4f'%(k,v) for k,v in d['kernel_ms'].items()))"
done; done
