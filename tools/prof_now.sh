#!/bin/bash
# rocprofv3 kernel stats of the default config-2 bench on this tree (GPU box): tools/prof_now.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o b -- \
  python "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-extras > "$O/prof.log" 2>&1 || { tail -5 "$O/prof.log"; exit 1; }
rm -f "$O"/prof/*.db "$O"/prof/*kernel_trace.csv
cd "$R" && python tools/prof_summary.py "$O/prof/b_kernel_stats.csv" 22
