#!/bin/bash
# rocprofv3 kernel stats of the default config-2 bench for the shipped library and library variants
# (GPU box):  tools/prof_ab.sh TAG KERNEL_REGEX variant...
set -o pipefail
TAG=$1; PAT=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in default "$@"; do
  if [ "$v" = default ]; then lib=$R/p-div-gnn_amd/pdg/libpdivgnn_hip.so; else lib=$R/variants/$v/libpdivgnn_hip.so; fi
  PDG_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$v" -o b -- \
    python "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-extras > "$O/$v.log" 2>&1 || { tail -5 "$O/$v.log"; exit 1; }
  rm -f "$O/$v"/*.db "$O/$v"/*kernel_trace.csv
  echo "== $v"
  (cd "$R" && python tools/prof_summary.py "$O/$v/b_kernel_stats.csv" 22 | grep -E "$PAT|total")
done
