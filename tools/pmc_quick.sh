#!/bin/bash
# One rocprofv3 PMC pass over a short bench run (GPU box): tools/pmc_quick.sh TAG "COUNTERS..." [bench args]
set -o pipefail
TAG=$1; CNT=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc $CNT --output-format csv -d "$O/p" -o bench -- \
  python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras "$@" > "$O/log" 2>&1 || { tail -5 "$O/log"; exit 1; }
cd "$R"
python tools/pmc_sq.py "$O/p/bench_counter_collection.csv" 16 > "$O/summary.txt"
rm -f "$O"/p/*.db
cat "$O/summary.txt"
