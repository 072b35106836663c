#!/bin/bash
# Measurement pass on the GPU box (run through gpurun from the repo root):
#   GPU parity tests, the default bench line (config 2 + config 3/4/5 sub-results), rocprofv3 kernel stats and
#   the two PMC passes (FETCH_SIZE, WRITE_SIZE) of the default bench command.
# Every GPU step has its own time limit; the script stops at the first failure.
#   usage: tools/gpu_measure.sh TAG [all|tests|bench|prof]
set -o pipefail
TAG=${1:-run}
WHAT=${2:-all}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -3 "$O/$name.log"
  return $rc
}
cd "$R" || exit 1
if [ "$WHAT" = all ] || [ "$WHAT" = tests ]; then
  step pytest_gpu 1150 python -u -m pytest tests -m gpu -x -v --timeout 1100 --timeout-method thread || exit 1
fi
if [ "$WHAT" = all ] || [ "$WHAT" = bench ]; then
  step bench2 600 python bench.py || exit 1
fi
if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
  cd /tmp && export TMPDIR=/tmp
  step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o bench -- \
    python "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-extras || exit 1
  step pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o bench -- \
    python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras || exit 1
  step pmc_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o bench -- \
    python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras || exit 1
fi
if [ "$WHAT" = all ] || [ "$WHAT" = prof ]; then
  cd "$R"
  TREE=$(python -c "import bench; print(bench.tree_hash())")
  { echo "tree $TREE"; python tools/prof_summary.py "$O/prof/bench_kernel_stats.csv" 22; } > "$O/prof_summary.txt"
  python tools/pmc_summary.py "$O/pmc_fetch/bench_counter_collection.csv" \
    "$O/pmc_write/bench_counter_collection.csv" --json "$O/pmc_traffic.json" --tree "$TREE" > "$O/pmc_traffic.txt"
  rm -f "$O"/prof/*kernel_trace.csv "$O"/*/*.db
  cat "$O/prof_summary.txt" "$O/pmc_traffic.txt"
fi
echo "all done"
