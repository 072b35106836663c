#!/bin/bash
# Round-6 end-of-round measurement on the GPU box, in three gpurun calls (each under the 1200 s limit):
#   tools/final_r06.sh TAG tests      the GPU test suite (parity log -> gpurun_out/TAG/parity.jsonl)
#   tools/final_r06.sh TAG countersA  PMC + SQ counters of configs 2 and 3 (tools/counters_cfg.sh)
#   tools/final_r06.sh TAG countersB  configs 4 and 5, the rocprofv3 kernel trace / stats of the default bench
#                                     (its event window: tools/prof_window.py; its gaps: tools/gap_window.py),
#                                     then the default bench line, which finds every config's counters of
#                                     its own tree in profiles/ (copy countersA's files there first)
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=$1; WHAT=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
TREE=$(python -c "import bench; print(bench.tree_hash())")
echo "tree $TREE"
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
case "$WHAT" in
  tests)
    rm -f "$R/gpurun_out/parity.jsonl"
    step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread || exit 1
    cp "$R/gpurun_out/parity.jsonl" "$O/parity.jsonl" ;;
  countersA)
    step c2 500 bash tools/counters_cfg.sh "$TAG" 2 || exit 1
    step c3 500 bash tools/counters_cfg.sh "$TAG" 3 || exit 1 ;;
  countersB)
    step c4 500 bash tools/counters_cfg.sh "$TAG" 4 || exit 1
    step c5 300 bash tools/counters_cfg.sh "$TAG" 5 || exit 1
    cd /tmp && export TMPDIR=/tmp
    step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o bench -- \
      python "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-extras || exit 1
    cd "$R"
    { echo "tree $TREE"; python tools/prof_summary.py "$O/prof/bench_kernel_stats.csv" 22; } > "$O/prof_summary.txt"
    python tools/prof_window.py "$O/prof/bench_kernel_trace.csv" 3 --json "$O/prof_window.json" > "$O/prof_window.txt"
    python tools/gap_window.py "$O/prof/bench_kernel_trace.csv" --steps 12 --skip 3 --json "$O/gaps.json" > "$O/gaps.txt"
    grep '^{' "$O/prof.log" | tail -1 > "$O/prof_bench_line.json"
    rm -f "$O"/prof/*kernel_trace.csv "$O"/prof/*.db
    step bench 600 python bench.py || exit 1
    grep '^{' "$O/bench.log" | tail -1 > "$O/bench_line.json"
    python -c "import json; d = json.load(open('$O/bench_line.json')); print(d['value'], d['ms_per_step'], d['tree'], d['traffic_tree_match'], d['roofline']['frac'], d['roofline']['frac_pmc'])" ;;
esac
echo "all done"
