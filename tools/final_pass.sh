#!/bin/bash
# End-of-round measurement pass on the GPU box, in two gpurun calls (each under the 1200 s limit):
#   tools/final_pass.sh TAG tests     GPU test suite (the full-size parity log lands in gpurun_out/parity.jsonl)
#   tools/final_pass.sh TAG measure   rocprofv3 kernel stats, the two PMC passes (FETCH_SIZE, WRITE_SIZE), then
#                                     the default bench line, which finds the PMC traffic of the same tree
#                                     (the PMC summary is copied to profiles/${ROUND:-r05}_pmc_traffic.json first)
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=$1
WHAT=$2
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
TREE=$(python -c "import bench; print(bench.tree_hash())")
echo "tree $TREE"
if [ "$WHAT" = tests ]; then
  rm -f "$R/gpurun_out/parity.jsonl"
  step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout 1000 --timeout-method thread || exit 1
  cp "$R/gpurun_out/parity.jsonl" "$O/parity.jsonl"
fi
if [ "$WHAT" = measure ]; then
  cd /tmp && export TMPDIR=/tmp
  step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o bench -- \
    python "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-extras || exit 1
  step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o bench -- \
    python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras || exit 1
  step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o bench -- \
    python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras || exit 1
  cd "$R"
  { echo "tree $TREE"; python tools/prof_summary.py "$O/prof/bench_kernel_stats.csv" 22; } > "$O/prof_summary.txt"
  python tools/pmc_summary.py "$O/pmc_fetch/bench_counter_collection.csv" \
    "$O/pmc_write/bench_counter_collection.csv" --json "$O/pmc_traffic.json" --tree "$TREE" > "$O/pmc_traffic.txt"
  # the bench's event window (its last 3 timed steps) in the same profiled process, beside its own line
  python tools/prof_window.py "$O/prof/bench_kernel_trace.csv" 3 --json "$O/prof_window.json" > "$O/prof_window.txt"
  grep '^{' "$O/prof.log" | tail -1 > "$O/prof_bench_line.json"
  rm -f "$O"/prof/*kernel_trace.csv "$O"/*/*.db
  cp "$O/pmc_traffic.json" "$R/profiles/${ROUND:-r05}_pmc_traffic.json"
  # SQ counters of the same tree (MFMA busy, wave-cycle split), two passes with kernel traces, before the
  # bench line so that it carries the counter MFMA busy beside its flop-derived frac_mfma
  bash tools/sq_pass.sh "$TAG/sq" > "$O/sq_pass.log" 2>&1 || { tail -5 "$O/sq_pass.log"; exit 1; }
  cp "$R/gpurun_out/$TAG/sq/sq.txt" "$R/profiles/${ROUND:-r05}_sq.txt"
  cp "$R/gpurun_out/$TAG/sq/sq.json" "$R/profiles/${ROUND:-r05}_sq.json"
  step bench 500 python bench.py || exit 1
  grep '^{' "$O/bench.log" | tail -1 > "$O/bench_line.json"
  python -c "import json; d = json.load(open('$O/bench_line.json')); print(d['value'], d['ms_per_step'], d['tree'], d['traffic_tree_match'], d['roofline'])"
fi
echo "all done"
