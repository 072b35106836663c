#!/bin/bash
# Two rocprofv3 SQ counter passes (each with --kernel-trace for the durations) over a short bench run
# on the GPU box, summarised per kernel by tools/sq_summary.py:  tools/sq_pass.sh TAG [bench args]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
TREE=$(python -c "import bench; print(bench.tree_hash())")
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d "$O/sqA" -o b -- \
  python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras "$@" > "$O/sqA.log" 2>&1 \
  || { echo "pass A failed"; tail -5 "$O/sqA.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  --kernel-trace --output-format csv -d "$O/sqB" -o b -- \
  python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras "$@" > "$O/sqB.log" 2>&1 \
  || { echo "pass B failed"; tail -5 "$O/sqB.log"; exit 1; }
cd "$R"
rm -f "$O"/sq?/*.db "$O"/sq?/*/*.db
python tools/sq_summary.py "$O/sqA" "$O/sqB" --tree "$TREE" --json "$O/sq.json" > "$O/sq.txt"
cat "$O/sq.txt"
