#!/bin/bash
# PMC traffic and SQ counters of one bench config on the GPU box (counters for every
# config, not only the main line's):   tools/counters_cfg.sh TAG CONFIG [ROUND]
# Four rocprofv3 passes over `bench.py --config C --steps 2 --warmup 1 --no-extras`, each its own run
# and time limit (FETCH_SIZE; WRITE_SIZE; SQ pass A; SQ pass B), then
#   profiles/${ROUND}_pmc_traffic_cC.json / .txt   (2*FETCH_SIZE + WRITE_SIZE per dispatch, tree in _meta)
#   profiles/${ROUND}_sq_cC.json / .txt            (MFMA busy, wave-cycle split)
# Config 2 writes the unsuffixed names bench.py's main line reads.
set -o pipefail
TAG=$1; C=$2; ROUND=${3:-r06}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG/c$C
mkdir -p "$O"
cd "$R" || exit 1
TREE=$(python -c "import bench; print(bench.tree_hash())")
SUF=$([ "$C" = 2 ] && echo "" || echo "_c$C")
ARGS="--config $C --steps 2 --warmup 1 --no-cpu-baseline --no-extras"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o b -- \
  python "$R/bench.py" $ARGS > "$O/pmc_fetch.log" 2>&1 || { echo "FETCH pass failed"; tail -5 "$O/pmc_fetch.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o b -- \
  python "$R/bench.py" $ARGS > "$O/pmc_write.log" 2>&1 || { echo "WRITE pass failed"; tail -5 "$O/pmc_write.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d "$O/sqA" -o b -- python "$R/bench.py" $ARGS > "$O/sqA.log" 2>&1 \
  || { echo "SQ pass A failed"; tail -5 "$O/sqA.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES \
  --kernel-trace --output-format csv -d "$O/sqB" -o b -- python "$R/bench.py" $ARGS > "$O/sqB.log" 2>&1 \
  || { echo "SQ pass B failed"; tail -5 "$O/sqB.log"; exit 1; }
cd "$R"
rm -f "$O"/*/*.db "$O"/*/*/*.db
python tools/pmc_summary.py "$O/pmc_fetch/b_counter_collection.csv" "$O/pmc_write/b_counter_collection.csv" \
  --json "$O/pmc_traffic.json" --tree "$TREE" > "$O/pmc_traffic.txt"
python tools/sq_summary.py "$O/sqA" "$O/sqB" --tree "$TREE" --json "$O/sq.json" > "$O/sq.txt"
cp "$O/pmc_traffic.json" "$R/profiles/${ROUND}_pmc_traffic${SUF}.json"
cp "$O/pmc_traffic.txt" "$R/profiles/${ROUND}_pmc_traffic${SUF}.txt"
cp "$O/sq.json" "$R/profiles/${ROUND}_sq${SUF}.json"
cp "$O/sq.txt" "$R/profiles/${ROUND}_sq${SUF}.txt"
echo "config $C tree $TREE"; head -12 "$O/sq.txt"
