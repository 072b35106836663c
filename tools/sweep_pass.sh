#!/bin/bash
# The published-workload sweep on the GPU box: its parity test, the sweep line (bench.py --sweep-only) and
# a rocprofv3 kernel trace of the same sweep (kernel sum per forward beside the wall times).
#   tools/sweep_pass.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_published.py -x -v -s --timeout 240 --timeout-method thread \
  > "$O/pytest_published.log" 2>&1 || { tail -30 "$O/pytest_published.log"; exit 1; }
tail -3 "$O/pytest_published.log"
timeout -k 10 300 python bench.py --sweep-only > "$O/sweep.log" 2>&1 || { tail -20 "$O/sweep.log"; exit 1; }
grep '^{' "$O/sweep.log" | tail -1 > "$O/sweep_line.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o sweep -- \
  python "$R/bench.py" --sweep-only > "$O/sweep_prof.log" 2>&1 || { tail -20 "$O/sweep_prof.log"; exit 1; }
cd "$R"
python tools/sweep_trace.py "$O/prof/sweep_kernel_trace.csv" "$O/sweep_line.json" > "$O/sweep_trace.txt"
rm -f "$O"/prof/*.db
cat "$O/sweep_trace.txt"
echo "all done"
