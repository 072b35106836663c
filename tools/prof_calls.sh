#!/bin/bash
# Per-dispatch durations (us) of the kernels matching a pattern, in launch order, over the last timed
# step of a short config-2 bench under rocprofv3 (GPU box):  tools/prof_calls.sh TAG PATTERN
set -o pipefail
TAG=$1; PAT=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/t" -o b -- \
  python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras > "$O/t.log" 2>&1 || { tail -5 "$O/t.log"; exit 1; }
rm -f "$O"/t/*.db
python - "$O/t/b_kernel_trace.csv" "$PAT" <<'PY'
import csv, re, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
hits = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows
        if re.search(sys.argv[2], r["Kernel_Name"])]
for name, us in hits[-40:]:
    print(f"{name[:60]:60s} {us:8.1f} us")
PY
rm -f "$O"/t/b_kernel_trace.csv
