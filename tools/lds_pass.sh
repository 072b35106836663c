#!/bin/bash
# One rocprofv3 LDS counter pass (bank-conflict cycles over all LDS cycles, per kernel) over a short bench
# run on the GPU box:  tools/lds_pass.sh TAG
set -o pipefail
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS \
  --kernel-trace --output-format csv -d "$O/lds" -o b -- \
  python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras > "$O/lds.log" 2>&1 \
  || { echo "LDS pass failed"; tail -5 "$O/lds.log"; exit 1; }
cd "$R"
rm -f "$O"/lds/*.db
python - "$O/lds/b_counter_collection.csv" > "$O/lds.txt" <<'PY'
import csv, sys
from collections import defaultdict
tot = defaultdict(lambda: defaultdict(float)); disp = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:60]
    tot[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
print(f"{'kernel':60s} {'disp':>5s} {'conflict/active':>15s} {'unaligned/active':>16s} {'LDS insts/disp':>15s}")
rows = []
for k, c in tot.items():
    act = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
    if act <= 0:
        continue
    rows.append((act / len(disp[k]), k, len(disp[k]), c.get("SQ_LDS_BANK_CONFLICT", 0) / act,
                 c.get("SQ_LDS_UNALIGNED_STALL", 0) / act, c.get("SQ_INSTS_LDS", 0) / len(disp[k])))
for act, k, n, bc, un, ins in sorted(rows, reverse=True)[:20]:
    print(f"{k:60s} {n:5d} {bc:15.3f} {un:16.3f} {ins:15.0f}")
PY
cat "$O/lds.txt"
