#!/bin/bash
# rocprofv3 kernel stats of the config-2 bench per library variant (GPU box), printed side by side
# for the kernels matching a pattern:  tools/prof_variants.sh TAG PATTERN v1 v2 ...  ("default" = shipped)
set -o pipefail
TAG=$1; PAT=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then lib=$R/p-div-gnn_amd/pdg/libpdivgnn_hip.so; else lib=$R/variants/$v/libpdivgnn_hip.so; fi
  PDG_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$v" -o b -- \
    python "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-extras > "$O/$v.log" 2>&1 \
    || { echo "$v failed"; tail -5 "$O/$v.log"; exit 1; }
  rm -f "$O/$v"/*.db
  python - "$O/$v/b_kernel_stats.csv" "$v" "$PAT" <<'PY'
import csv, re, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{sys.argv[2]}: total {tot / 7 / 1e6:.3f} ms/step (7 steps incl. warmup)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if re.search(sys.argv[3], r["Name"]):
        print(f"{sys.argv[2]}:   {r['Name'][:50]:50s} calls {int(r['Calls']):5d}  avg {float(r['AverageNs']) / 1e3:8.1f} us")
PY
done
