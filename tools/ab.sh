#!/bin/bash
# A/B timing of library variants (variants/<name>/libpdivgnn_hip.so) with bench.py.
#   usage: tools/ab.sh OUTTAG CONFIG name1 name2 ...   ("default" = the shipped library)
set -o pipefail
TAG=$1; CFG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/$TAG"
for v in "$@"; do
  # a variant is either a library (variants/<v>/libpdivgnn_hip.so, run by this tree's bench) or a
  # whole tree (variants/<v>/bench.py with its own in-tree library)
  benchpy=$R/bench.py
  if [ "$v" = default ]; then lib=$R/p-div-gnn_amd/pdg/libpdivgnn_hip.so
  elif [ -f "$R/variants/$v/bench.py" ]; then benchpy=$R/variants/$v/bench.py; lib=$R/variants/$v/p-div-gnn_amd/pdg/libpdivgnn_hip.so
  else lib=$R/variants/$v/libpdivgnn_hip.so; fi
  PDG_LIB=$lib timeout -k 10 300 python "$benchpy" --config "$CFG" --no-cpu-baseline --no-extras \
    > "$R/gpurun_out/$TAG/$v.c$CFG.log" 2>&1 || { echo "$v failed"; tail -5 "$R/gpurun_out/$TAG/$v.c$CFG.log"; exit 1; }
  python - "$R/gpurun_out/$TAG/$v.c$CFG.log" "$v" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[2]:10s} cfg {d['config']['workload'][:30]:30s} {d['value']:>12.0f} nodes/s  {d['ms_per_step']:8.3f} ms  "
      + " ".join(f"{k}={v:.4f}" for k, v in d["kernel_ms"].items()))
PY
done
