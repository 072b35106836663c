#!/bin/bash
# Times the data-parallel collectives on RCCL with one rank (GPU box): the default config-2 bench through
# a one-rank "nccl" process group, replica mode (one gradient all-reduce per step) and exact
# sync-LayerNorm mode (2 + 3 S forward and as many backward 16-byte all-reduces per step).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-rccl}
mkdir -p "$O"
for mode in replica sync; do
  PDG_FORCE_PG=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 \
    timeout -k 10 300 python "$R/bench.py" --no-cpu-baseline --no-extras --dp-mode $mode > "$O/$mode.log" 2>&1 \
    || { tail -5 "$O/$mode.log"; exit 1; }
  python - "$O/$mode.log" $mode <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
pr = d["config"]["per_rank"]
print(sys.argv[2], d.get("backend"), d["ms_per_step"], "allreduce_ms", pr["allreduce_ms"], "sync_ln_collectives_ms",
      pr["sync_ln_collectives_ms"], "compute_ms", pr["compute_ms"])
PY
done
