#!/bin/bash
# One SQ counter pass per library variant (GPU box): tools/pmc_sq_variants.sh TAG "COUNTERS" KERNEL_SUBSTRING v1 v2 ...
set -o pipefail
TAG=$1; CNT=$2; KS=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then lib=$R/p-div-gnn_amd/pdg/libpdivgnn_hip.so; else lib=$R/variants/$v/libpdivgnn_hip.so; fi
  PDG_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $CNT --output-format csv -d "$O/$v" -o b -- \
    python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras > "$O/$v.log" 2>&1 \
    || { echo "$v failed"; tail -5 "$O/$v.log"; exit 1; }
  rm -f "$O/$v"/*.db
  python "$R/tools/pmc_sq.py" "$O/$v/b_counter_collection.csv" 40 | grep -- "$KS" | sed "s/^/$v: /" | cut -c1-330
done
