#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per dispatch of one kernel for several library variants (GPU box).
#   usage: tools/pmc_variants.sh TAG KERNEL_SUBSTRING name1 name2 ...   ("default" = the shipped library)
set -o pipefail
TAG=$1; KS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  if [ "$v" = default ]; then lib=$R/p-div-gnn_amd/pdg/libpdivgnn_hip.so; else lib=$R/variants/$v/libpdivgnn_hip.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    PDG_LIB=$lib timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$O/$v.$c" -o b -- \
      python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-extras > "$O/$v.$c.log" 2>&1 \
      || { echo "$v $c failed"; tail -5 "$O/$v.$c.log"; exit 1; }
    rm -f "$O/$v.$c"/*.db
  done
  python "$R/tools/pmc_summary.py" "$O/$v.FETCH_SIZE/b_counter_collection.csv" "$O/$v.WRITE_SIZE/b_counter_collection.csv" \
    | grep -- "$KS" | sed "s/^/$v: /"
done
