#!/bin/bash
# Engine-variant A/B on the GPU box: bitwise gradient check of every variant against the first, then
# config-2 timing (tools/ab_env.sh, two passes).   usage: tools/ab_var.sh TAG "ENV1" "ENV2" ...
# ("-" = no variable: the shipped defaults)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
i=0
for e in "$@"; do
  [ "$e" = "-" ] && e="PDG_AB=1"
  env PDG_AB=1 $e timeout -k 10 180 python tools/grads_dump.py "$O/g_$i.pt" > "$O/g_$i.log" 2>&1 \
    || { echo "grads_dump $e failed"; tail -5 "$O/g_$i.log"; exit 1; }
  if [ $i -gt 0 ]; then
    echo "bitwise $e vs $1:"; python tools/grads_dump.py --compare "$O/g_$i.pt" "$O/g_0.pt" | tail -3
  fi
  i=$((i + 1))
done
args=()
for e in "$@"; do [ "$e" = "-" ] && args+=("PDG_AB=1") || args+=("$e"); done
bash tools/ab_env.sh "$TAG" "${args[@]}"
