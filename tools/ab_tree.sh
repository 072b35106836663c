#!/bin/bash
# A/B of the working tree against whole-tree variants (variants/<v>/: a git export with its own in-tree
# library, e.g. the previous commit): bitwise gradient check, then config-2 timing twice each.
#   usage: tools/ab_tree.sh TAG v1 [v2 ...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 180 python tools/grads_dump.py "$O/g_default.pt" > "$O/g_default.log" 2>&1 || { tail -5 "$O/g_default.log"; exit 1; }
for v in "$@"; do
  timeout -k 10 180 python "variants/$v/tools/grads_dump.py" "$O/g_$v.pt" > "$O/g_$v.log" 2>&1 || { tail -5 "$O/g_$v.log"; exit 1; }
  echo "bitwise default vs $v:"; python tools/grads_dump.py --compare "$O/g_default.pt" "$O/g_$v.pt" | tail -3
done
bash tools/ab.sh "$TAG" 2 default "$@" default "$@"
