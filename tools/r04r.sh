#!/bin/bash
# edge encoder backward software-pipelined (PDG_EEB_PIPE 1..3 library variants): bitwise gradients against
# the shipped library, then config-2 timing of each (tools/ab.sh, two passes)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04r
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 180 python tools/grads_dump.py "$O/g_default.pt" > "$O/g_default.log" 2>&1 || { tail -5 "$O/g_default.log"; exit 1; }
for v in eebpipe1 eebpipe2 eebpipe3; do
  PDG_LIB=$R/variants/$v/libpdivgnn_hip.so timeout -k 10 180 python tools/grads_dump.py "$O/g_$v.pt" > "$O/g_$v.log" 2>&1 \
    || { tail -5 "$O/g_$v.log"; exit 1; }
  echo "bitwise default vs $v:"; python tools/grads_dump.py --compare "$O/g_default.pt" "$O/g_$v.pt" | tail -2
done
bash tools/ab.sh r04r 2 default eebpipe1 eebpipe2 eebpipe3 default eebpipe1 eebpipe2 eebpipe3
