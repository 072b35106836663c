#!/bin/bash
# paired weight gradients software-pipelined (variants wgp2 / wgp3: PDG_WGP_PIPE=2 / 3): bitwise, timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04z2
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 180 python tools/grads_dump.py "$O/g_default.pt" > "$O/g_default.log" 2>&1 || { tail -5 "$O/g_default.log"; exit 1; }
for v in wgp2 wgp3; do
  PDG_LIB=$R/variants/$v/libpdivgnn_hip.so timeout -k 10 180 python tools/grads_dump.py "$O/g_$v.pt" > "$O/g_$v.log" 2>&1 \
    || { tail -5 "$O/g_$v.log"; exit 1; }
  echo "bitwise default vs $v:"; python tools/grads_dump.py --compare "$O/g_default.pt" "$O/g_$v.pt" | tail -2
done
bash tools/ab.sh r04z2 2 default wgp2 wgp3 default wgp2 wgp3
