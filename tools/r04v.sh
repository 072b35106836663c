#!/bin/bash
# the Wc pass in 16-row rounds two deep with scheduling groups (variants/gout2w, PDG_GOUT2=2): bitwise, timing
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04v
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 180 python tools/grads_dump.py "$O/g_default.pt" > "$O/g_default.log" 2>&1 || { tail -5 "$O/g_default.log"; exit 1; }
for v in gout2w; do
  PDG_LIB=$R/variants/$v/libpdivgnn_hip.so timeout -k 10 180 python tools/grads_dump.py "$O/g_$v.pt" > "$O/g_$v.log" 2>&1 \
    || { tail -5 "$O/g_$v.log"; exit 1; }
  echo "bitwise default vs $v:"; python tools/grads_dump.py --compare "$O/g_default.pt" "$O/g_$v.pt" | tail -2
done
bash tools/ab.sh r04v 2 default gout2w default gout2w default gout2w
