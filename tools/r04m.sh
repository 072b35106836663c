#!/bin/bash
# GPU suite + full-size config 2 + measurement, then the warp-specialized weight-gradient pair kernel A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
bash tools/r04h.sh r04m || exit $?
O=gpurun_out/r04m
for v in default wgp_ws; do
  lib=p-div-gnn_amd/pdg/libpdivgnn_hip.so; [ $v = default ] || lib=variants/$v/libpdivgnn_hip.so
  PDG_LIB=$lib timeout -k 10 200 python tools/grads_dump.py $O/g_$v.pt >> $O/gd.log 2>&1 || { tail -5 $O/gd.log; exit 1; }
done
python tools/grads_dump.py --compare $O/g_default.pt $O/g_wgp_ws.pt | tail -4
bash tools/ab.sh r04m 2 default wgp_ws default wgp_ws
