#!/bin/bash
# node_net software-pipelined variants: bitwise check of the gradients, then same-box A/B timing pairs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=gpurun_out/${1:-r04i}
mkdir -p $O
for v in default nn_p1 nn_p2 nn_p3; do
  lib=p-div-gnn_amd/pdg/libpdivgnn_hip.so; [ $v = default ] || lib=variants/$v/libpdivgnn_hip.so
  PDG_LIB=$lib timeout -k 10 200 python tools/grads_dump.py $O/g_$v.pt >> $O/gd.log 2>&1 || { tail -5 $O/gd.log; exit 1; }
done
for v in nn_p1 nn_p2 nn_p3; do echo "== $v vs default"; python tools/grads_dump.py --compare $O/g_default.pt $O/g_$v.pt | tail -3; done
bash tools/ab.sh ${1:-r04i} 2 default nn_p1 nn_p2 nn_p3 default nn_p1 nn_p2 nn_p3
