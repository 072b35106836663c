#!/bin/bash
# round-4 GPU pass: DP / trainer / model tests, the streaming probe, edge-forward variant A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 120 tools/membench2 > $O/membench2.jsonl 2>&1 || { tail -5 $O/membench2.jsonl; exit 1; }
cat $O/membench2.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_adam.py tests/test_gpu_dist.py tests/test_gpu_train_harness.py \
  tests/test_gpu_trainer_graph.py tests/test_gpu_model.py -x -v --timeout 400 --timeout-method thread \
  > $O/tests.log 2>&1
rc=$?
tail -12 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
# edge-forward variants: bitwise / close check, then timing pairs
for v in default efcd efcx efcdx ebwx allx; do
  lib=p-div-gnn_amd/pdg/libpdivgnn_hip.so; [ $v = default ] || lib=variants/$v/libpdivgnn_hip.so
  PDG_LIB=$lib timeout -k 10 200 python tools/grads_dump.py $O/g_$v.pt >> $O/gd.log 2>&1 || { tail -5 $O/gd.log; exit 1; }
done
for v in efcd efcx efcdx ebwx allx; do echo "== $v vs default"; python tools/grads_dump.py --compare $O/g_default.pt $O/g_$v.pt | tail -4; done
bash tools/ab.sh r04a 2 default efcd efcx efcdx ebwx allx default allx efcdx
