#!/bin/bash
# round-4 first GPU pass: DP / trainer / model tests, the streaming probe, the SQ counter passes
set -o pipefail
mkdir -p gpurun_out/r04a
timeout -k 10 700 python -u -m pytest tests/test_gpu_adam.py tests/test_gpu_dist.py tests/test_gpu_train_harness.py \
  tests/test_gpu_trainer_graph.py tests/test_gpu_model.py -x -v --timeout 400 --timeout-method thread \
  > gpurun_out/r04a/tests.log 2>&1
rc=$?
tail -25 gpurun_out/r04a/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 tools/membench2 > gpurun_out/r04a/membench2.jsonl 2>&1 || exit 1
cat gpurun_out/r04a/membench2.jsonl
bash tools/sq_pass.sh r04a
# A/B: deferred a2 stores in the edge forward (variants/efcd), bitwise check then timing pairs
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 200 python tools/grads_dump.py gpurun_out/r04a/g_default.pt > gpurun_out/r04a/gd.log 2>&1 || { tail -5 gpurun_out/r04a/gd.log; exit 1; }
PDG_LIB=variants/efcd/libpdivgnn_hip.so timeout -k 10 200 python tools/grads_dump.py gpurun_out/r04a/g_efcd.pt >> gpurun_out/r04a/gd.log 2>&1 || { tail -5 gpurun_out/r04a/gd.log; exit 1; }
python tools/grads_dump.py --compare gpurun_out/r04a/g_default.pt gpurun_out/r04a/g_efcd.pt
bash tools/ab.sh r04a 2 default efcd default efcd
