# node_net with whole-row tiled a1 / a2 stores: op and model tests, then A/B against variants/base, configs 2 and 5
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06x}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 240 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc -ne 0 ] && exit 1
for rep in 1 2; do bash tools/ab.sh $TAG 2 base default || exit 1; done
for rep in 1 2; do bash tools/ab.sh $TAG 5 base default || exit 1; done
