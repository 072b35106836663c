# whole-row tiled stores in edge_bwd_w2: the model tests, then A/B against variants/base at configs 2 and 3
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06v}; O=$R/gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_fullsize.py -x -q --timeout 240 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc -ne 0 ] && exit 1
for rep in 1 2; do bash tools/ab.sh $TAG 2 base default || exit 1; done
for rep in 1 2; do bash tools/ab.sh $TAG 3 base default || exit 1; done
