# pipelined gemm_sum2 (PDG_GSUM2_PIPE): its op test, then configs 2 and 3 alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06z}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 240 --timeout-method thread -k "gemm_sum2" > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc -ne 0 ] && exit 1
for rep in 1 2; do for v in 0 1; do for c in 2 3; do
  env PDG_AB=1 PDG_GSUM2_PIPE=$v timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-extras > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1])
print('gsum2_pipe=$v c$c %8.3f ms gemm_sum2 %.4f'%(d['ms_per_step'], d['kernel_ms']['gemm_sum2']))"
done; done; done
