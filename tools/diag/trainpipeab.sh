# the pipelined edge forward in training (PDG_EDGE_FWD_TRAIN_PIPE: a1 rows from the product layout): its op test,
# then configs 2 and 3 alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06w}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 240 --timeout-method thread -k "fwd_pipe or fwd_infer" > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc -ne 0 ] && exit 1
for rep in 1 2; do for v in 0 1; do for c in 2 3; do
  env PDG_AB=1 PDG_EDGE_FWD_TRAIN_PIPE=$v timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-extras > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1])
print('train_pipe=$v c$c %8.3f ms edge_fwd %.4f edge_bwd %.4f'%(d['ms_per_step'], d['kernel_ms']['edge_fwd'], d['kernel_ms']['edge_bwd']))"
done; done; done
