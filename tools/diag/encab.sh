# the pipelined edge encoder forward (PDG_ENC_PIPE): its op test, then configs 2 and 5 alternating
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r06t}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 240 --timeout-method thread -k "enc_fwd" > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; [ $rc -ne 0 ] && exit 1
for rep in 1 2; do for v in 0 1; do for c in 2 5; do
  env PDG_AB=1 PDG_ENC_PIPE=$v timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-extras > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1])
print('enc_pipe=$v c$c %8.3f ms edge_enc_fwd %.4f'%(d['ms_per_step'], d['kernel_ms']['edge_enc_fwd']))"
done; done; done
