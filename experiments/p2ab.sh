set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 240 --timeout-method thread -k "p2_matches_coop" > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc -ne 0 ] && exit 1
for rep in 1 2; do for v in 0 1; do for c in 2 5; do
  env PDG_AB=1 PDG_EDGE_FWD_P2=$v timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-extras > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1])
print('p2=$v c$c %8.3f ms edge_fwd %.4f'%(d['ms_per_step'], d['kernel_ms']['edge_fwd']))"
done; done; done
