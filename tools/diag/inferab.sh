# the inference edge forward (pdg_edge_fwd_infer) against pdg_edge_fwd_coop (engine variant fwd_infer_pipe off):
# config 5 and the published sweep, same library, alternating (the tests ran in the previous call)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06q}; O=$R/gpurun_out/$TAG; mkdir -p $O
for rep in 1 2; do for v in 0 1; do
  env PDG_AB=1 PDG_EDGE_FWD_INFER=$v timeout -k 10 300 python bench.py --config 5 --no-cpu-baseline --no-extras > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  python -c "
import json
d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][-1])
print('infer_pipe=$v c5 %8.3f ms edge_fwd %.4f'%(d['ms_per_step'], d['kernel_ms']['edge_fwd']))"
done; done
for v in 0 1; do
  env PDG_AB=1 PDG_EDGE_FWD_INFER=$v timeout -k 10 300 python bench.py --sweep-only > $O/sweep_$v.log 2>&1 || { tail -5 $O/sweep_$v.log; exit 1; }
  python - $O/sweep_$v.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
rows = d["published_sweep"]["rows"]
print("infer_pipe=" + sys.argv[2], " ".join(f"{r['nodes']}:{r['fwd_replay']['mean_ms']:.3f}/{r['replay_gpu_ms']:.3f}" for r in rows))
PY
done
