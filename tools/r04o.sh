#!/bin/bash
# pair weight gradients at 4 waves per SIMD (2 blocks per CU, 128 VGPRs) vs the default 1 block per CU
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 200 python tools/grads_dump.py $O/g_default.pt > $O/gd.log 2>&1 || { tail -5 $O/gd.log; exit 1; }
PDG_LIB=variants/wgp_lb4/libpdivgnn_hip.so PDG_AB=1 PDG_PAIR_BLOCKS_PER_CU=2 timeout -k 10 200 python tools/grads_dump.py \
  $O/g_lb4.pt >> $O/gd.log 2>&1 || { tail -5 $O/gd.log; exit 1; }
python tools/grads_dump.py --compare $O/g_default.pt $O/g_lb4.pt | tail -3
run() {  # run NAME [env...]
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }
  python - $O/$name.log $name <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"{sys.argv[2]:8s} {d['value']:>12.0f} nodes/s {d['ms_per_step']:8.3f} ms")
PY
}
for rep in 1 2; do
  run default
  run lb4 PDG_LIB=variants/wgp_lb4/libpdivgnn_hip.so PDG_AB=1 PDG_PAIR_BLOCKS_PER_CU=2
done
cd /tmp && export TMPDIR=/tmp
for v in default lb4; do
  if [ $v = lb4 ]; then export PDG_LIB=$R/variants/wgp_lb4/libpdivgnn_hip.so PDG_AB=1 PDG_PAIR_BLOCKS_PER_CU=2; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$v -o b -- \
    python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras > $R/$O/prof_$v.log 2>&1 || { tail -5 $R/$O/prof_$v.log; exit 1; }
  grep -E "wgrad_x6_pair2|wgrad_x6_jobs" $R/$O/prof_$v/b_kernel_stats.csv | cut -d, -f1-4
done
