#!/bin/bash
# Copy one round-6 measurement pass (tools/final_r06.sh TAG tests / countersA / countersB, tools/sweep_pass.sh
# TAG/sweep) from gpurun_out/TAG into profiles/r06_*, stamped with this tree, and print the figures DESIGN §6
# quotes.   tools/collect_r06.sh TAG
set -e
G=gpurun_out/$1; P=profiles
TREE=$(python -c "import bench; print(bench.tree_hash())")
cp $G/bench_line.json $P/r06_bench_config2.json
cp $G/prof_bench_line.json $P/r06_bench_config2_profiled.json
cp $G/gaps.json $P/r06_gaps.json; cp $G/gaps.txt $P/r06_gaps.txt
cp $G/parity.jsonl $P/r06_parity.jsonl
cp $G/prof/bench_kernel_stats.csv $P/r06_rocprof_kernel_stats.csv
cp $G/prof_summary.txt $P/r06_rocprof_summary.txt
cp $G/prof_window.json $P/r06_rocprof_window.json; cp $G/prof_window.txt $P/r06_rocprof_window.txt
for C in 2 3 4 5; do SUF=$([ $C = 2 ] && echo "" || echo "_c$C")
  for f in pmc_traffic sq; do for x in json txt; do cp $G/c$C/$f.$x $P/r06_$f$SUF.$x; done; done; done
{ echo "tree $TREE"; tail -4 $G/pytest_gpu.log; } > $P/r06_gpu_suite.txt
if [ -d $G/sweep ]; then
  { echo "tree $TREE"; cat $G/sweep/sweep_trace.txt; } > $P/r06_sweep_trace.txt
  cp $G/sweep/sweep_line.json $P/r06_sweep_line.json; cp $G/sweep/prof/sweep_kernel_stats.csv $P/r06_sweep_kernel_stats.csv
fi
python - <<'PY'
import json
d = json.load(open('profiles/r06_bench_config2.json'))
r = d['roofline']
print('tree', d['tree'], 'match', d['traffic_tree_match'])
print('c2 value %.0f ms %.3f launch %.4f frac %.4f pmc %.4f gp %.4f ro %.4f mfma %.3f cpu %.1f' % (
    d['value'], d['ms_per_step'], r['avg_launch_ms'], r['frac'], r['frac_pmc'], r['frac_gather_priced'],
    r['frac_reads_only'], d['mfma_busy_counters']['edge_fwd'], d['cpu_baseline']['value']))
for c in ['config3', 'config4', 'config5']:
    x = d['sub_results'][c]; rr = x['roofline']
    print(c, 'value %.0f ms %.3f frac %.4f pmc %.4f launch %.4f' % (x['value'], x['ms_per_step'], rr['frac'], rr['frac_pmc'], rr['avg_launch_ms']))
for row in d['sub_results']['published_sweep']['rows']:
    print('sweep', row['nodes'], row['fwd']['mean_ms'], row['fwd_prepro']['mean_ms'], row['fwd_replay']['mean_ms'],
          row['replay_gpu_ms'], row['speedup_vs_reference_fwd'], row['outputs_bitwise_equal'])
p = json.load(open('profiles/r06_pmc_traffic.json')); s = json.load(open('profiles/r06_sq.json'))['kernels']
w = json.load(open('profiles/r06_rocprof_window.json'))
sq = {k['kernel']: k for k in s}; ks = w['kernels']
for wn in ['edge_bwd_w2_kernel<true>', 'edge_fwd_coop_kernel<true, true, true>', 'edge_gout_wc_kernel<true, true>',
           'pq_scatter_bwd_kernel<true>', 'node_bwd_coop_kernel', 'segment_sum_kernel', 'node_net_x6_kernel',
           'gemm_sum2_coop_kernel<true, true>', 'node_pq_x6_kernel<true>', 'ln_colsum_nodes_kernel']:
    n = [k for k in ks if wn in k][0]; v = ks[n]; mb = p[n]['total'] / 1e6
    b = sq.get(n, {}).get('mfma_busy_at_2.4GHz')
    print(f"| `{n.split('(')[0].replace('void ', '')}` | {v['calls_per_step']:.0f} | {v['avg_us']:.1f} | "
          f"{v['calls_per_step'] * v['avg_us'] / 1e3:.3f} | {mb:.0f} | {mb * 1e6 / (v['avg_us'] * 1e-6) / 1e12:.2f} | "
          f"{('%.1f %%' % (100 * b)) if b else '—'} |")
PY
sed -n 2p $P/r06_gaps.txt; tail -1 $P/r06_rocprof_window.txt; tail -1 $P/r06_gpu_suite.txt
