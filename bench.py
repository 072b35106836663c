#!/usr/bin/env python3
"""P-DivGNN training throughput on MI355X: mesh-nodes/sec (fwd+bwd), 1..8 GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step is one full training step of the reference's hot loop
(scripts/gnn_train.py:154-207) on one minibatch resident in HBM: forward of
EncodeProcessDecode (10 message-passing steps, latent 128), per-graph NMSE
(+ lambda * divergence for config 3), backward, RCCL all-reduce of the flat
gradient bucket (N > 1) and the Adam update — all on the HIP kernels of
libpdivgnn_hip.so.  Workload per GPU (weak scaling, graph-level data
parallelism): BASELINE.json configs[1] = 8 synthetic periodic triangulated
71x71 meshes (5,041 nodes, 29,968 edges each).  value = nodes processed by all
ranks / max-over-ranks wall time.  --config 5 times inference instead (one
forward of a 100k-node mesh, 15 layers, model.forward under no_grad as
gnn_inference.py calls it; metric mesh-nodes/sec (inference)).

Also reported: the roofline of the dominant kernel (HIP events around its
launches inside the timed region) and the reference algorithm's CPU path (the
op-for-op oracle restatement) timed on this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT), str(ROOT / "p-div-gnn_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PMC_FILE = ROOT / "profiles" / "r01_pmc_traffic.json"   # rocprofv3 --pmc of this bench (tools/gpu_measure.sh)
PMC_NAMES = {"edge_fwd": "void edge_fwd_kernel<true, true>", "edge_bwd": "void edge_bwd_kernel<true>",
             "segment_sum": "segment_sum_kernel", "node_net": "node_net_kernel", "pq_scatter_bwd": "pq_scatter_bwd_kernel",
             "wgrad_W2": "wgrad_x6_kernel", "edge_bwd_w2": "void edge_bwd_w2_kernel<true>",
             "edge_gout": "void edge_gout_wc_kernel<true>"}
PEAK_FP32_MFMA = 157.3e12   # MI355X dense fp32 MFMA, /opt/skills/guides/MI355X_MICROARCH.md
PEAK_BF16_MFMA = 16 * PEAK_FP32_MFMA   # dense bf16 MFMA (2.5 PF; the fp32 rate is 1/16 of it, same guide)
X6 = 6                      # bf16x6: six bf16 products per fp32-accurate product
PEAK_HBM = 8.0e12           # MI355X HBM3E spec bandwidth (same guide; 6.3 TB/s measured copy)
L = 128

CONFIGS = {
    2: dict(workload="P-GNN linear-elastic, 8 x 5,041-node periodic meshes per GPU, fwd+bwd (BASELINE configs[1])",
            graphs=8, n=71, hole=(0.0, 0.0), divergence=False, steps=10),
    3: dict(workload="P-DivGNN with divergence loss (lambda=10), 32 x 5,041-node periodic meshes per GPU",
            graphs=32, n=71, hole=(0.0, 0.0), divergence=True, steps=10),
    4: dict(workload="P-DivGNN hole plates, 8 x ~4.8k-node meshes per GPU (global batch 8*N)",
            graphs=8, n=71, hole=(0.08, 0.12), divergence=True, steps=10),
    5: dict(workload="inference, one synthetic 100,489-node periodic mesh per GPU, 15 MP layers (BASELINE configs[4])",
            graphs=1, n=317, hole=(0.0, 0.0), divergence=False, steps=15, inference=True),
}


def build_batch(cfg, seed, device):
    from pdg import graph, meshgen
    samples = meshgen.make_dataset(cfg["graphs"], n=cfg["n"], hole_radius=cfg["hole"], seed=seed)
    datas = [graph.sample_to_data(s) for s in samples]
    return graph.Batch.from_data_list(datas).to(device), samples


def dataset_stats(b):
    return {"mean_pos": b.pos.mean(), "std_pos": b.pos.std(), "mean_mean_stress": b.mean_stress.mean(),
            "std_mean_stress": b.mean_stress.std(), "mean_local_stress": b.local_stress.mean(),
            "std_local_stress": b.local_stress.std(), "mean_edge_weight": b.edge_attr.mean(),
            "std_edge_weight": b.edge_attr.std()}


def cpu_baseline(cfg, samples, seconds: float = 20.0):
    """The reference algorithm on this host's CPU cores: oracle/epd_oracle.py (the op-for-op
    restatement of models.py + gnn_train.py losses, validated against the reference's own
    outputs in tests/golden), fp32, one graph of the workload per step."""
    from oracle import epd_oracle as O
    from pdg import graph
    threads = max(1, min(16, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    d = graph.sample_to_data(samples[0])
    b = graph.Batch.from_data_list([d])
    st = {k: v.float() for k, v in dataset_stats(b).items()}
    P = {k: v.requires_grad_(True) for k, v in O.init_params().items()}
    args = (b.pos, b.mean_stress, b.nodes_types, b.edge_index, b.edge_attr)
    gt = (b.local_stress - st["mean_local_stress"]) / st["std_local_stress"]

    infer = cfg.get("inference", False)

    def step():
        if infer:
            with torch.no_grad():
                O.epd_forward(P, st, *args, cfg["steps"], scale_output=True)
            return
        pred = O.epd_forward(P, st, *args, cfg["steps"], scale_output=False)
        total, _, _ = O.batch_loss(pred, gt, b.ptr, [d.op_div_matrix], b.nodes_types, cfg["divergence"], 10.0)
        for p in P.values():
            p.grad = None
        total.backward()

    step()  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el > seconds or n >= 50:
            break
    what = "inference forwards" if infer else f"training steps (fwd+NMSE{'+div' if cfg['divergence'] else ''}+bwd)"
    return {"value": round(n * d.num_nodes / el, 1), "unit": "nodes/s", "cores": threads, "kind": "port",
            "sample": f"{n} {what} of one {d.num_nodes}-node graph, {cfg['steps']} MP steps, fp32, torch CPU "
                      f"({threads} threads), oracle/epd_oracle.py"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--dp-mode", default="replica", choices=["replica", "sync"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--graph", action="store_true",
                    help="replay forward+backward from a HIP graph captured in warmup (measured no faster: DESIGN §6)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; PDG_DIST_BACKEND=gloo with more ranks than GPUs only rehearses the
    # multi-rank flow (ranks share devices round-robin)
    backend = os.environ.get("PDG_DIST_BACKEND", "nccl")
    dev_index = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    pg = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
        pg = dist.group.WORLD

    from gnn_local_stress.models import EncodeProcessDecode
    from pdg.plan import plan_for
    from pdg.trainer import Trainer

    cfg = CONFIGS[args.config]
    batch, samples = build_batch(cfg, seed=69 + rank, device=device)
    stats = dataset_stats(batch)
    if pg is not None:  # dataset statistics are global constants of the training set
        v = torch.stack([stats[k].float() for k in stats])
        dist.all_reduce(v)
        stats = {k: v[i] / world for i, k in enumerate(stats)}
    torch.manual_seed(69)
    model = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=cfg["steps"], latent_size=L,
                                input_nodes_features_size=6, output_nodes_features_size=3, **stats).to(device)
    trainer = Trainer(model, lr=1e-3, divergence=cfg["divergence"], divergence_penalty=10.0, process_group=pg,
                      dp_mode=args.dp_mode, capture=args.graph)
    plan = plan_for(batch)
    N, E = plan.n_nodes, plan.n_edges

    infer = cfg.get("inference", False)
    if infer:
        def run_step():
            with torch.no_grad():
                return {"total": model(batch, scale_output=True).local_stress.abs().mean()}
    else:
        def run_step():
            return trainer.step(batch)
    for _ in range(args.warmup):
        run_step()
    torch.cuda.synchronize()
    eng = trainer.engine
    # HIP events bracket the timed kernels' launches in the last `ev_steps` steps of the timed
    # region (each event pair costs a few us of queue time; sampling keeps the region clean)
    timed_kernels = ["edge_fwd", "edge_bwd", "edge_gout", "wgrad_W2", "segment_sum", "node_net", "node_bwd",
                     "node_pq", "gemm_sum2", "pq_scatter_bwd"]
    fused = eng.fused_edge_wgrad
    ev_steps = min(args.steps, 3)
    graph_steps = 0 if (infer or not trainer.capture) else args.steps - ev_steps
    if pg is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i == args.steps - ev_steps:
            # the event-timed steps launch eagerly (events cannot bracket launches inside a graph
            # replay); the other timed steps replay the graph captured during warmup
            trainer.capture = False
            eng.timed = {k: [] for k in timed_kernels}
        out = run_step()
    torch.cuda.synchronize()
    if pg is not None:
        dist.barrier()
    el = time.perf_counter() - t0
    ev = eng.timed
    eng.timed = None
    if pg is not None:
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    loss = float(out["total"])

    ev = {k: v for k, v in ev.items() if v}
    kt = {k: sum(a.elapsed_time(b) for a, b in v) / len(v) * 1e-3 for k, v in ev.items()}
    ktot = {k: sum(a.elapsed_time(b) for a, b in v) * 1e-3 for k, v in ev.items()}
    S = cfg["steps"]
    nslab_bytes = getattr(eng, "_nslabs_e", 256) * (L * L + L) * 4
    # algorithmic work per launch (DESIGN.md "Kernels"): executed MFMA flops and the bytes the
    # kernel must read/write (inputs once, outputs once, int32 indices)
    # per kernel: ([(executed MFMA flops, the peak of that instruction type)], bytes); an fp32-accurate
    # 128x128 product per row costs 2*L*L fp32 flops on the fp32 MFMA, or 6x that in bf16 (bf16x6)
    g = 2 * L * L
    work = {
        # W_c product (fp32 MFMA) + 2 W2 products (bf16x6) per edge; reads a2e_prev, e_prev, 4 gathered
        # P/Q rows, src, dst; writes e_t, a2m, a2e and, when training, a1m, a1e
        "edge_fwd": ([(E * g, PEAK_FP32_MFMA), (E * 2 * g * X6, PEAK_BF16_MFMA)],
                     E * ((9 if infer else 11) * 4 * L + 8)),
        # fused (pdg_edge_bwd_w2): 2 W2^T products + 2 weight-gradient products per edge (bf16x6);
        # reads gaggr[dst], ge_next, a2m, a1m, a2e, a1e, dst; writes gz1m, gz1e, gC; one slab
        # read+write per block.  unfused (pdg_edge_bwd): W2^T x2 (bf16x6) + Wc^T (fp32); writes
        # gz2m, gz1m, gz2e, gz1e, gC, ge_out
        "edge_bwd": (([(E * 4 * g * X6, PEAK_BF16_MFMA)], E * (9 * 4 * L + 4) + 2 * nslab_bytes) if fused
                     else ([(E * 2 * g * X6, PEAK_BF16_MFMA), (E * g, PEAK_FP32_MFMA)], E * (12 * 4 * L + 4))),
        # fused Wc path (pdg_edge_gout_wc): Wc^T product + weight-gradient product (bf16x6); reads gC,
        # e, ge_next and the LayerNorm input of e (column sums), writes ge_out; one slab read+write
        "edge_gout": ([(E * 2 * g * X6, PEAK_BF16_MFMA)], E * 5 * 4 * L + 2 * nslab_bytes),
        # all steps' W2 segments: 2E rows per step of (G, X) 512-byte rows, one 64 KB slab per block
        "wgrad_W2": ([(S * 2 * E * g * X6, PEAK_BF16_MFMA)], S * 2 * E * 2 * 4 * L + 512 * (L * L + L) * 4),
        # dst-segment sum of LN(a2m): reads a2m (E rows) and rowptr, writes aggr (+ x-hat sums)
        "segment_sum": ([], 4 * L * E + 4 * (N + 1) + (1 if infer else 2) * 4 * L * N),
        # node_net, 2 fp32 GEMMs (K = 256, 128) per node: reads aggr, x; writes a2n (+ a1n)
        "node_net": ([(N * 2 * L * (2 * L + L), PEAK_FP32_MFMA)], 2 * 4 * L * N + (1 if infer else 2) * 4 * L * N),
        "pq_scatter_bwd": ([], 2 * 4 * L * E + 4 * E + 8 * (N + 1) + 2 * 4 * L * N),
    }

    pmc = {}
    if PMC_FILE.exists() and args.config == 2:
        data = json.loads(PMC_FILE.read_text())
        for k, prefix in PMC_NAMES.items():
            if fused and k == "edge_bwd":
                prefix = PMC_NAMES["edge_bwd_w2"]
            hit = [v for name, v in data.items() if name.startswith(prefix)]
            if hit:
                pmc[k] = round(hit[0]["total"])

    def roof(k):
        terms, nbytes = work[k]
        t = kt[k]
        flops = sum(f for f, _ in terms)
        t_peak = sum(f / pk for f, pk in terms)     # matrix-core time at peak rate
        f_mfma = t_peak / t
        f_hbm = nbytes / t / PEAK_HBM
        bound = "mfma" if f_mfma >= f_hbm else "hbm"
        if bound == "mfma":   # executed flops / time against the flop-weighted peak of the mix
            ach, peak, unit = flops / t / 1e12, flops / t_peak / 1e12, "TFLOP/s"
        else:
            ach, peak, unit = nbytes / t / 1e9, PEAK_HBM / 1e9, "GB/s"
        return {"kernel": k, "bound": bound, "achieved": round(ach, 2), "peak": round(peak, 1), "unit": unit,
                "frac": round(ach / peak, 4), "traffic": pmc.get(k),
                "traffic_source": (f"profiles/{PMC_FILE.name}: 2*FETCH_SIZE+WRITE_SIZE per dispatch"
                                   + (" (mean over all weights' wgrad dispatches)" if k == "wgrad_W2" else "")
                                   if k in pmc else None),
                "flops_per_launch": flops,
                "bytes_per_launch": nbytes, "frac_mfma": round(f_mfma, 4), "frac_hbm": round(f_hbm, 4),
                "avg_launch_ms": round(t * 1e3, 4), "share_of_step": round(ktot[k] / (el * ev_steps / args.steps), 4)}

    dominant = max([k for k in ("edge_fwd", "edge_bwd", "edge_gout", "wgrad_W2") if k in ktot], key=lambda k: ktot[k])
    if rank == 0:
        res = {
            "metric": ("mesh-nodes/sec (inference) on periodic FEM graphs" if infer
                       else "mesh-nodes/sec (fwd+bwd) on periodic FEM graphs"),
            "value": round(world * N * args.steps / el, 1),
            "unit": "nodes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic periodic triangulated meshes (pdg.meshgen, seed 69+rank), random-init weights (seed 69)",
            "config": {"workload": cfg["workload"], "graphs_per_gpu": cfg["graphs"], "nodes_per_gpu": N,
                       "edges_per_gpu": E, "global_batch": cfg["graphs"] * world,
                       "message_passing_steps": cfg["steps"], "latent": L, "divergence": cfg["divergence"],
                       "parallelism": f"graph-DP x{world}" + ("" if args.dp_mode == "replica" else " (sync-LN)"), "final_loss": round(loss, 6),
                       "hip_graph_steps": graph_steps},
            "roofline": roof(dominant),
            "roofline_gather_scatter": [roof(k) for k in ("segment_sum", "pq_scatter_bwd") if k in kt],
            "roofline_node_net": roof("node_net") if "node_net" in kt else None,
            "kernel_ms": {k: round(v * 1e3, 4) for k, v in kt.items()},
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(cfg, samples, args.cpu_seconds)
        else:
            res["cpu_baseline"] = None
        print(json.dumps(res), flush=True)
    if pg is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
