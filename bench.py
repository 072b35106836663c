#!/usr/bin/env python3
"""P-DivGNN training throughput on MI355X: mesh-nodes/sec (fwd+bwd), 1..8 GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step is one full training step of the reference's hot loop
(scripts/gnn_train.py:154-207) on one minibatch resident in HBM: forward of
EncodeProcessDecode (10 message-passing steps, latent 128), per-graph NMSE
(+ lambda * divergence for config 3), backward, RCCL all-reduce of the flat
gradient bucket (N > 1) and the Adam update — all on the HIP kernels of
libpdivgnn_hip.so.  Workload per GPU (weak scaling, graph-level data
parallelism): BASELINE.json configs[1] = 8 synthetic periodic triangulated
71x71 meshes (5,041 nodes, 29,968 edges each).  value = nodes processed by all
ranks / max-over-ranks wall time.

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

PEAK_FP32_MFMA = 157.3e12   # MI355X dense fp32 MFMA, /opt/skills/guides/MI355X_MICROARCH.md
PEAK_HBM = 8.0e12           # MI355X HBM3E spec bandwidth
L = 128

CONFIGS = {
    2: dict(workload="P-GNN linear-elastic, 8 x 5,041-node periodic meshes per GPU, fwd+bwd (BASELINE configs[1])",
            graphs=8, n=71, hole=(0.0, 0.0), divergence=False, steps=10),
    3: dict(workload="P-DivGNN with divergence loss (lambda=10), 32 x 5,041-node periodic meshes per GPU",
            graphs=32, n=71, hole=(0.0, 0.0), divergence=True, steps=10),
    4: dict(workload="P-DivGNN hole plates, 8 x ~4.8k-node meshes per GPU (global batch 8*N)",
            graphs=8, n=71, hole=(0.08, 0.12), divergence=True, steps=10),
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

    def step():
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
    return {"value": round(n * d.num_nodes / el, 1), "unit": "nodes/s", "cores": threads, "kind": "port",
            "sample": f"{n} training steps (fwd+NMSE{'+div' if cfg['divergence'] else ''}+bwd) of one "
                      f"{d.num_nodes}-node graph, {cfg['steps']} MP steps, fp32, torch CPU "
                      f"({threads} threads), oracle/epd_oracle.py"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    pg = None
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=device)
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
    trainer = Trainer(model, lr=1e-3, divergence=cfg["divergence"], divergence_penalty=10.0, process_group=pg)
    plan = plan_for(batch)
    N, E = plan.n_nodes, plan.n_edges

    for _ in range(args.warmup):
        trainer.step(batch)
    torch.cuda.synchronize()
    eng = trainer.engine
    timed_kernels = ["edge_fwd", "edge_bwd", "wgrad_W2", "segment_sum", "pq_scatter_bwd"]
    eng.timed = {k: [] for k in timed_kernels}
    if pg is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = trainer.step(batch)
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

    kt = {k: sum(a.elapsed_time(b) for a, b in v) / max(len(v), 1) * 1e-3 for k, v in ev.items()}
    ktot = {k: sum(a.elapsed_time(b) for a, b in v) * 1e-3 for k, v in ev.items()}
    flop_edge = E * 3 * 2 * L * L           # 3 (128x128) GEMMs per edge and launch, executed
    rooflines = {
        "edge_fwd": ("mfma", flop_edge, PEAK_FP32_MFMA, "TFLOP/s"),
        "edge_bwd": ("mfma", flop_edge, PEAK_FP32_MFMA, "TFLOP/s"),
        "wgrad_W2": ("mfma", cfg["steps"] * 2 * E * 2 * L * L, PEAK_FP32_MFMA, "TFLOP/s"),
        "segment_sum": ("hbm", 512 * E + 4 * (N + 1) + 512 * N, PEAK_HBM, "GB/s"),
        "pq_scatter_bwd": ("hbm", 2 * 512 * E + 4 * E + 8 * (N + 1) + 2 * 512 * N, PEAK_HBM, "GB/s"),
    }

    def roof(k):
        bound, work, peak, unit = rooflines[k]
        ach = work / kt[k]
        scale = 1e12 if unit == "TFLOP/s" else 1e9
        return {"kernel": k, "bound": bound, "achieved": round(ach / scale, 2), "peak": round(peak / scale, 1),
                "unit": unit, "frac": round(ach / peak, 4), "traffic": None,
                "work_per_launch": work, "avg_launch_ms": round(kt[k] * 1e3, 4),
                "share_of_step": round(ktot[k] / el, 4)}

    dominant = max(["edge_fwd", "edge_bwd", "wgrad_W2"], key=lambda k: ktot[k])
    if rank == 0:
        res = {
            "metric": "mesh-nodes/sec (fwd+bwd) on periodic FEM graphs",
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
                       "parallelism": f"graph-DP x{world}", "final_loss": round(loss, 6)},
            "roofline": roof(dominant),
            "roofline_gather_scatter": [roof("segment_sum"), roof("pq_scatter_bwd")],
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
