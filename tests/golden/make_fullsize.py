"""Oracle results at the BASELINE sizes, cached as fixtures for tests/test_gpu_fullsize.py.

    python tests/golden/make_fullsize.py [config ...]      (default: 2 3 4 5)

For each of bench.CONFIGS 2-5 this builds the exact batch bench.py times (seed 69, on the CPU), the
model's initial parameters (torch.manual_seed(69), the dataset statistics of that batch) and runs the
CPU oracle (oracle/epd_oracle.py, test infrastructure) in float64 AND float32: the float64 output field,
loss and every parameter gradient, and the float32 run's distances to float64 (the reference fp32 CPU
path's own error, per tensor).  The test on the GPU box checks a hash of the batch arrays and parameters
against the fixture's before using it and recomputes live when they differ, so a stale fixture can
never pass for the current workload.  Saved: tests/golden/fullsize_c{N}.npz (float64 output and
gradients rounded to float32, far below the 1e-5 / 3e-5 tolerances they are compared at).

Why cached: the float64 oracle at configs 3 / 4 takes 200-340 s of the GPU box's 16 host cores, most
of the GPU suite's 900 s budget; generating here takes that time once.
"""
from __future__ import annotations

import hashlib
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "p-div-gnn_amd"), str(ROOT / "tests")]

OUT = Path(__file__).resolve().parent


def workload_hash(batch, params: dict, stats: dict) -> str:
    """sha256 (16 hex) of everything the oracle's result depends on: the batch arrays (CPU copies),
    the divergence operators, the parameters and the 8 statistics."""
    h = hashlib.sha256()
    b = batch
    for t in (b.pos, b.mean_stress, b.local_stress, b.nodes_types, b.edge_index, b.edge_attr, b.ptr):
        a = t.detach().cpu().contiguous().numpy()
        h.update(str(a.dtype).encode() + str(a.shape).encode())
        h.update(a.tobytes())
    for d in b._data_list:
        op = d.op_div_matrix.coalesce()
        h.update(op.indices().numpy().tobytes())
        h.update(op.values().numpy().tobytes())
    for k in sorted(params):
        h.update(k.encode())
        h.update(params[k].detach().cpu().contiguous().numpy().tobytes())
    for k in sorted(stats):
        h.update(f"{k}={float(stats[k])!r}".encode())
    return h.hexdigest()[:16]


def exact_stats(b) -> dict:
    """bench.dataset_stats (datasets.py:283-291's mean / unbiased std of the batch) computed host-
    independently: exactly rounded sums (math.fsum over float64) rounded once to float32.  torch's CPU
    reductions split the work by thread count and vector width, so the same batch gave statistics a few
    ulps apart on two hosts, and with them different fixtures."""
    import math
    out = {}
    for name, t in (("pos", b.pos), ("mean_stress", b.mean_stress), ("local_stress", b.local_stress),
                    ("edge_weight", b.edge_attr)):
        x = t.detach().cpu().double().reshape(-1).tolist()
        n = len(x)
        mean = math.fsum(x) / n
        var = math.fsum((v - mean) ** 2 for v in x) / (n - 1)
        key_m = "mean_" + name if name != "edge_weight" else "mean_edge_weight"
        out[key_m] = float(np.float32(mean))
        out[key_m.replace("mean_", "std_", 1)] = float(np.float32(math.sqrt(var)))
    return {k: out[k] for k in ("mean_pos", "std_pos", "mean_mean_stress", "std_mean_stress", "mean_local_stress",
                                "std_local_stress", "mean_edge_weight", "std_edge_weight")}


def workload_parts(batch, params: dict, stats: dict) -> dict:
    """Component hashes of workload_hash (to find which input differs between two hosts)."""
    out = {}
    b = batch
    for name in ("pos", "mean_stress", "local_stress", "nodes_types", "edge_index", "edge_attr", "ptr"):
        out[name] = hashlib.sha256(getattr(b, name).detach().cpu().contiguous().numpy().tobytes()).hexdigest()[:8]
    h = hashlib.sha256()
    for d in b._data_list:
        op = d.op_div_matrix.coalesce()
        h.update(op.indices().numpy().tobytes())
        h.update(op.values().numpy().tobytes())
    out["op_div"] = h.hexdigest()[:8]
    h = hashlib.sha256()
    for k in sorted(params):
        h.update(params[k].detach().cpu().contiguous().numpy().tobytes())
    out["params"] = h.hexdigest()[:8]
    out["stats"] = hashlib.sha256(repr(sorted(stats.items())).encode()).hexdigest()[:8]
    return out


def workload(config: int, device="cpu"):
    """(cfg, batch, stats as floats, params) of a BASELINE config, as the tests and bench build it."""
    import bench
    from gnn_local_stress.models import EncodeProcessDecode
    cfg = bench.CONFIGS[config]
    batch, _ = bench.build_batch(cfg, seed=69, device="cpu")
    stats = exact_stats(batch)
    torch.manual_seed(69)
    model = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=cfg["steps"], latent_size=128,
                                input_nodes_features_size=6, output_nodes_features_size=3,
                                **{k: torch.tensor(v) for k, v in stats.items()})
    params = {k: v.detach().clone() for k, v in model.state_dict().items()}
    return cfg, batch.to(device), stats, params


def oracle(params, stats, batch, steps, dtype, divergence, train, checkpoint=False):
    """The oracle on the workload (float64 or float32): (pred, total, nmse, grads)."""
    from oracle import epd_oracle as O
    P = {k: v.detach().cpu().to(dtype).clone().requires_grad_(train) for k, v in params.items()}
    st = {k: torch.tensor(v, dtype=dtype) for k, v in stats.items()}
    b = batch
    args = (b.pos.cpu().to(dtype), b.mean_stress.cpu().to(dtype), b.nodes_types.cpu(), b.edge_index.cpu(),
            b.edge_attr.cpu().to(dtype))
    with torch.set_grad_enabled(train):
        pred = O.epd_forward(P, st, *args, steps, scale_output=not train, checkpoint_steps=checkpoint)
    if not train:
        return pred.detach(), None, None, None
    gt = (b.local_stress.cpu().to(dtype) - st["mean_local_stress"]) / st["std_local_stress"]
    ops = [d.op_div_matrix.to(dtype) for d in b._data_list] if divergence else None
    total, nmse, _ = O.batch_loss(pred, gt, b.ptr, ops, b.nodes_types.cpu(), divergence, 10.0)
    total.backward()
    return pred.detach(), float(total), float(nmse), {k: v.grad for k, v in P.items()}


def rel(a, b) -> float:
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def make(config: int) -> Path:
    t0 = time.time()
    cfg, batch, stats, params = workload(config)
    train = not cfg.get("inference")
    big = batch.num_edges > 500_000
    p64, t64, n64, g64 = oracle(params, stats, batch, cfg["steps"], torch.float64, cfg["divergence"], train, big)
    p32, t32, _, g32 = oracle(params, stats, batch, cfg["steps"], torch.float32, cfg["divergence"], train, big)
    rec = {"hash": np.array(workload_hash(batch, params, stats)), "config": np.array(config),
           "pred64": p64.float().numpy(), "f32_vs_f64": np.array(rel(p32, p64)),
           "host": np.array(f"{os.cpu_count()} CPUs, torch {torch.__version__}, {torch.get_num_threads()} threads"),
           "seconds": np.array(time.time() - t0)}
    for k, v in stats.items():
        rec[f"stat.{k}"] = np.array(v)
    if train:
        rec.update(total64=np.array(t64), nmse64=np.array(n64), loss32_vs_f64=np.array(abs(t32 - t64) / abs(t64)))
        for k in g64:
            rec[f"grad64.{k}"] = g64[k].float().numpy()
            rec[f"grad32_vs_f64.{k}"] = np.array(rel(g32[k], g64[k]))
    path = OUT / f"fullsize_c{config}.npz"
    np.savez_compressed(path, **rec)
    print(f"config {config}: {path.name} ({path.stat().st_size / 1e6:.1f} MB) in {time.time() - t0:.0f} s", flush=True)
    return path


def _heartbeat(period: float = 30.0):
    """A line on stdout every `period` s (a long silent run on the GPU box is taken to be hung)."""
    import threading
    t0 = time.time()

    def beat():
        while True:
            time.sleep(period)
            print(f"  ... {time.time() - t0:.0f} s", flush=True)
    threading.Thread(target=beat, daemon=True).start()


if __name__ == "__main__":
    _heartbeat()
    for c in [int(a) for a in sys.argv[1:]] or [2, 3, 4, 5]:
        print(f"config {c} ...", flush=True)
        make(c)
