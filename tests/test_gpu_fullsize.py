"""Parity at the BASELINE workloads themselves (BASELINE.json configs[1] to [4]): the exact
batches bench.py times, run through the exact benchmarked path (pdg.trainer.Trainer for
training, EncodeProcessDecode.forward under no_grad for inference), checked against the CPU
oracle (oracle/epd_oracle.py) in float32 AND float64 on this host.

* config 2 — 8 x 5,041-node periodic meshes (N = 40,328, E = 239,744), 10 MP steps, NMSE,
  forward + backward;
* config 3 — 32 x 5,041 nodes (N = 161,312, E = 958,976), NMSE + 10 x divergence, forward +
  backward (the divergence stencil at full size);
* config 4 — 64 hyperelastic-style hole plates (N = 312,688, E = 1,853,216 at seed 69: internal-
  boundary nodes labelled -1, strain +-0.15), NMSE + 10 x divergence, forward + backward: the
  largest graph-LayerNorm reductions of any config (2.4e8 elements per edge LayerNorm, 3.7e7
  rows per W2 weight gradient) and the only one with the -1 divergence mask at scale
  (scripts/gnn_train.py:79-86);
* config 5 — one 317 x 317 periodic mesh (N = 100,489, E = 601,672), 15 MP steps, inference.

Tolerances (north_star "within 1e-5 rel fp32"; the same rules as tests/test_gpu_model.py):
output field and losses within 1e-5 relative (L2) of both oracles; every parameter gradient
within max(3e-5, 2 x the fp32 oracle's own distance to fp64) of the fp64 oracle (round 4: the
fixed floor tightened from 1e-4 to 3e-5, 1.5x the worst gradient error on record, config 4's
edge_encoder.0.weight at 2.0e-5).  These are the
sizes at which the bf16x6 products (W2 in the edge kernels, every weight gradient) and the fp64
graph-LayerNorm reductions accumulate the most terms (up to 9.6e5 rows per LayerNorm and 2e7
rows per weight gradient), so they are where a precision shortfall would show.

At configs 3 and 4 the oracle keeps activations of one message-passing step at a time
(checkpoint_steps: ~35 GB of host memory in float64 instead of ~170 GB) and the float32 oracle
runs only when a gradient is outside the fixed 3e-5 bound (it can only loosen the bound) or when
PDG_PARITY_FP32=1 asks for the record (profiles/r04_parity.jsonl holds such a run: the fp32
oracle's own distance to fp64 beside the GPU's, per tensor): the float64 run alone takes a few
minutes of host CPU.  A heartbeat line is appended to
gpurun_out/fullsize_heartbeat.log every 20 s while a test runs (long silent runs look hung).
Every test appends its measured errors as one JSON line to gpurun_out/parity.jsonl (and to
$PDG_PARITY_LOG when set), so the margins to the tolerances are on record, not only "passed".
"""
import json
import os
import threading
import time
from pathlib import Path

import pytest
import torch

from gpu_common import dev, rel

pytestmark = pytest.mark.gpu

OUT_TOL = 1e-5
GRAD_TOL = 3e-5


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.fixture(autouse=True)
def _heartbeat(request):
    out = Path(os.environ.get("GRAFT_REPO_ROOT", Path(__file__).resolve().parents[1])) / "gpurun_out"
    stop = threading.Event()

    def beat():
        t0 = time.time()
        while not stop.wait(20.0):
            try:
                out.mkdir(exist_ok=True)
                with open(out / "fullsize_heartbeat.log", "a") as f:
                    f.write(f"{request.node.name} running {time.time() - t0:.0f} s\n")
            except OSError:
                pass
    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()
    th.join()


def _log(rec):
    rec = {**rec, "out_tol": OUT_TOL, "grad_tol_rule": f"max({GRAD_TOL}, 2 x fp32-oracle vs fp64)"}
    out = Path(os.environ.get("GRAFT_REPO_ROOT", Path(__file__).resolve().parents[1])) / "gpurun_out"
    paths = [out / "parity.jsonl"] + ([Path(os.environ["PDG_PARITY_LOG"])] if os.environ.get("PDG_PARITY_LOG") else [])
    for path in paths:
        try:
            path.parent.mkdir(parents=True, exist_ok=True)
            with open(path, "a") as f:
                f.write(json.dumps(rec) + "\n")
        except OSError:
            pass
    print("parity:", json.dumps(rec))


def _workload(config):
    import bench
    cfg = bench.CONFIGS[config]
    batch, _ = bench.build_batch(cfg, seed=69, device=dev())
    stats = bench.dataset_stats(batch)
    from gnn_local_stress.models import EncodeProcessDecode
    torch.manual_seed(69)
    model = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=cfg["steps"], latent_size=128,
                                input_nodes_features_size=6, output_nodes_features_size=3, **stats).to(dev())
    return cfg, batch, {k: float(v) for k, v in stats.items()}, model


def _oracle(params, stats, batch, steps, dtype, divergence, train, checkpoint=False):
    from oracle import epd_oracle as O
    P = {k: v.detach().cpu().to(dtype).clone().requires_grad_(train) for k, v in params.items()}
    st = {k: torch.tensor(v, dtype=dtype) for k, v in stats.items()}
    b = batch
    args = (b.pos.cpu().to(dtype), b.mean_stress.cpu().to(dtype), b.nodes_types.cpu(), b.edge_index.cpu(),
            b.edge_attr.cpu().to(dtype))
    with torch.set_grad_enabled(train):
        pred = O.epd_forward(P, st, *args, steps, scale_output=not train, checkpoint_steps=checkpoint)
    if not train:
        return pred, None, None, None
    gt = (b.local_stress.cpu().to(dtype) - st["mean_local_stress"]) / st["std_local_stress"]
    ops = [d.op_div_matrix.to(dtype) for d in b._data_list] if divergence else None
    total, nmse, _ = O.batch_loss(pred, gt, b.ptr, ops, b.nodes_types.cpu(), divergence, 10.0)
    total.backward()
    return pred.detach(), float(total), float(nmse), {k: v.grad for k, v in P.items()}


@pytest.mark.parametrize("config", [pytest.param(2, marks=pytest.mark.timeout(900)),
                                    pytest.param(3, marks=pytest.mark.timeout(900)),
                                    pytest.param(4, marks=pytest.mark.timeout(1100))])
def test_training_step_at_baseline_size(config):
    from pdg.trainer import Trainer
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg, batch, stats, model = _workload(config)
    params = {k: v.detach().clone() for k, v in model.state_dict().items()}
    with torch.no_grad():
        pred = model(batch, scale_output=False).local_stress.cpu()
    tr = Trainer(model, lr=1e-3, divergence=cfg["divergence"], divergence_penalty=10.0)
    out = tr.step(batch)                      # the benchmarked step: forward, loss, backward, Adam
    torch.cuda.synchronize()
    total, nmse = float(out["total"]), float(out["nmse"])
    grads = {n: tr.G[n].detach().cpu().clone() for n in tr.G}
    del tr, out
    big = batch.num_edges > 500_000
    t0 = time.time()
    p64, t64, n64, g64 = _oracle(params, stats, batch, cfg["steps"], torch.float64, cfg["divergence"], True, big)
    rec = {"config": config, "nodes": batch.num_nodes, "edges": batch.num_edges, "graphs": batch.num_graphs,
           "internal_boundary_nodes": int((batch.nodes_types == -1).sum()),
           "pred_vs_f64": rel(pred, p64), "loss_vs_f64": abs(total - t64) / abs(t64),
           "nmse_vs_f64": abs(nmse - n64) / abs(n64), "grads": {}}
    need32 = (not big or os.environ.get("PDG_PARITY_FP32") == "1"
              or any(rel(grads[n], g64[n]) > GRAD_TOL for n in g64))
    g32 = None
    if need32:
        p32, t32, _, g32 = _oracle(params, stats, batch, cfg["steps"], torch.float32, cfg["divergence"], True, big)
        rec.update(pred_vs_f32=rel(pred, p32), f32_vs_f64=rel(p32, p64), loss_f32_vs_f64=abs(t32 - t64) / abs(t64))
    for name in g64:
        rec["grads"][name] = (rel(grads[name], g64[name]), rel(g32[name], g64[name]) if g32 else None)
    worst = max(rec["grads"], key=lambda n: rec["grads"][n][0])
    rec["worst_grad"] = [worst, *rec["grads"][worst]]
    rec["oracle_s"] = round(time.time() - t0, 1)
    _log(rec)
    assert rec["pred_vs_f64"] < OUT_TOL and rec.get("pred_vs_f32", 0.0) < OUT_TOL, rec
    assert rec["loss_vs_f64"] < OUT_TOL and rec["nmse_vs_f64"] < OUT_TOL, rec
    for name, (got, ref32) in rec["grads"].items():
        assert got <= max(GRAD_TOL, 2 * (ref32 or 0.0)), (name, got, ref32)


@pytest.mark.timeout(900)
def test_inference_at_baseline_size():
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg, batch, stats, model = _workload(5)
    params = {k: v.detach().clone() for k, v in model.state_dict().items()}
    with torch.no_grad():                     # gnn_inference.py:58-60
        out = model(batch, scale_output=True).local_stress.cpu()
    ref64, _, _, _ = _oracle(params, stats, batch, cfg["steps"], torch.float64, False, False)
    ref32, _, _, _ = _oracle(params, stats, batch, cfg["steps"], torch.float32, False, False)
    rec = {"config": 5, "nodes": batch.num_nodes, "edges": batch.num_edges, "out_vs_f64": rel(out, ref64),
           "out_vs_f32": rel(out, ref32), "f32_vs_f64": rel(ref32, ref64)}
    _log(rec)
    assert rec["out_vs_f64"] < OUT_TOL and rec["out_vs_f32"] < OUT_TOL, rec
