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

The oracle's results at these sizes are cached fixtures (tests/golden/fullsize_c{2,3,4,5}.npz, made by
tests/golden/make_fullsize.py with the same oracle in float64 and float32): the float64 run alone takes
200-340 s of the GPU box's host cores at configs 3 / 4, most of the suite's budget.  Each fixture carries a
hash of the batch arrays, divergence operators, initial parameters and statistics it was computed from;
the test hashes its own workload and uses the fixture only when they are equal, otherwise (or with
PDG_FULLSIZE_LIVE=1) it runs the oracle live (configs 3 / 4 keeping one message-passing step's activations
at a time: checkpoint_steps).  Every config now has the fp32 oracle's own distance to fp64 per tensor
(the fixture's host; an fp32 CPU result is host-dependent).  A heartbeat line is appended to
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

import sys

from gpu_common import dev, rel

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))

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
    """The bench's batch and the model's initial state, built on the host exactly as the fixture
    generator builds them (statistics from the host copy of the batch), then moved to the GPU."""
    from make_fullsize import workload
    from gnn_local_stress.models import EncodeProcessDecode
    cfg, batch, stats, params = workload(config)
    model = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=cfg["steps"], latent_size=128,
                                input_nodes_features_size=6, output_nodes_features_size=3,
                                **{k: torch.tensor(v) for k, v in stats.items()})
    model.load_state_dict(params)
    return cfg, batch, stats, params, model.to(dev())


def _reference(config, cfg, batch, stats, params):
    """The oracle's float64 results and the float32 run's distances: from the fixture when its workload
    hash equals this workload's, else computed live.  Returns (rec, source)."""
    import numpy as np
    from make_fullsize import oracle, workload_hash
    path = Path(__file__).resolve().parent / "golden" / f"fullsize_c{config}.npz"
    h = workload_hash(batch, params, stats)
    if path.exists() and os.environ.get("PDG_FULLSIZE_LIVE") != "1":
        z = np.load(path, allow_pickle=False)
        if str(z["hash"]) == h:
            rec = {"pred64": torch.from_numpy(z["pred64"]), "f32_vs_f64": float(z["f32_vs_f64"])}
            if "total64" in z.files:
                rec.update(total64=float(z["total64"]), nmse64=float(z["nmse64"]),
                           grad64={k[7:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("grad64.")},
                           grad32_vs_f64={k[14:]: float(z[k]) for k in z.files if k.startswith("grad32_vs_f64.")})
            return rec, f"{path.name} (hash {h})"
        source = f"live: {path.name} hash {z['hash']} != workload {h}"
    else:
        source = "live" if path.exists() else f"live: no {path.name}"
    train = not cfg.get("inference")
    big = batch.num_edges > 500_000
    p64, t64, n64, g64 = oracle(params, stats, batch, cfg["steps"], torch.float64, cfg["divergence"], train, big)
    p32, _, _, g32 = oracle(params, stats, batch, cfg["steps"], torch.float32, cfg["divergence"], train, big)
    rec = {"pred64": p64, "f32_vs_f64": rel(p32, p64)}
    if train:
        rec.update(total64=t64, nmse64=n64, grad64=g64, grad32_vs_f64={k: rel(g32[k], g64[k]) for k in g64})
    return rec, source


@pytest.mark.parametrize("config", [pytest.param(2, marks=pytest.mark.timeout(900)),
                                    pytest.param(3, marks=pytest.mark.timeout(900)),
                                    pytest.param(4, marks=pytest.mark.timeout(1100))])
def test_training_step_at_baseline_size(config):
    from pdg.trainer import Trainer
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg, batch, stats, params, model = _workload(config)
    gbatch = batch.to(dev())
    with torch.no_grad():
        pred = model(gbatch, scale_output=False).local_stress.cpu()
    tr = Trainer(model, lr=1e-3, divergence=cfg["divergence"], divergence_penalty=10.0)
    out = tr.step(gbatch)                     # the benchmarked step: forward, loss, backward, Adam
    torch.cuda.synchronize()
    total, nmse = float(out["total"]), float(out["nmse"])
    grads = {n: tr.G[n].detach().cpu().clone() for n in tr.G}
    del tr, out, gbatch
    t0 = time.time()
    ref, source = _reference(config, cfg, batch, stats, params)
    g64 = ref["grad64"]
    rec = {"config": config, "nodes": batch.num_nodes, "edges": batch.num_edges, "graphs": batch.num_graphs,
           "internal_boundary_nodes": int((batch.nodes_types == -1).sum()), "oracle_source": source,
           "pred_vs_f64": rel(pred, ref["pred64"]), "f32_vs_f64": ref["f32_vs_f64"],
           "loss_vs_f64": abs(total - ref["total64"]) / abs(ref["total64"]),
           "nmse_vs_f64": abs(nmse - ref["nmse64"]) / abs(ref["nmse64"]), "grads": {}}
    for name in g64:
        rec["grads"][name] = (rel(grads[name], g64[name]), ref["grad32_vs_f64"][name])
    worst = max(rec["grads"], key=lambda n: rec["grads"][n][0])
    rec["worst_grad"] = [worst, *rec["grads"][worst]]
    rec["worst_margin"] = max(g / max(GRAD_TOL, 2 * r) for g, r in rec["grads"].values())
    rec["oracle_s"] = round(time.time() - t0, 1)
    _log(rec)
    # the fp32 oracle's output is within f32_vs_f64 of fp64, so both bounds below hold against it too
    assert rec["pred_vs_f64"] < OUT_TOL and rec["pred_vs_f64"] + rec["f32_vs_f64"] < 2 * OUT_TOL, rec
    assert rec["loss_vs_f64"] < OUT_TOL and rec["nmse_vs_f64"] < OUT_TOL, rec
    for name, (got, ref32) in rec["grads"].items():
        assert got <= max(GRAD_TOL, 2 * ref32), (name, got, ref32)


@pytest.mark.timeout(900)
def test_inference_at_baseline_size():
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg, batch, stats, params, model = _workload(5)
    with torch.no_grad():                     # gnn_inference.py:58-60
        out = model(batch.to(dev()), scale_output=True).local_stress.cpu()
    ref, source = _reference(5, cfg, batch, stats, params)
    rec = {"config": 5, "nodes": batch.num_nodes, "edges": batch.num_edges, "oracle_source": source,
           "out_vs_f64": rel(out, ref["pred64"]), "f32_vs_f64": ref["f32_vs_f64"]}
    _log(rec)
    assert rec["out_vs_f64"] < OUT_TOL and rec["out_vs_f64"] + rec["f32_vs_f64"] < 2 * OUT_TOL, rec
