#!/usr/bin/env python3
"""Minibatch assembly cost: host PyG-style collate + H2D + plan build vs DeviceGraphStore.batch.

    python tools/bench_collate.py [--graphs 64] [--reps 20]
Prints one JSON line per batch size (ms per batch, median over reps, device synchronised)."""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "p-div-gnn_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    from pdg import graph, meshgen
    from pdg.collate import DeviceGraphStore
    from pdg.plan import plan_for
    dev = torch.device("cuda:0")
    samples = meshgen.make_dataset(args.graphs, n=71, hole_radius=(0.0, 0.0), seed=69)
    datas = [graph.sample_to_data(s) for s in samples]
    t0 = time.perf_counter()
    store = DeviceGraphStore(datas, dev)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    g = torch.Generator().manual_seed(0)
    for bs in (8, 32):
        host, devt = [], []
        for r in range(args.reps + 2):
            idx = torch.randperm(args.graphs, generator=g)[:bs].tolist()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            b = graph.Batch.from_data_list([datas[i] for i in idx]).to(dev)
            plan_for(b)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            b2 = store.batch(idx)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            if r >= 2:
                host.append(t1 - t0)
                devt.append(t2 - t1)
        host.sort()
        devt.sort()
        n = int(b2.ptr[-1])
        print(json.dumps({"what": "minibatch assembly", "graphs_per_batch": bs, "nodes": n,
                          "edges": int(b2.edge_index.shape[1]),
                          "host_collate_h2d_plan_ms": round(host[len(host) // 2] * 1e3, 3),
                          "device_collate_ms": round(devt[len(devt) // 2] * 1e3, 3),
                          "speedup": round(host[len(host) // 2] / devt[len(devt) // 2], 1),
                          "store_build_s": round(build_s, 2), "store_graphs": args.graphs}), flush=True)


if __name__ == "__main__":
    main()
