"""Preprocessing timing (the reference's "with preprocessing" series,
benchmark_gnn_fem.py:388-415): graph build of one mesh on the host (the restatement of
FaceToEdge + lengths + compute_periodic_graph + coalesce, numpy/torch CPU) vs on the device
(pdg_mesh_graph, points and triangles already in HBM).  Prints one JSON line per mesh."""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "p-div-gnn_amd")]

from pdg import meshgen  # noqa: E402
from pdg.devgraph import mesh_graph  # noqa: E402


def host(pos, faces):
    n = len(pos)
    ei = meshgen.faces_to_edges(faces, n)
    ea = meshgen.edge_lengths(pos, ei)
    pr, pc = meshgen.periodic_pairs(pos)
    return meshgen.coalesce(np.concatenate([ei, np.stack([pr, pc])], 1),
                            np.concatenate([ea, np.zeros(len(pr), np.float32)]), n)


for n in (71, 160, 317):
    s = meshgen.hole_plate(n=n, hole_radius=0.0, periodic=True, seed=1)
    t0 = time.perf_counter()
    for _ in range(3):
        host(s.pos, s.faces)
    th = (time.perf_counter() - t0) / 3
    p, f = torch.from_numpy(s.pos).cuda(), torch.from_numpy(s.faces).cuda()
    for _ in range(3):
        mesh_graph(p, f)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 20
    for _ in range(reps):
        mesh_graph(p, f)
    torch.cuda.synchronize()
    td = (time.perf_counter() - t0) / reps
    print(json.dumps({"mesh": f"{n}x{n}", "nodes": s.num_nodes, "edges": s.num_edges,
                      "host_ms": round(th * 1e3, 3), "device_ms": round(td * 1e3, 3),
                      "device_note": "includes the one edge-count readback (host sync) per call"}))
