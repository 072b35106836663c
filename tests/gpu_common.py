"""Shared helpers for the GPU parity tests (run on the MI355X box)."""
from __future__ import annotations

import numpy as np
import torch

from golden_io import load
from pdg import graph, meshgen


def rel(a, b) -> float:
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def dev():
    return torch.device("cuda:0")


def make_batch(samples, periodic=True, device=None):
    datas = [graph.sample_to_data(s, periodic) for s in samples]
    b = graph.Batch.from_data_list(datas)
    return b.to(device or dev())


def dataset_stats(batch) -> dict:
    """Scalar standardisation constants as datasets.py:283-291 computes them."""
    return {
        "mean_pos": batch.pos.mean(), "std_pos": batch.pos.std(),
        "mean_mean_stress": batch.mean_stress.mean(), "std_mean_stress": batch.mean_stress.std(),
        "mean_local_stress": batch.local_stress.mean(), "std_local_stress": batch.local_stress.std(),
        "mean_edge_weight": batch.edge_attr.mean(), "std_edge_weight": batch.edge_attr.std(),
    }


def golden_batch(name: str):
    """Rebuild the golden case's batch on the GPU from the fixture arrays."""
    g = load(name)
    ptr = g["ptr"]
    datas = []
    ei = g["edge_index"]
    for i in range(len(ptr) - 1):
        s, t = int(ptr[i]), int(ptr[i + 1])
        m = (ei[0] >= s) & (ei[0] < t)
        datas.append(graph.Data(
            edge_index=torch.from_numpy(ei[:, m] - s), edge_attr=torch.from_numpy(g["edge_attr"][m]),
            pos=torch.from_numpy(g["pos"][s:t]), mean_stress=torch.from_numpy(g["mean_stress"][s:t]),
            local_stress=torch.from_numpy(g["local_stress"][s:t]), op_div_matrix=g["op_divs"][i],
            surfaces_nodes_for_div=torch.from_numpy(g["nodes_types"][s:t]),
            nodes_types=torch.from_numpy(g["nodes_types"][s:t])))
    return g, graph.Batch.from_data_list(datas).to(dev())
