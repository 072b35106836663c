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


def capture_forward(model, device=None):
    """Keep the forward context (the activations on the device) of the model's next forward: the
    returned dict gets ``ctx`` (pdg.engine.FwdCtx) when it runs."""
    eng = model._engine_for(device or dev())
    cap = {}
    fwd = eng.forward

    def keep(*a, **k):
        y, ctx = fwd(*a, **k)
        cap["ctx"] = ctx
        return y, ctx
    eng.forward = keep
    return cap


def gpu_relu_masks(ctx) -> dict:
    """The GPU forward's relu masks (a = relu(h) stored, so a > 0 <=> h > 0) under the keys of
    oracle.epd_oracle.ReluRegion, edges in the caller's edge_index order (the GPU's edge rows are
    dst-sorted: row r is edge plan.perm[r]).  Relus whose output the engine does not keep (the
    edge encoder's layer 1, recomputed in the backward; the last step's unused edge update) are left
    to the oracle's own relu."""
    perm = ctx.plan.perm.long().cpu()
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel())

    def m(t, edge=False):
        if t is None:
            return None
        b = t.detach().cpu() > 0
        return b[inv] if edge else b
    out = {"enc_n.1": m(ctx.a1_ne), "enc_n.2": m(ctx.a2_ne), "enc_e.1": m(ctx.a1_ee, True),
           "enc_e.2": m(ctx.a2_ee, True), "dec.1": m(ctx.a1d)}
    for t, d in enumerate(ctx.per_step):
        out.update({f"s{t}.m.1": m(d["a1m"], True), f"s{t}.m.2": m(d["a2m"], True), f"s{t}.e.1": m(d["a1e"], True),
                    f"s{t}.e.2": m(d["a2e"], True), f"s{t}.n.1": m(d["a1n"]), f"s{t}.n.2": m(d["a2n"])})
    return {k: v for k, v in out.items() if v is not None}


def mask_flips(masks: dict, pre64: dict) -> list:
    """(key, bits flipped against the fp64 pre-activations, largest |h64| among them, rms of h64) per
    relu layer with at least one flipped bit."""
    out = []
    for k, msk in masks.items():
        h = pre64[k].double()
        bad = msk != (h > 0)
        n = int(bad.sum())
        if n:
            out.append((k, n, float(h[bad].abs().max()), float(h.pow(2).mean().sqrt())))
    return out
