"""Device graph plan: the CSR view of a (batched) graph that the HIP kernels consume.

Built once per batch from the reference's inputs (``edge_index`` coalesced,
i.e. sorted by (src, dst) — ``datasets.py:119``; per-graph node offsets
``ptr``; the divergence operators) and cached on the batch object:

* dst-sorted edge order (stable, so within a destination the sources stay
  ascending = the order PyG's ``scatter_add_`` accumulates in);
* ``rowptr_dst`` (N+1) over that order, ``src``/``dst`` of each sorted edge,
  ``perm`` = original edge id of each sorted edge (for ``edge_attr``);
* ``perm_src``/``rowptr_src``: the sorted edges grouped by source, for the
  backward of the ``x[src]`` gathers;
* divergence operator A in CSR over global rows with graph-local columns, and
  A^T grouped by global node (``at_*``) for the backward SpMV.

Edge order is internal: the model only returns node outputs
(``models.py:322-326``), so the reordering is invisible to callers.
"""
from __future__ import annotations

import torch


def _rowptr(keys: torch.Tensor, n: int) -> torch.Tensor:
    counts = torch.bincount(keys, minlength=n)
    rp = torch.zeros(n + 1, dtype=torch.int64, device=keys.device)
    rp[1:] = torch.cumsum(counts, 0)
    return rp.to(torch.int32)


class GraphPlan:
    def __init__(self, edge_index: torch.Tensor, num_nodes: int, ptr: torch.Tensor | None = None,
                 op_rows: torch.Tensor | None = None, op_cols: torch.Tensor | None = None,
                 op_vals: torch.Tensor | None = None) -> None:
        dev = edge_index.device
        n = int(num_nodes)
        self.n_nodes = n
        self.n_edges = int(edge_index.shape[1])
        src = edge_index[0].long()
        dst = edge_index[1].long()
        if self.n_edges:
            assert int(src.max()) < n and int(dst.max()) < n and int(src.min()) >= 0 and int(dst.min()) >= 0, \
                "edge_index out of range"
        key = dst * n + src
        order = torch.sort(key, stable=True).indices
        self.perm = order.to(torch.int32)
        self.src = src[order].to(torch.int32).contiguous()
        self.dst = dst[order].to(torch.int32).contiguous()
        self.rowptr_dst = _rowptr(dst, n)
        key2 = self.src.long() * n + self.dst.long()
        self.perm_src = torch.sort(key2, stable=True).indices.to(torch.int32).contiguous()
        self.rowptr_src = _rowptr(src, n)
        if ptr is None:
            ptr = torch.tensor([0, n], dtype=torch.int64, device=dev)
        self.ptr = ptr.to(dev).to(torch.int32).contiguous()
        self.n_graphs = int(self.ptr.numel() - 1)
        self.has_div = op_rows is not None
        if self.has_div:
            self._build_div(op_rows.to(dev).long(), op_cols.to(dev).long(), op_vals.to(dev).float())

    def _build_div(self, rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor) -> None:
        n = self.n_nodes
        ptr = self.ptr.long()
        g = torch.searchsorted(ptr, rows, right=True) - 1
        off = ptr[g]
        ng = ptr[g + 1] - off
        keep = cols < 2 * ng          # reference slices [:, :2N_i] (gnn_train.py:74)
        rows, cols, vals, off, ng = rows[keep], cols[keep], vals[keep], off[keep], ng[keep]
        order = torch.sort(rows, stable=True).indices
        self.a_rowptr = _rowptr(rows, n)
        self.a_col = cols[order].to(torch.int32).contiguous()
        self.a_val = vals[order].contiguous()
        node = off + torch.where(cols < ng, cols, cols - ng)
        comp = (cols >= ng).to(torch.int32)
        order_t = torch.sort(node, stable=True).indices
        self.at_rowptr = _rowptr(node, n)
        self.at_row = rows[order_t].to(torch.int32).contiguous()
        self.at_comp = comp[order_t].contiguous()
        self.at_val = vals[order_t].contiguous()


def plan_for(data) -> GraphPlan:
    """Return (and cache on ``data``) the plan of a Data/Batch-like object."""
    plan = data.__dict__.get("_plan_cache") if hasattr(data, "__dict__") else None
    ei = data.edge_index
    key = (ei.data_ptr(), tuple(ei.shape), ei.device)
    if plan is not None and plan[0] == key:
        return plan[1]
    ptr = data.__dict__.get("ptr") if hasattr(data, "__dict__") else None
    rows = data.__dict__.get("op_div_rows") if hasattr(data, "__dict__") else None
    p = GraphPlan(ei, data.num_nodes if hasattr(data, "num_nodes") else data.pos.shape[0], ptr,
                  rows, data.__dict__.get("op_div_cols") if rows is not None else None,
                  data.__dict__.get("op_div_vals") if rows is not None else None)
    try:
        data.__dict__["_plan_cache"] = (key, p)
    except Exception:
        pass
    return p
