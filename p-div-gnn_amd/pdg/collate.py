"""Device-side minibatch assembly from an HBM-resident dataset.

The reference collates every minibatch on the host (``gnn_train.py:387-394``:
PyG ``DataLoader`` -> ``Batch.from_data_list``), copies it to the GPU and, in
this build, derives the dst-sorted graph plan from it.  With 288 GB of HBM the
whole dataset fits on the device, so :class:`DeviceGraphStore` keeps every
graph resident together with its own plan pieces (graph-local dst-sorted CSR,
source grouping, divergence CSR / CSR^T) and assembles a batch with ONE HIP
launch (``pdg_collate``): each batched array is a concatenation of per-graph
segments, index arrays shifted by the graph's node / edge / nonzero offset.
No sort is needed: graphs occupy disjoint increasing node ranges, so the
batch's stable (dst, src) order is the concatenation of the graphs' orders.

The result is attribute-for-attribute the ``Batch.from_data_list(...).to(dev)``
of the same graphs with the ``GraphPlan`` that ``plan_for`` would build
(tested bitwise in ``tests/test_gpu_collate.py``).
"""
from __future__ import annotations

from typing import Sequence

import numpy as np
import torch

from .graph import Batch, Data
from .lib import lib, stream_handle
from .plan import GraphPlan

F32, B32, B64 = 0, 1, 2
_JOB = np.dtype([("src", "<u8"), ("dst", "<u8"), ("count", "<i8"), ("add", "<i8"), ("kind", "<i4"),
                 ("pad", "<i4")])
assert _JOB.itemsize == 40

# per-graph arrays kept resident: name -> (source, per-node/edge width, kind)
_NODE_F32 = (("pos", 2), ("mean_stress", 3), ("local_stress", 3))
_NODE_I64 = ("nodes_types", "surfaces_nodes_for_div")


class DeviceGraphStore:
    """A dataset of ``Data`` graphs resident in HBM; ``batch(indices)`` collates on device."""

    def __init__(self, datas: Sequence[Data], device) -> None:
        self.device = torch.device(device)
        self.datas = list(datas)
        dev = self.device
        G = len(self.datas)
        self.n = np.array([d.num_nodes for d in self.datas], dtype=np.int64)
        self.e = np.array([d.num_edges for d in self.datas], dtype=np.int64)
        plans = []
        for d in self.datas:
            op = d.__dict__.get("op_div_matrix")
            rows = cols = vals = None
            if op is not None:
                op = op.coalesce()
                rows, cols = op.indices()[0], op.indices()[1]
                vals = op.values()
            plans.append(GraphPlan(d.edge_index.to(dev), d.num_nodes, None, rows, cols, vals))
        self.has_div = all(p.has_div for p in plans)
        self.nnz = np.array([p.a_col.numel() if self.has_div else 0 for p in plans], dtype=np.int64)
        self.nnzt = np.array([p.at_row.numel() if self.has_div else 0 for p in plans], dtype=np.int64)

        def flat(parts, dtype):
            return torch.cat([p.reshape(-1).to(dev, dtype) for p in parts]).contiguous()

        def starts(counts):
            return np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)

        self.off_n, self.off_e = starts(self.n), starts(self.e)
        self.off_nnz, self.off_nnzt = starts(self.nnz), starts(self.nnzt)
        self.off_n1 = starts(self.n + 1)
        a = {}
        for k, w in _NODE_F32:
            a[k] = flat([d.__dict__[k] for d in self.datas], torch.float32)
        for k in _NODE_I64:
            a[k] = flat([d.__dict__[k] for d in self.datas], torch.int64)
        a["edge_attr"] = flat([d.edge_attr for d in self.datas], torch.float32)
        a["ei0"] = flat([d.edge_index[0] for d in self.datas], torch.int64)
        a["ei1"] = flat([d.edge_index[1] for d in self.datas], torch.int64)
        for k in ("perm", "src", "dst", "perm_src"):
            a[k] = flat([getattr(p, k) for p in plans], torch.int32)
        for k in ("rowptr_dst", "rowptr_src"):
            a[k] = flat([getattr(p, k) for p in plans], torch.int32)
        if self.has_div:
            for k in ("a_rowptr", "at_rowptr"):
                a[k] = flat([getattr(p, k) for p in plans], torch.int32)
            for k in ("a_col", "at_row", "at_comp"):
                a[k] = flat([getattr(p, k) for p in plans], torch.int32)
            for k in ("a_val", "at_val"):
                a[k] = flat([getattr(p, k) for p in plans], torch.float32)
        self.arrays = a
        self._zero32 = torch.zeros(max(int(self.n.max()), 1) + 1, dtype=torch.int32, device=dev)
        self._zero64 = torch.zeros(max(int(self.n.max()), 1) + 1, dtype=torch.int64, device=dev)
        self.num_graphs = G

    # ------------------------------------------------------------------ batch assembly
    def batch(self, indices: Sequence[int]) -> Batch:
        idx = [int(i) for i in indices]
        if not idx:
            raise ValueError("empty batch")
        dev = self.device
        a = self.arrays
        n, e = self.n[idx], self.e[idx]
        bn = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)     # batch node offsets (= ptr)
        be = np.concatenate([[0], np.cumsum(e)]).astype(np.int64)
        N, E = int(bn[-1]), int(be[-1])
        f32 = dict(dtype=torch.float32, device=dev)
        i32 = dict(dtype=torch.int32, device=dev)
        i64 = dict(dtype=torch.int64, device=dev)
        jobs = []
        max_count = [1]

        def job(src: torch.Tensor, src_off: int, dst: torch.Tensor, dst_off: int, count: int, add: int, kind: int):
            if count <= 0:
                return
            es = src.element_size()
            jobs.append((src.data_ptr() + es * src_off, dst.data_ptr() + es * dst_off, count, add, kind, 0))
            max_count[0] = max(max_count[0], count)

        out = Batch()
        for k, w in _NODE_F32:
            t = torch.empty(N, w, **f32)
            for j, g in enumerate(idx):
                job(a[k], w * int(self.off_n[g]), t, w * int(bn[j]), w * int(n[j]), 0, F32)
            setattr(out, k, t)
        for k in _NODE_I64:
            t = torch.empty(N, 1, **i64)
            for j, g in enumerate(idx):
                job(a[k], int(self.off_n[g]), t, int(bn[j]), int(n[j]), 0, B64)
            setattr(out, k, t)
        ea = torch.empty(E, **f32)
        ei = torch.empty(2, E, **i64)
        bvec = torch.empty(N, **i64)
        for j, g in enumerate(idx):
            job(a["edge_attr"], int(self.off_e[g]), ea, int(be[j]), int(e[j]), 0, F32)
            job(a["ei0"], int(self.off_e[g]), ei[0], int(be[j]), int(e[j]), int(bn[j]), B64)
            job(a["ei1"], int(self.off_e[g]), ei[1], int(be[j]), int(e[j]), int(bn[j]), B64)
            job(self._zero64, 0, bvec, int(bn[j]), int(n[j]), j, B64)
        out.edge_attr, out.edge_index, out.batch = ea, ei, bvec
        ptr64, eptr64 = torch.empty(len(idx) + 1, **i64), torch.empty(len(idx) + 1, **i64)
        ptr32 = torch.empty(len(idx) + 1, **i32)
        for j in range(len(idx) + 1):
            job(self._zero64, 0, ptr64, j, 1, int(bn[j]), B64)
            job(self._zero64, 0, eptr64, j, 1, int(be[j]), B64)
            job(self._zero32, 0, ptr32, j, 1, int(bn[j]), B32)
        out.ptr, out._eptr = ptr64, eptr64

        # plan: graph-local pieces shifted into the batch
        plan = GraphPlan.__new__(GraphPlan)
        plan.n_nodes, plan.n_edges, plan.n_graphs, plan.ptr = N, E, len(idx), ptr32
        for k, add_by in (("perm", "e"), ("src", "n"), ("dst", "n"), ("perm_src", "e")):
            t = torch.empty(E, **i32)
            for j, g in enumerate(idx):
                job(a[k], int(self.off_e[g]), t, int(be[j]), int(e[j]), int(be[j] if add_by == "e" else bn[j]), B32)
            setattr(plan, k, t)

        def rowptr(key: str, add: np.ndarray, total: int) -> torch.Tensor:
            t = torch.empty(N + 1, **i32)
            for j, g in enumerate(idx):
                job(a[key], int(self.off_n1[g]), t, int(bn[j]), int(n[j]), int(add[j]), B32)
            job(self._zero32, 0, t, N, 1, total, B32)
            return t

        plan.rowptr_dst = rowptr("rowptr_dst", be, E)
        plan.rowptr_src = rowptr("rowptr_src", be, E)
        plan.has_div = self.has_div
        if self.has_div:
            nz, nzt = self.nnz[idx], self.nnzt[idx]
            bz = np.concatenate([[0], np.cumsum(nz)]).astype(np.int64)
            bzt = np.concatenate([[0], np.cumsum(nzt)]).astype(np.int64)
            plan.a_rowptr = rowptr("a_rowptr", bz, int(bz[-1]))
            plan.at_rowptr = rowptr("at_rowptr", bzt, int(bzt[-1]))
            for k, cnt, offs, boff, add_rows, kind in (
                    ("a_col", nz, self.off_nnz, bz, False, B32), ("a_val", nz, self.off_nnz, bz, False, F32),
                    ("at_row", nzt, self.off_nnzt, bzt, True, B32), ("at_comp", nzt, self.off_nnzt, bzt, False, B32),
                    ("at_val", nzt, self.off_nnzt, bzt, False, F32)):
                t = torch.empty(int(boff[-1]), **(f32 if kind == F32 else i32))
                for j, g in enumerate(idx):
                    job(a[k], int(offs[g]), t, int(boff[j]), int(cnt[j]), int(bn[j]) if add_rows else 0, kind)
                setattr(plan, k, t)

        table = torch.from_numpy(np.array(jobs, dtype=_JOB).view(np.uint8)).to(dev, non_blocking=True)
        lib.pdg_collate(table.data_ptr(), len(jobs), max_count[0], stream_handle(dev))
        out._collate_table = table           # keep the job table alive until the launch has run
        out._data_list = [self.datas[g] for g in idx]
        out.__dict__["_plan_cache"] = ((ei.data_ptr(), tuple(ei.shape), ei.device), plan)
        return out

    def batches(self, batch_size: int, shuffle: bool = False, generator: torch.Generator | None = None):
        """Iterate over minibatches like PyG's DataLoader(batch_size, shuffle) (gnn_train.py:387-394):
        the same order and the same global-RNG draws (pdg.graph.index_loader)."""
        from .graph import index_loader
        for idx in index_loader(self.num_graphs, batch_size, shuffle, generator):
            yield self.batch(idx)
