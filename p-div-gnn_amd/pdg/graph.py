"""PyG-compatible ``Data`` / ``Batch`` containers without torch_geometric.

PyG is not installed here nor on the GPU box, so the drop-in supplies the
small part of its data API that the hot path's callers use:

* ``Data(**attrs)`` attribute bag with ``.to(device)``, ``num_nodes``,
  ``num_edges`` (``gnn_local_stress/models.py:294-326`` reads ``edge_index``,
  ``pos``, ``mean_stress``, ``nodes_types``, ``edge_attr``);
* ``Batch.from_data_list``: PyG collate semantics — node attributes
  concatenated, ``edge_index`` offset by the running node count, ``batch`` and
  ``ptr`` vectors, ``batch_size`` (``scripts/gnn_train.py:193``), ``batch[i]``
  (``gnn_local_stress/data_utils.py:25-33``);
* a device-side graph plan (``GraphPlan``) attached to the batch: the
  dst-sorted CSR the HIP kernels consume, built once per batch.
"""
from __future__ import annotations

from typing import Any, Iterable

import numpy as np
import torch

from . import meshgen

_NODE_KEYS = ("pos", "mean_stress", "local_stress", "nodes_types", "surfaces_nodes_for_div", "x")
_EDGE_KEYS = ("edge_attr",)


class Data:
    """Minimal attribute container with PyG ``Data`` semantics."""

    def __init__(self, **kwargs: Any) -> None:
        for k, v in kwargs.items():
            setattr(self, k, v)

    def keys(self) -> list[str]:
        return [k for k in self.__dict__ if not k.startswith("_")]

    def __getitem__(self, key: str) -> Any:
        return getattr(self, key)

    def __setitem__(self, key: str, value: Any) -> None:
        setattr(self, key, value)

    def __contains__(self, key: str) -> bool:
        return key in self.keys()

    def __getattr__(self, key: str) -> Any:
        # PyG returns None for missing attributes
        if key.startswith("__"):
            raise AttributeError(key)
        return None

    @property
    def num_nodes(self) -> int:
        for k in ("pos", "mean_stress", "x", "local_stress"):
            v = self.__dict__.get(k)
            if v is not None:
                return int(v.shape[0])
        raise AttributeError("num_nodes")

    @property
    def num_edges(self) -> int:
        ei = self.__dict__.get("edge_index")
        return 0 if ei is None else int(ei.shape[1])

    def to(self, device: Any, non_blocking: bool = False) -> "Data":
        out = self.__class__.__new__(self.__class__)
        for k, v in self.__dict__.items():
            if isinstance(v, torch.Tensor):
                v = v.to(device, non_blocking=non_blocking)
            elif hasattr(v, "to") and not isinstance(v, (type, np.ndarray)) and k.startswith("_plan"):
                v = v.to(device)
            out.__dict__[k] = v
        return out

    def __repr__(self) -> str:
        parts = []
        for k, v in self.__dict__.items():
            if k.startswith("_"):
                continue
            if isinstance(v, torch.Tensor):
                parts.append(f"{k}={list(v.shape)}")
            else:
                parts.append(f"{k}={v!r}"[:40])
        return f"{self.__class__.__name__}({', '.join(parts)})"


def sample_to_data(s: meshgen.MeshSample, periodic: bool = True) -> Data:
    """A ``MeshSample`` in the reference's per-graph ``Data`` layout (``datasets.py:232-281``)."""
    n = s.num_nodes
    op = torch.sparse_coo_tensor(
        torch.from_numpy(np.stack([s.op_div_rows, s.op_div_cols])),
        torch.from_numpy(s.op_div_vals), (n, 2 * n), dtype=torch.float32).coalesce()
    labels = torch.from_numpy(s.node_types).unsqueeze(1)
    return Data(
        edge_index=torch.from_numpy(s.edge_index),
        edge_attr=torch.from_numpy(s.edge_attr),
        pos=torch.from_numpy(s.pos),
        mean_stress=torch.ones(n, 3) * torch.from_numpy(s.mean_stress),
        local_stress=torch.from_numpy(s.local_stress),
        op_div_matrix=op,
        surfaces_nodes_for_div=labels,
        nodes_types=labels,
        is_periodic=periodic,
    )


class Batch(Data):
    """Collated mini-batch (PyG ``Batch`` subset)."""

    @classmethod
    def from_data_list(cls, data_list: Iterable[Data]) -> "Batch":
        data_list = list(data_list)
        b = cls()
        counts = [d.num_nodes for d in data_list]
        ecounts = [d.num_edges for d in data_list]
        ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        eptr = np.concatenate([[0], np.cumsum(ecounts)]).astype(np.int64)
        for k in _NODE_KEYS + _EDGE_KEYS:
            vals = [d.__dict__.get(k) for d in data_list]
            if all(v is not None for v in vals):
                setattr(b, k, torch.cat(vals, 0))
        b.edge_index = torch.cat(
            [d.edge_index + int(ptr[i]) for i, d in enumerate(data_list)], 1)
        b.batch = torch.repeat_interleave(torch.arange(len(data_list)), torch.tensor(counts))
        b.ptr = torch.from_numpy(ptr)
        b._eptr = torch.from_numpy(eptr)
        b._data_list = data_list
        # collated divergence operator: global rows, graph-local columns
        if all(d.__dict__.get("op_div_matrix") is not None for d in data_list):
            rows, cols, vals = [], [], []
            for i, d in enumerate(data_list):
                op = d.op_div_matrix.coalesce()
                idx = op.indices()
                rows.append(idx[0] + int(ptr[i]))
                cols.append(idx[1])
                vals.append(op.values())
            b.op_div_rows = torch.cat(rows)
            b.op_div_cols = torch.cat(cols)
            b.op_div_vals = torch.cat(vals)
        return b

    @property
    def batch_size(self) -> int:
        return int(self.ptr.numel() - 1)

    num_graphs = batch_size

    def __len__(self) -> int:
        return self.batch_size

    def __getitem__(self, idx: Any) -> Any:
        if isinstance(idx, str):
            return getattr(self, idx)
        # PyG slices the batch's *current* attributes (gnn_train.py:167 rewrites
        # local_stress before slicing), so do the same.
        n0, n1 = int(self.ptr[idx]), int(self.ptr[idx + 1])
        e0, e1 = int(self._eptr[idx]), int(self._eptr[idx + 1])
        out = Data()
        for k in _NODE_KEYS:
            v = self.__dict__.get(k)
            if v is not None:
                setattr(out, k, v[n0:n1])
        for k in _EDGE_KEYS:
            v = self.__dict__.get(k)
            if v is not None:
                setattr(out, k, v[e0:e1])
        out.edge_index = self.edge_index[:, e0:e1] - n0
        op = self._data_list[idx].__dict__.get("op_div_matrix")
        if op is not None:
            out.op_div_matrix = op.to(self.edge_index.device)
        return out

    def to_data_list(self) -> list[Data]:
        return [self[i] for i in range(len(self))]

    def to(self, device: Any, non_blocking: bool = False) -> "Batch":
        out = super().to(device, non_blocking=non_blocking)
        out._data_list = self._data_list
        return out


class DataLoader(torch.utils.data.DataLoader):
    """PyG ``DataLoader`` (gnn_train.py:387-394, gnn_inference.py:103-107): like PyG's, a
    ``torch.utils.data.DataLoader`` whose collate is ``Batch.from_data_list``.  Being the torch
    loader itself, it draws from torch's global RNG exactly as the reference's loaders do (one
    base seed per iterator, plus the RandomSampler's seed when shuffling), so a seeded run visits
    the graphs in the reference's order.  As in PyG, the collate is fixed: a ``collate_fn`` is
    refused (TypeError) rather than silently replaced."""

    def __init__(self, dataset, batch_size: int = 1, shuffle: bool = False,
                 generator: torch.Generator | None = None, **kwargs: Any) -> None:
        if "collate_fn" in kwargs:
            raise TypeError("pdg.graph.DataLoader collates with Batch.from_data_list (as PyG's DataLoader); "
                            "it takes no collate_fn")
        super().__init__(dataset, batch_size=batch_size, shuffle=shuffle, generator=generator,
                         collate_fn=Batch.from_data_list, **kwargs)


def index_loader(num_graphs: int, batch_size: int, shuffle: bool,
                 generator: torch.Generator | None = None) -> torch.utils.data.DataLoader:
    """The graph-index lists a PyG ``DataLoader(dataset, batch_size, shuffle)`` over ``num_graphs``
    graphs would collate, in the same order and with the same global-RNG draws (a torch
    DataLoader over ``range(num_graphs)`` with a list collate).  Device-resident stores
    (``pdg.collate.DeviceGraphStore``) collate these indices on the GPU."""
    return torch.utils.data.DataLoader(range(num_graphs), batch_size=batch_size, shuffle=shuffle,
                                       generator=generator, collate_fn=list)
