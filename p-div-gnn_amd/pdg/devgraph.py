"""Mesh graph construction on the device.

The reference builds every sample's graph on the host before training or
inference (``scripts/benchmark_gnn_fem.py:388-415`` ``convert_mesh_to_graph``, the
"with preprocessing" series; ``datasets.py:247-263``): PyG ``FaceToEdge``
(``convert_utils.py:47-60``), Euclidean edge lengths (``datasets.py:182-188``) and
``compute_periodic_graph`` (``datasets.py:39-119``), then ``.to(device)``.  Here the
mesh goes to HBM as it is (points, triangles) and one ``pdg_mesh_graph`` call
builds the coalesced periodic graph there (csrc/pdg_graph.hip): bitwise the
host restatement's ``edge_index`` and ``edge_attr`` (``tests/test_gpu_devgraph.py``).
"""
from __future__ import annotations

import torch

from .graph import Data
from .lib import lib, stream_handle

SIDE_MAX = 4096


def mesh_graph(points: torch.Tensor, faces: torch.Tensor, periodic: bool = True):
    """Coalesced ``edge_index`` (2, E) int64 and ``edge_attr`` (E,) float32 of a triangle
    mesh on the device: FaceToEdge + lengths [+ periodic connections with zero length].
    ``points`` (N, 2|3) float32 and ``faces`` (F, 3) int64 on a HIP device.  Raises
    ValueError for geometry ``compute_periodic_graph`` cannot pair (one host sync)."""
    if points.device.type != "cuda" or faces.device.type != "cuda":
        raise RuntimeError("mesh_graph needs device tensors (the HIP path has no CPU fallback)")
    pts = points.contiguous().float()
    fcs = faces.contiguous().to(torch.int64)
    n, dim = pts.shape
    nf = fcs.shape[0]
    if dim not in (2, 3) or (nf and fcs.shape[1] != 3):
        raise ValueError("points must be (N, 2|3) and faces (F, 3)")
    dev = pts.device
    nbytes = lib.pdg_mesh_graph_scratch_bytes(n, nf)
    if nbytes < 0:
        raise ValueError("empty mesh")
    scratch = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    cap = 6 * nf + (4 * SIDE_MAX + 4 if periodic else 0)
    ei = torch.empty(2, max(cap, 1), dtype=torch.int64, device=dev)
    ea = torch.empty(max(cap, 1), dtype=torch.float32, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)
    lib.pdg_mesh_graph(n, pts.data_ptr(), dim, nf, fcs.data_ptr() if nf else None, int(periodic), ei[0].data_ptr(),
                       ei[1].data_ptr(), ea.data_ptr(), cap, cnt.data_ptr(), scratch.data_ptr(), nbytes,
                       stream_handle(dev))
    e = int(cnt.item())
    if e < 0:
        raise ValueError("periodic graph: opposite sides must hold the same number of nodes, each corner "
                         f"exactly one node, each side at most {SIDE_MAX} nodes (datasets.py:39-119)")
    return ei[:, :e].contiguous(), ea[:e].clone()


def convert_mesh_to_graph(points: torch.Tensor, faces: torch.Tensor, mean_stress, node_labels: torch.Tensor,
                          periodic: bool = True) -> Data:
    """``benchmark_gnn_fem.py:388-415`` on the device: the graph of one FEM sample, ready for
    ``EncodeProcessDecode`` (pos reduced to (x, y) float32, mean stress broadcast to every
    node, node labels as both ``surfaces_nodes_for_div`` and ``nodes_types``)."""
    edge_index, edge_attr = mesh_graph(points, faces, periodic)
    n = points.shape[0]
    dev = points.device
    labels = node_labels.to(dev).reshape(-1, 1).to(torch.int64)
    ms = torch.as_tensor(mean_stress, dtype=torch.float32, device=dev).reshape(1, 3)
    return Data(edge_index=edge_index, edge_attr=edge_attr, pos=points[:, :2].float().contiguous(),
                face=faces.T.contiguous(), mean_stress=torch.ones(n, 3, device=dev) * ms,
                surfaces_nodes_for_div=labels, nodes_types=labels.clone(), is_periodic=periodic)
