"""``gnn_local_stress.datasets`` mirror: ``NodeType`` (reference datasets.py:33-36), the
graph construction of the input format and ``MeshStressFieldDatasetInMemory``
(datasets.py:232-311) reading the reference's on-disk schema without pyvista or
PyG:

* ``dataset.csv`` with ``mesh_filename`` / ``data_filename`` columns
  (``scripts/generate_dataset.py:770``);
* meshes: legacy VTK polygon surfaces (``pv_mesh.save``, generate_dataset.py:556-584),
  parsed by :mod:`gnn_local_stress.vtk_io`;
* fields: ``.npz`` with ``stress_field``, ``mean_stress``, ``op_div_matrix_*``,
  ``node_labels`` (generate_dataset.py:586-598), loaded with ``allow_pickle=False``.

Graph construction follows datasets.py:247-281 step by step: triangles ->
undirected coalesced edges (PyG ``FaceToEdge``), edge lengths from the stored
3-D points, periodic connections with zero length (``compute_periodic_graph``,
datasets.py:39-119), ``pos[:, :2]`` in float32, mean stress broadcast to every
node, the sparse divergence operator, node labels as both
``surfaces_nodes_for_div`` and ``nodes_types``.
"""
from __future__ import annotations

from enum import IntEnum
from pathlib import Path

import numpy as np
import torch

from pdg import meshgen
from pdg.graph import Batch, Data

from .vtk_io import read_legacy_vtk


class NodeType(IntEnum):
    INTERNAL_BOUNDARY = -1
    INTERNAL = 0
    EXTERNAL_BOUNDARY = 1


def mesh_to_graph(points: np.ndarray, faces: np.ndarray) -> Data:
    """convert_utils.py:47-60: pos = points, undirected coalesced edges of the cells -- PyG
    ``FaceToEdge`` for triangles, ``_quad_face_to_edge`` (:63-81) for quads (the reference decides by
    the first cell's type; the VTK reader refuses mixed cell sizes)."""
    n = len(points)
    if faces.shape[1] == 3:
        ei = meshgen.faces_to_edges(faces, n)
    elif faces.shape[1] == 4:
        ei = meshgen.quad_faces_to_edges(faces, n)
    else:
        raise ValueError(f"cells with {faces.shape[1]} vertices: only triangle and quad meshes are supported")
    return Data(pos=torch.from_numpy(np.ascontiguousarray(points)),
                edge_index=torch.from_numpy(ei),
                face=torch.from_numpy(np.ascontiguousarray(faces.T)))


def compute_node_distances_as_edge_weights(graph: Data) -> torch.Tensor:
    """datasets.py:182-188."""
    d = graph.pos[graph.edge_index[0]] - graph.pos[graph.edge_index[1]]
    return torch.linalg.vector_norm(d, dim=1)


def compute_periodic_graph(graph: Data) -> Data:
    """datasets.py:39-119: opposite-side and corner connections with zero edge weight, coalesced."""
    pos2 = graph.pos[:, :-1].numpy() if graph.pos.shape[1] == 3 else graph.pos.numpy()
    rows, cols = meshgen.periodic_pairs(pos2)
    ei = np.concatenate([graph.edge_index.numpy(), np.stack([rows, cols])], 1)
    ea = np.concatenate([graph.edge_attr.numpy().astype(np.float32), np.zeros(len(rows), np.float32)])
    ei, ea = meshgen.coalesce(ei, ea, graph.num_nodes)
    return Data(edge_index=torch.from_numpy(ei), pos=graph.pos, edge_attr=torch.from_numpy(ea), face=graph.face,
                org_edge_index=graph.edge_index)


def init_op_div_matrix(mesh_data) -> torch.Tensor:
    """datasets.py:191-213."""
    idx = torch.vstack((torch.from_numpy(np.asarray(mesh_data["op_div_matrix_row_indices"], np.int64)),
                        torch.from_numpy(np.asarray(mesh_data["op_div_matrix_col_indices"], np.int64))))
    vals = torch.from_numpy(np.asarray(mesh_data["op_div_matrix_data"], np.float32))
    shape = torch.Size([int(x) for x in mesh_data["op_div_matrix_shape"]])
    return torch.sparse_coo_tensor(idx, vals, shape, dtype=torch.float32).coalesce()


def von_mises_stress(sx, sy, sxy):
    """datasets.py:216-229."""
    return np.sqrt(0.5 * ((sx - sy) ** 2 + sx ** 2 + sy ** 2 + 6 * sxy ** 2))


def load_sample(mesh_filename: str | Path, data_filename: str | Path, periodic_graph: bool = True,
                device=None) -> Data:
    """One dataset sample exactly as datasets.py:247-281 builds it.  With a HIP ``device`` the
    graph (FaceToEdge, lengths, periodic connections, coalesce) is built there by
    ``pdg.devgraph.mesh_graph`` (the same edges, and bitwise the same lengths
    for single-precision VTK points -- double-precision points are rounded to fp32 first, where
    the reference takes the lengths in fp64 and rounds them: within 1 ulp) and the sample's
    tensors stay on the host until the caller moves them."""
    points, faces = read_legacy_vtk(mesh_filename)
    # the device graph builder (pdg_mesh_graph) takes triangles; quad meshes (convert_utils.py:63-81,
    # not used by the reference's datasets) are built by the host restatement below on any device
    if device is not None and torch.device(device).type == "cuda" and faces.shape[1] == 3:
        from pdg.devgraph import mesh_graph
        ei, ea = mesh_graph(torch.from_numpy(np.ascontiguousarray(points, np.float32)).to(device),
                            torch.from_numpy(np.ascontiguousarray(faces, np.int64)).to(device), periodic_graph)
        graph = Data(pos=torch.from_numpy(np.ascontiguousarray(points)), edge_index=ei.cpu(), edge_attr=ea.cpu(),
                     face=torch.from_numpy(np.ascontiguousarray(faces.T)))
    else:
        graph = mesh_to_graph(points, faces)
        graph.edge_attr = compute_node_distances_as_edge_weights(graph).float()
        if periodic_graph:
            graph = compute_periodic_graph(graph)
    graph.is_periodic = periodic_graph
    with np.load(data_filename, allow_pickle=False) as mesh_data:
        stress_field = torch.from_numpy(mesh_data["stress_field"]).float()
        msx, msy, msxy = (float(v) for v in mesh_data["mean_stress"])
        graph.pos = graph.pos[:, :2].float()
        graph.mean_stress = torch.ones(stress_field.shape) * torch.tensor((msx, msy, msxy), dtype=torch.float32)
        graph.local_stress = stress_field
        graph.op_div_matrix = init_op_div_matrix(mesh_data)
        graph.von_mises = von_mises_stress(msx, msy, msxy)
        graph.surfaces_nodes_for_div = torch.from_numpy(np.asarray(mesh_data["node_labels"], np.int64)).unsqueeze(1)
    graph.nodes_types = graph.surfaces_nodes_for_div
    return graph


class MeshStressFieldDatasetInMemory:
    """datasets.py:232-311 without PyG: ``len``, indexing, the eight scalar
    standardisation constants of the whole set (:283-291) and the collated data."""

    def __init__(self, dataframe, transform=None, periodic_graph: bool = True, device=None) -> None:
        self.dataframe = dataframe
        self.transform = transform
        self.graphs = [load_sample(m, d, periodic_graph, device)
                       for m, d in zip(dataframe["mesh_filename"], dataframe["data_filename"])]
        data = Batch.from_data_list(self.graphs)
        self.mean_pos = data.pos.mean()
        self.std_pos = data.pos.std()
        self.mean_mean_stress = data.mean_stress.mean()
        self.std_mean_stress = data.mean_stress.std()
        self.mean_local_stress = data.local_stress.mean()
        self.std_local_stress = data.local_stress.std()
        self.mean_edge_weight = data.edge_attr.mean()
        self.std_edge_weight = data.edge_attr.std()
        self.data = data

    def __len__(self) -> int:
        return len(self.graphs)

    def __getitem__(self, i: int) -> Data:
        g = self.graphs[i]
        return self.transform(g) if self.transform is not None else g

    def stats(self) -> dict:
        """The constructor keywords of EncodeProcessDecode (gnn_train.py:397-411)."""
        return {k: getattr(self, k) for k in ("mean_pos", "std_pos", "mean_mean_stress", "std_mean_stress",
                                              "mean_local_stress", "std_local_stress", "mean_edge_weight",
                                              "std_edge_weight")}
