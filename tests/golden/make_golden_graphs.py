"""Generate tests/golden/mesh_to_graph.npz from the REFERENCE's mesh -> graph conversion
(``gnn_local_stress/convert_utils.py:47-81``: ``mesh_to_graph`` and ``_quad_face_to_edge``).

Run in the build container only (needs /root/reference, never shipped):

    python tests/golden/make_golden_graphs.py

pyvista, fedoo and torch_geometric are not installed; make_golden.py's stand-ins are registered,
extended with what this path touches, following the libraries' documented semantics:

* ``pyvista``: a mesh object with ``points``, the flat ``faces`` array ([k, i0, .., ik-1, k, ...])
  and ``get_cell(0).type``; ``CellType.QUAD`` / ``CellType.TRIANGLE`` (VTK cell ids 9 / 5);
* ``torch_geometric.utils.to_undirected(edge_index, num_nodes)``: edges and their reverses,
  coalesced (sorted by (row, col), duplicates removed);
* ``torch_geometric.transforms.FaceToEdge(remove_faces)``: edge_index =
  to_undirected(cat([face[:2], face[1:], face[::2]], 1)), face dropped when remove_faces.

The reference's own ``mesh_to_graph`` / ``_quad_face_to_edge`` then run unchanged on a quad grid
with a scrambled node numbering, a triangulated hole plate (pdg.meshgen) and a quad mesh whose cells
are listed clockwise; the fixture holds each case's points, cells and the edge_index the reference
produced.  tests/test_dataset_io.py compares gnn_local_stress.datasets.mesh_to_graph against it
bit for bit.  What it pins: the reference's quad-side selection, the triangle / quad dispatch and
the undirected coalesced edge order; PyG's to_undirected itself only through the stand-in above.
"""
from __future__ import annotations

import enum
import os
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))

import make_golden as mg  # noqa: E402  (stand-ins and paths)


class CellType(enum.IntEnum):
    TRIANGLE = 5
    QUAD = 9


class _Cell:
    def __init__(self, t):
        self.type = t


class StubMesh:
    """The pyvista mesh attributes mesh_to_graph reads."""

    def __init__(self, points: np.ndarray, cells: np.ndarray):
        self.points = np.ascontiguousarray(points, dtype=np.float32)
        k = cells.shape[1]
        self.faces = np.concatenate([np.full((len(cells), 1), k), cells], 1).astype(np.int64).reshape(-1)
        self._type = CellType.QUAD if k == 4 else CellType.TRIANGLE

    def get_cell(self, i):
        return _Cell(self._type)


def to_undirected(edge_index, num_nodes=None, **_):
    n = int(num_nodes) if num_nodes is not None else int(edge_index.max()) + 1
    e = torch.cat([edge_index, edge_index.flip(0)], 1)
    key = torch.unique(e[0] * n + e[1], sorted=True)
    return torch.stack([key // n, key % n])


class FaceToEdge:
    def __init__(self, remove_faces: bool = True):
        self.remove_faces = remove_faces

    def __call__(self, data):
        face = data.face
        ei = torch.cat([face[:2], face[1:], face[::2]], 1)
        data.edge_index = to_undirected(ei, num_nodes=data.num_nodes)
        if self.remove_faces:
            data.face = None
        return data


def install():
    mg.install_stubs()
    pv = sys.modules["pyvista"]
    pv.CellType = CellType
    pyg = sys.modules["torch_geometric"]
    pyg.utils.to_undirected = to_undirected
    pyg.transforms.FaceToEdge = FaceToEdge


def cases():
    rng = np.random.default_rng(4)
    out = {}
    # quad grid 6 x 5 nodes, node numbering scrambled (cells refer to the permuted ids)
    nx, ny = 6, 5
    pts = np.array([[x, y, 0.0] for y in range(ny) for x in range(nx)], np.float32)
    quads = np.array([[y * nx + x, y * nx + x + 1, (y + 1) * nx + x + 1, (y + 1) * nx + x]
                      for y in range(ny - 1) for x in range(nx - 1)], np.int64)
    perm = rng.permutation(nx * ny)
    inv = np.argsort(perm)
    out["quad_scrambled"] = (pts[perm], inv[quads])
    # the same grid, cells listed clockwise
    out["quad_clockwise"] = (pts, quads[:, ::-1].copy())
    # a triangulated hole plate (the datasets' element type)
    from pdg import meshgen
    s = meshgen.hole_plate(9, hole_radius=0.25, seed=2)
    pts3 = np.concatenate([s.pos, np.zeros((s.num_nodes, 1), np.float32)], 1)
    out["tri_hole_plate"] = (pts3, s.faces.astype(np.int64))
    return out


def main():
    install()
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
    sys.path.insert(0, str(mg.REF))
    from gnn_local_stress import convert_utils   # reference module
    rec = {}
    for name, (pts, cells) in cases().items():
        g = convert_utils.mesh_to_graph(StubMesh(pts, cells))
        rec[f"{name}_points"] = pts
        rec[f"{name}_cells"] = cells
        rec[f"{name}_edge_index"] = g.edge_index.numpy().astype(np.int64)
        print(name, pts.shape, cells.shape, g.edge_index.shape)
    np.savez_compressed(HERE / "mesh_to_graph.npz", **rec)


if __name__ == "__main__":
    main()
