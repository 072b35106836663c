"""Seeded synthetic periodic hole-plate meshes in the reference's graph format.

The reference builds its graphs from gmsh/fedoo FEM datasets that cannot be
produced here (fedoo, gmsh, pyvista are absent).  This module generates meshes
with the same *input format* the hot path consumes:

* triangulated 2D plate on [0, L]^2 with an optional circular hole,
  interior-only jitter so that opposite boundary nodes stay periodic;
* ``edge_index``: FaceToEdge + to_undirected (both directions, coalesced),
  as ``gnn_local_stress/convert_utils.py:47-60``;
* ``edge_attr``: Euclidean edge length (``datasets.py:182-188``);
* periodic edges left<->right, bottom<->top (sorted along the side) and the two
  diagonal corner pairs with ``edge_attr = 0``, then coalesced
  (``datasets.py:39-119``);
* ``node_types`` in {-1 internal boundary (hole), 0 internal, 1 external}
  (``datasets.py:33-36``, ``:133-179``);
* ``op_div``: a P1 nodal divergence operator A (N x 2N, local columns: first N
  are d/dx, next N are d/dy), the role of ``op_div_matrix``
  (``datasets.py:191-213``);  A is an *input* of the loss, so its exact FEM
  weights do not matter for parity;
* a smooth synthetic target ``local_stress`` around a random mean stress;  with
  ``strain_range`` (BASELINE config 4, the hyperelastic dataset: imposed mean strains in
  ±0.15, ``scripts/generate_dataset_hyperelast.py:631``) the mean stress comes from a
  stiffening (non-linear) response to a random mean strain and the concentration field
  grows with the strain.  Targets only enter the loss, never the cost of a step.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

NODE_INTERNAL_BOUNDARY = -1
NODE_INTERNAL = 0
NODE_EXTERNAL_BOUNDARY = 1


@dataclass
class MeshSample:
    pos: np.ndarray            # (N, 2) float32
    faces: np.ndarray          # (F, 3) int64
    node_types: np.ndarray     # (N,) int64
    edge_index: np.ndarray     # (2, E) int64, coalesced (sorted by (src, dst))
    edge_attr: np.ndarray      # (E,) float32
    op_div_rows: np.ndarray    # (nnz,) int64
    op_div_cols: np.ndarray    # (nnz,) int64
    op_div_vals: np.ndarray    # (nnz,) float32
    mean_stress: np.ndarray    # (3,) float32
    local_stress: np.ndarray   # (N, 3) float32

    @property
    def num_nodes(self) -> int:
        return int(self.pos.shape[0])

    @property
    def num_edges(self) -> int:
        return int(self.edge_index.shape[1])


def _grid_triangles(n: int) -> np.ndarray:
    i, j = np.meshgrid(np.arange(n - 1), np.arange(n - 1), indexing="xy")
    i = i.ravel()
    j = j.ravel()
    p00 = j * n + i
    p10 = p00 + 1
    p01 = p00 + n
    p11 = p01 + 1
    even = ((i + j) % 2) == 0
    t1 = np.where(even[:, None], np.stack([p00, p10, p11], 1), np.stack([p00, p10, p01], 1))
    t2 = np.where(even[:, None], np.stack([p00, p11, p01], 1), np.stack([p10, p11, p01], 1))
    return np.concatenate([t1, t2], 0).astype(np.int64)


def coalesce(edge_index: np.ndarray, edge_attr: np.ndarray | None, num_nodes: int):
    """Sort by (row, col) and sum-reduce duplicates (PyG ``coalesce`` semantics)."""
    key = edge_index[0].astype(np.int64) * num_nodes + edge_index[1]
    order = np.argsort(key, kind="stable")
    key = key[order]
    uniq, first = np.unique(key, return_index=True)
    ei = np.stack([uniq // num_nodes, uniq % num_nodes]).astype(np.int64)
    if edge_attr is None:
        return ei, None
    ea = edge_attr[order]
    # sum duplicates in sorted order
    ea_sum = np.add.reduceat(ea.astype(np.float32), first) if len(ea) else ea
    return ei, ea_sum.astype(np.float32)


def faces_to_edges(faces: np.ndarray, num_nodes: int) -> np.ndarray:
    e = np.concatenate([faces[:, [0, 1]], faces[:, [1, 2]], faces[:, [0, 2]]], 0).T
    e = np.concatenate([e, e[::-1]], 1)
    ei, _ = coalesce(e, None, num_nodes)
    return ei


def quad_faces_to_edges(faces: np.ndarray, num_nodes: int) -> np.ndarray:
    """convert_utils.py:63-81 (``_quad_face_to_edge``): the four sides (f0,f1), (f1,f2), (f2,f3),
    (f0,f3) of every quad, made undirected and coalesced (PyG ``to_undirected``)."""
    e = np.concatenate([faces[:, [0, 1]], faces[:, [1, 2]], faces[:, [2, 3]], faces[:, [0, 3]]], 0).T
    e = np.concatenate([e, e[::-1]], 1)
    ei, _ = coalesce(e, None, num_nodes)
    return ei


def edge_lengths(pos: np.ndarray, edge_index: np.ndarray) -> np.ndarray:
    """Euclidean edge length in float32, computed as datasets.py:182-188 does."""
    import torch
    p = torch.from_numpy(np.ascontiguousarray(pos, dtype=np.float32))
    ei = torch.from_numpy(edge_index)
    return torch.linalg.vector_norm(p[ei[0]] - p[ei[1]], dim=1).numpy().astype(np.float32)


def periodic_pairs(pos: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Periodic connections in the order ``datasets.py:39-119`` appends them."""
    min_x, min_y = pos.min(0)
    max_x, max_y = pos.max(0)
    idx = np.arange(len(pos))

    def side(mask):
        m = np.where(mask)[0]
        # np.lexsort with keys (x, y): primary key is y, then x
        return m[np.lexsort((pos[m, 0], pos[m, 1]))]

    left = side(pos[:, 0] == min_x)
    right = side(pos[:, 0] == max_x)
    upper = side(pos[:, 1] == max_y)
    lower = side(pos[:, 1] == min_y)

    def corner(x, y):
        c = idx[(pos[:, 0] == x) & (pos[:, 1] == y)]
        assert len(c) == 1
        return c[0]

    corners = np.array([corner(min_x, min_y), corner(min_x, max_y),
                        corner(max_x, min_y), corner(max_x, max_y)])
    assert len(left) == len(right) and len(upper) == len(lower)
    rows = np.concatenate([left, right, lower, upper, corners])
    cols = np.concatenate([right, left, upper, lower, corners[::-1]])
    return rows.astype(np.int64), cols.astype(np.int64)


def p1_divergence_operator(pos: np.ndarray, faces: np.ndarray):
    """Area-averaged P1 divergence operator A = [Dx | Dy] of shape (N, 2N)."""
    n = len(pos)
    p = pos.astype(np.float64)
    a, b, c = faces[:, 0], faces[:, 1], faces[:, 2]
    xa, ya = p[a, 0], p[a, 1]
    xb, yb = p[b, 0], p[b, 1]
    xc, yc = p[c, 0], p[c, 1]
    det = (xb - xa) * (yc - ya) - (xc - xa) * (yb - ya)  # 2 * signed area
    area = 0.5 * np.abs(det)
    gx = np.stack([yb - yc, yc - ya, ya - yb], 1) / det[:, None]
    gy = np.stack([xc - xb, xa - xc, xb - xa], 1) / det[:, None]
    rows, cols, vals = [], [], []
    wsum = np.zeros(n)
    np.add.at(wsum, faces.ravel(), np.repeat(area, 3))
    for vi in range(3):
        i = faces[:, vi]
        for vn in range(3):
            nn = faces[:, vn]
            rows += [i, i]
            cols += [nn, nn + n]
            vals += [area * gx[:, vn], area * gy[:, vn]]
    rows = np.concatenate(rows)
    cols = np.concatenate(cols)
    vals = np.concatenate(vals) / wsum[rows]
    key = rows * (2 * n) + cols
    uniq, inv = np.unique(key, return_inverse=True)
    acc = np.zeros(len(uniq))
    np.add.at(acc, inv, vals)
    return (uniq // (2 * n)).astype(np.int64), (uniq % (2 * n)).astype(np.int64), acc.astype(np.float32)


def hole_plate(n: int = 71, hole_radius: float = 0.0, length: float = 100.0,
               jitter: float = 0.15, periodic: bool = True, seed: int = 69,
               stress_scale: float = 100.0, strain_range: tuple[float, float] | None = None) -> MeshSample:
    """One synthetic sample.  ``hole_radius`` is a fraction of ``length``."""
    rng = np.random.default_rng(seed)
    h = length / (n - 1)
    gi, gj = np.meshgrid(np.arange(n), np.arange(n), indexing="xy")
    pos = np.stack([gi.ravel() * h, gj.ravel() * h], 1)
    faces = _grid_triangles(n)
    if hole_radius > 0:
        center = np.array([length / 2, length / 2])
        r = np.linalg.norm(pos - center, axis=1)
        removed = r < hole_radius * length
        faces = faces[~removed[faces].any(1)]
    used = np.zeros(len(pos), bool)
    used[faces.ravel()] = True
    remap = -np.ones(len(pos), np.int64)
    remap[used] = np.arange(used.sum())
    pos = pos[used]
    faces = remap[faces]
    num_nodes = len(pos)

    # boundary edges (belong to exactly one face)
    fe = np.sort(np.concatenate([faces[:, [0, 1]], faces[:, [1, 2]], faces[:, [0, 2]]], 0), 1)
    ue, cnt = np.unique(fe, axis=0, return_counts=True)
    bnodes = np.unique(ue[cnt == 1].ravel())
    outer = (np.isclose(pos[:, 0], 0) | np.isclose(pos[:, 1], 0)
             | np.isclose(pos[:, 0], (n - 1) * h) | np.isclose(pos[:, 1], (n - 1) * h))
    node_types = np.full(num_nodes, NODE_INTERNAL, np.int64)
    node_types[bnodes] = NODE_INTERNAL_BOUNDARY
    node_types[outer] = NODE_EXTERNAL_BOUNDARY

    interior = node_types == NODE_INTERNAL
    pos = pos + interior[:, None] * rng.uniform(-jitter * h, jitter * h, size=pos.shape)
    pos = pos.astype(np.float32)

    edge_index = faces_to_edges(faces, num_nodes)
    edge_attr = edge_lengths(pos, edge_index)
    if periodic:
        pr, pc = periodic_pairs(pos)
        ei = np.concatenate([edge_index, np.stack([pr, pc])], 1)
        ea = np.concatenate([edge_attr, np.zeros(len(pr), np.float32)])
        edge_index, edge_attr = coalesce(ei, ea, num_nodes)

    rows, cols, vals = p1_divergence_operator(pos, faces)

    mean = (rng.uniform(-1.0, 1.0, size=3) * stress_scale).astype(np.float32)
    stiffen = 0.0
    if strain_range is not None:
        # hyperelastic-like targets: stiffening response sigma = k eps (1 + 4 |eps|) to a mean strain
        eps = rng.uniform(strain_range[0], strain_range[1], size=3)
        mean = (10.0 * stress_scale * eps * (1.0 + 4.0 * np.abs(eps))).astype(np.float32)
        stiffen = 4.0 * float(np.abs(eps).max())
    center = np.array([length / 2, length / 2])
    rel = pos.astype(np.float64) - center
    rr = np.maximum(np.linalg.norm(rel, axis=1), 1e-6)
    th = np.arctan2(rel[:, 1], rel[:, 0])
    rad = max(hole_radius * length, 0.5 * h)
    f = (rad / np.maximum(rr, rad)) ** 2
    wave = np.sin(2 * np.pi * pos[:, 0] / length) * np.cos(2 * np.pi * pos[:, 1] / length)
    amp = 0.1 * np.abs(mean).max() + 1e-3
    sxx = mean[0] * (1 + f * np.cos(2 * th)) + 0.5 * mean[2] * f * np.sin(2 * th) + amp * wave
    syy = mean[1] * (1 - f * np.cos(2 * th)) - 0.5 * mean[2] * f * np.sin(2 * th) - amp * wave
    sxy = mean[2] * (1 + f) + 0.25 * (mean[0] - mean[1]) * f * np.sin(2 * th) + 0.5 * amp * wave
    local = np.stack([sxx, syy, sxy], 1)
    if stiffen:
        local = local * (1.0 + stiffen * f)[:, None]
    local = local.astype(np.float32)
    return MeshSample(pos=pos, faces=faces, node_types=node_types, edge_index=edge_index,
                      edge_attr=edge_attr, op_div_rows=rows, op_div_cols=cols,
                      op_div_vals=vals, mean_stress=mean, local_stress=local)


def dataset_specs(num_graphs: int, hole_radius: tuple[float, float] = (0.0, 0.0),
                  seed: int = 69) -> list[tuple[float, int]]:
    """(hole radius, sample seed) of each graph ``make_dataset`` builds, without building it."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(num_graphs):
        r = float(rng.uniform(*hole_radius)) if hole_radius[1] > 0 else 0.0
        out.append((r, int(rng.integers(0, 2**31 - 1))))
    return out


def hole_plate_node_count(n: int, hole_radius: float, length: float = 100.0) -> int:
    """Node count of ``hole_plate(n, hole_radius)`` (geometry only: cheap, for sharding)."""
    h = length / (n - 1)
    gi, gj = np.meshgrid(np.arange(n), np.arange(n), indexing="xy")
    pos = np.stack([gi.ravel() * h, gj.ravel() * h], 1)
    faces = _grid_triangles(n)
    if hole_radius > 0:
        r = np.linalg.norm(pos - np.array([length / 2, length / 2]), axis=1)
        faces = faces[~(r < hole_radius * length)[faces].any(1)]
    return int(np.unique(faces.ravel()).size)


def make_dataset(num_graphs: int, n: int = 71, hole_radius: tuple[float, float] = (0.0, 0.0),
                 periodic: bool = True, seed: int = 69, jitter: float = 0.15,
                 strain_range: tuple[float, float] | None = None, indices=None) -> list[MeshSample]:
    """``num_graphs`` samples; hole radius drawn uniformly from ``hole_radius``.  ``indices``
    builds only those graphs of the dataset (a data-parallel shard), identical to the full build's."""
    specs = dataset_specs(num_graphs, hole_radius, seed)
    idx = range(num_graphs) if indices is None else indices
    return [hole_plate(n=n, hole_radius=specs[i][0], periodic=periodic, seed=specs[i][1], jitter=jitter,
                       strain_range=strain_range) for i in idx]
