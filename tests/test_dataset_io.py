"""Reference on-disk dataset schema without pyvista/PyG:
legacy-VTK meshes + .npz fields + dataset.csv -> the same graphs the synthetic
generator builds in memory; inference output files.  CPU only.

No real dataset ships with the reference, so the files are written here from
pdg.meshgen samples in every legacy layout the reader accepts (parity against
VTK itself is unpinned; see gnn_local_stress/vtk_io.py)."""
import json

import numpy as np
import pytest
import torch

from gnn_local_stress import datasets, vtk_io
from pdg import graph, meshgen

LAYOUTS = [dict(binary=True, layout="5.1", dataset="POLYDATA"), dict(binary=False, layout="5.1", dataset="POLYDATA"),
           dict(binary=True, layout="4.2", dataset="POLYDATA"), dict(binary=False, layout="4.2", dataset="UNSTRUCTURED_GRID"),
           dict(binary=True, layout="4.2", dataset="UNSTRUCTURED_GRID")]


def _write_sample(tmp, i, s, **vtk_kw):
    mesh = tmp / f"hole_plate_mesh_{i}.vtk"
    vtk_io.write_legacy_vtk(mesh, s.pos, s.faces, point_type="float", **vtk_kw)
    data = tmp / f"hole_plate_mesh_{i}.npz"
    np.savez(data, stress_field=s.local_stress, mean_stress=s.mean_stress.astype(np.float64),
             mean_strain=np.zeros(3), mean_stress_material=np.zeros(3),
             op_div_matrix_data=s.op_div_vals, op_div_matrix_col_indices=s.op_div_cols.astype(np.int32),
             op_div_matrix_row_indices=s.op_div_rows.astype(np.int32),
             op_div_matrix_shape=np.array([s.num_nodes, 2 * s.num_nodes]), op_mean_stress=np.zeros(3),
             node_labels=s.node_types)
    return mesh.as_posix(), data.as_posix()


@pytest.mark.parametrize("kw", LAYOUTS)
def test_vtk_round_trip(tmp_path, kw):
    s = meshgen.hole_plate(n=9, hole_radius=0.2, seed=3)
    p = tmp_path / "m.vtk"
    vtk_io.write_legacy_vtk(p, s.pos, s.faces, **kw)
    pts, faces = vtk_io.read_legacy_vtk(p)
    assert np.array_equal(faces, s.faces)
    assert np.array_equal(pts[:, :2], s.pos.astype(np.float64)) and not pts[:, 2].any()


def test_vtk_rejects_garbage(tmp_path):
    p = tmp_path / "bad.vtk"
    p.write_bytes(b"not a vtk file\n")
    with pytest.raises(ValueError):
        vtk_io.read_legacy_vtk(p)


@pytest.mark.parametrize("periodic", [True, False])
def test_dataset_from_files_equals_generator(tmp_path, periodic):
    import pandas as pd
    samples = meshgen.make_dataset(3, n=11, hole_radius=(0.1, 0.2), seed=7) + meshgen.make_dataset(1, n=9, seed=8)
    rows = [_write_sample(tmp_path, i, s, **LAYOUTS[i % len(LAYOUTS)]) for i, s in enumerate(samples)]
    df = pd.DataFrame({"mesh_filename": [r[0] for r in rows], "data_filename": [r[1] for r in rows]})
    ds = datasets.MeshStressFieldDatasetInMemory(df, periodic_graph=periodic)
    assert len(ds) == len(samples)
    for g, s in zip(ds.graphs, samples):
        # the generator's graph of the same sample (periodic or not)
        if periodic:
            ei, ea = s.edge_index, s.edge_attr
        else:
            ei = meshgen.faces_to_edges(s.faces, s.num_nodes)
            ea = meshgen.edge_lengths(s.pos, ei)
        assert torch.equal(g.edge_index, torch.from_numpy(ei))
        assert torch.equal(g.edge_attr, torch.from_numpy(ea))
        assert torch.equal(g.pos, torch.from_numpy(s.pos))
        assert torch.equal(g.local_stress, torch.from_numpy(s.local_stress))
        assert torch.equal(g.mean_stress[0], torch.from_numpy(s.mean_stress))
        assert torch.equal(g.nodes_types[:, 0], torch.from_numpy(s.node_types))
        d_ref = graph.sample_to_data(s).op_div_matrix.to_dense()
        assert torch.equal(g.op_div_matrix.to_dense(), d_ref)
    b = graph.Batch.from_data_list([graph.sample_to_data(s, periodic) for s in samples]) if periodic else None
    if b is not None:
        assert float(ds.mean_edge_weight) == float(b.edge_attr.mean())
        assert float(ds.std_pos) == float(b.pos.std())
    loader = graph.DataLoader(ds, batch_size=3)
    sizes = [bb.batch_size for bb in loader]
    assert sizes == [3, 1]


def test_double_precision_points_give_float64_edge_lengths(tmp_path):
    s = meshgen.hole_plate(n=7, seed=2)
    pos64 = s.pos.astype(np.float64) + 1e-9
    p = tmp_path / "d.vtk"
    vtk_io.write_legacy_vtk(p, pos64, s.faces, point_type="double")
    pts, faces = vtk_io.read_legacy_vtk(p)
    g = datasets.mesh_to_graph(pts, faces)
    ea = datasets.compute_node_distances_as_edge_weights(g)
    assert ea.dtype == torch.float64   # datasets.py:182-188 runs in the points' dtype, cast afterwards
    ref = np.linalg.norm(pos64[g.edge_index[0].numpy()] - pos64[g.edge_index[1].numpy()], axis=1)
    assert np.allclose(ea.numpy(), ref, rtol=0, atol=1e-12)


def test_inference_output_files(tmp_path):
    """predict_and_save's file layout, with a stand-in model (the HIP model runs in the GPU test)."""
    import pandas as pd
    from gnn_local_stress import inference
    samples = meshgen.make_dataset(3, n=9, seed=9)
    rows = [_write_sample(tmp_path, i, s) for i, s in enumerate(samples)]
    df = pd.DataFrame({"mesh_filename": [r[0] for r in rows], "data_filename": [r[1] for r in rows]})
    ds = datasets.MeshStressFieldDatasetInMemory(df)

    class Fake:
        def forward(self, b, scale_output=True, scale_input=True):
            return graph.Data(local_stress=b.pos.sum(1, keepdim=True).repeat(1, 3))

    loader = graph.DataLoader(ds, batch_size=2)
    names = inference.predict_and_save(Fake(), loader, tmp_path / "out", "cpu")
    assert [n.split("/")[-1] for n in names] == [f"hole_plate_mesh_{i}.npz" for i in range(3)]
    for i, n in enumerate(names):
        with np.load(n) as f, np.load(rows[i][1]) as org:
            assert set(f.files) == set(org.files)
            exp = ds.graphs[i].pos.sum(1, keepdim=True).repeat(1, 3).numpy()
            assert np.array_equal(f["stress_field"], exp)
            assert np.array_equal(f["op_div_matrix_data"], org["op_div_matrix_data"])


def test_quad_mesh_graph(tmp_path):
    """convert_utils.py:63-81: a quad mesh's graph has the four sides of every cell, undirected and
    coalesced -- checked on a hand-built 3 x 2-cell grid against the grid's own neighbour pairs, then
    through a VTK file and the dataset's periodic construction."""
    nx, ny = 4, 3                                  # nodes per row / column
    pts = np.array([[x * 10.0, y * 7.0, 0.0] for y in range(ny) for x in range(nx)], np.float32)
    quads = np.array([[y * nx + x, y * nx + x + 1, (y + 1) * nx + x + 1, (y + 1) * nx + x]
                      for y in range(ny - 1) for x in range(nx - 1)], np.int64)
    g = datasets.mesh_to_graph(pts, quads)
    want = set()
    for y in range(ny):
        for x in range(nx):
            v = y * nx + x
            if x + 1 < nx:
                want |= {(v, v + 1), (v + 1, v)}
            if y + 1 < ny:
                want |= {(v, v + nx), (v + nx, v)}
    ei = g.edge_index.numpy()
    assert set(map(tuple, ei.T.tolist())) == want and ei.shape[1] == len(want)   # no diagonals, no duplicates
    key = ei[0] * len(pts) + ei[1]
    assert np.all(np.diff(key) > 0)                 # coalesced: sorted by (row, col)
    # through the VTK reader (cell type 9) and the periodic dataset construction
    p = tmp_path / "q.vtk"
    vtk_io.write_legacy_vtk(p, pts, quads)
    pts2, faces2 = vtk_io.read_legacy_vtk(p)
    assert faces2.shape == (6, 4)
    g2 = datasets.mesh_to_graph(pts2, faces2)
    assert np.array_equal(g2.edge_index.numpy(), ei)
    g2.edge_attr = datasets.compute_node_distances_as_edge_weights(g2).float()
    lengths = dict(zip(map(tuple, ei.T.tolist()), g2.edge_attr.numpy().tolist()))
    assert lengths[(0, 1)] == 10.0 and lengths[(0, nx)] == 7.0
    gp = datasets.compute_periodic_graph(g2)
    assert gp.edge_index.shape[1] > ei.shape[1]     # periodic pairs added with zero length
    assert float(gp.edge_attr[gp.edge_attr == 0].sum()) == 0.0 and int((gp.edge_attr == 0).sum()) > 0
    with pytest.raises(ValueError):
        datasets.mesh_to_graph(pts, quads[:, :2])


def test_mesh_to_graph_matches_reference_fixture():
    """gnn_local_stress.datasets.mesh_to_graph against the reference's own convert_utils.mesh_to_graph /
    _quad_face_to_edge (convert_utils.py:47-81), run by tests/golden/make_golden_graphs.py on a quad
    grid with scrambled node ids, clockwise quads and a triangulated hole plate: edge_index bit for bit."""
    from pathlib import Path
    from gnn_local_stress import datasets
    g = np.load(Path(__file__).resolve().parent / "golden" / "mesh_to_graph.npz")
    names = sorted({k.rsplit("_", 1)[0] for k in g.files if k.endswith("_points")})
    assert names == ["quad_clockwise", "quad_scrambled", "tri_hole_plate"]
    for name in names:
        out = datasets.mesh_to_graph(g[f"{name}_points"], g[f"{name}_cells"])
        ref = g[f"{name}_edge_index"]
        assert out.edge_index.dtype == torch.int64
        assert np.array_equal(out.edge_index.numpy(), ref), name
