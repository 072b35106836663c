"""Device mesh-graph construction (csrc/pdg_graph.hip) against the host
restatement of the reference's graph build: FaceToEdge + coalesce (pdg.meshgen.faces_to_edges,
convert_utils.py:47-60), edge lengths (torch.linalg.vector_norm, datasets.py:182-188) and
compute_periodic_graph (pdg.meshgen.periodic_pairs + coalesce, datasets.py:39-119; the
golden fixtures pin that restatement against the reference itself).  Integer outputs and
the fp32 lengths must be bitwise equal."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _host_graph(pos, faces, periodic):
    from pdg import meshgen
    n = len(pos)
    ei = meshgen.faces_to_edges(faces, n)
    p = torch.from_numpy(np.ascontiguousarray(pos, dtype=np.float32))
    ea = torch.linalg.vector_norm(p[torch.from_numpy(ei[0])] - p[torch.from_numpy(ei[1])], dim=1).numpy()
    if periodic:
        pr, pc = meshgen.periodic_pairs(pos[:, :2])
        ei2 = np.concatenate([ei, np.stack([pr, pc])], 1)
        ea2 = np.concatenate([ea, np.zeros(len(pr), np.float32)])
        ei, ea = meshgen.coalesce(ei2, ea2, n)
    return ei, ea


def _device_graph(pos, faces, periodic):
    from pdg.devgraph import mesh_graph
    ei, ea = mesh_graph(torch.from_numpy(np.ascontiguousarray(pos, dtype=np.float32)).cuda(),
                        torch.from_numpy(faces).cuda(), periodic)
    return ei.cpu().numpy(), ea.cpu().numpy()


@pytest.mark.parametrize("n,hole,periodic", [(5, 0.0, True), (21, 0.25, True), (71, 0.3, True), (71, 0.0, True),
                                             (33, 0.2, False), (317, 0.0, True)])
def test_mesh_graph_matches_host(n, hole, periodic):
    from pdg import meshgen
    s = meshgen.hole_plate(n=n, hole_radius=hole, periodic=periodic, seed=3)
    ei_h, ea_h = _host_graph(s.pos, s.faces, periodic)
    ei_d, ea_d = _device_graph(s.pos, s.faces, periodic)
    assert np.array_equal(ei_d, ei_h)
    assert np.array_equal(ea_d.view(np.int32), ea_h.view(np.int32))
    # the generator's own graph (what the training path uses) is the same object
    assert np.array_equal(ei_d, s.edge_index) and np.array_equal(ea_d.view(np.int32), s.edge_attr.view(np.int32))


def test_three_dimensional_points_and_lengths():
    """pyvista meshes carry (x, y, z): sides come from (x, y), lengths from all three."""
    from pdg import meshgen
    s = meshgen.hole_plate(n=21, hole_radius=0.2, periodic=True, seed=9)
    rng = np.random.default_rng(1)
    pts = np.concatenate([s.pos, rng.uniform(-1, 1, (len(s.pos), 1)).astype(np.float32)], 1)
    ei_h, ea_h = _host_graph(pts, s.faces, True)
    ei_d, ea_d = _device_graph(pts, s.faces, True)
    assert np.array_equal(ei_d, ei_h)
    assert np.array_equal(ea_d.view(np.int32), ea_h.view(np.int32))


def test_invalid_periodic_geometry_raises():
    from pdg import meshgen
    s = meshgen.hole_plate(n=9, hole_radius=0.0, periodic=True, seed=2)
    pos = s.pos.copy()
    right = np.where(pos[:, 0] == pos[:, 0].max())[0]
    pos[right[len(right) // 2], 0] -= 0.01          # one right-side node leaves the side
    with pytest.raises(ValueError, match="opposite sides"):
        _device_graph(pos, s.faces, True)
    ei_d, _ = _device_graph(pos, s.faces, False)     # the plain mesh graph is still fine
    assert np.array_equal(ei_d, _host_graph(pos, s.faces, False)[0])


def test_single_triangle_and_isolated_node():
    pos = np.array([[0, 0], [1, 0], [0, 1], [5, 5]], np.float32)
    faces = np.array([[0, 1, 2]], np.int64)
    ei_d, ea_d = _device_graph(pos, faces, False)
    ei_h, ea_h = _host_graph(pos, faces, False)
    assert np.array_equal(ei_d, ei_h) and np.array_equal(ea_d, ea_h)


def test_convert_mesh_to_graph_feeds_the_model():
    """benchmark_gnn_fem.py:388-415 on the device, then one forward: same output as the
    host-built graph of the same sample."""
    from gnn_local_stress.models import EncodeProcessDecode
    from pdg import graph, meshgen
    from pdg.devgraph import convert_mesh_to_graph
    s = meshgen.hole_plate(n=21, hole_radius=0.25, periodic=True, seed=4)
    host = graph.sample_to_data(s).to("cuda")
    dev = convert_mesh_to_graph(torch.from_numpy(s.pos).cuda(), torch.from_numpy(s.faces).cuda(),
                                s.mean_stress, torch.from_numpy(s.node_types))
    torch.manual_seed(69)
    stats = {k: torch.tensor(v) for k, v in {"mean_pos": 50.0, "std_pos": 29.0, "mean_mean_stress": 0.0,
                                             "std_mean_stress": 60.0, "mean_local_stress": 0.0,
                                             "std_local_stress": 60.0, "mean_edge_weight": 9.0,
                                             "std_edge_weight": 4.0}.items()}
    m = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=3, latent_size=128,
                            input_nodes_features_size=6, output_nodes_features_size=3, **stats).to("cuda")
    with torch.no_grad():
        a = m(host).local_stress
        b = m(dev).local_stress
    assert torch.equal(a, b)


@pytest.mark.parametrize("periodic", [True, False])
def test_dataset_files_with_device_graph_build(tmp_path, periodic):
    """MeshStressFieldDatasetInMemory(device="cuda") builds each sample's graph on the device:
    the same graphs as the host build of the same files."""
    import pandas as pd
    from gnn_local_stress import datasets, vtk_io
    from pdg import meshgen
    samples = meshgen.make_dataset(3, n=13, hole_radius=(0.1, 0.25), seed=5)
    rows = []
    for i, s in enumerate(samples):
        mesh = tmp_path / f"m{i}.vtk"
        vtk_io.write_legacy_vtk(mesh, s.pos, s.faces, point_type="float")
        data = tmp_path / f"m{i}.npz"
        np.savez(data, stress_field=s.local_stress, mean_stress=s.mean_stress.astype(np.float64),
                 op_div_matrix_data=s.op_div_vals, op_div_matrix_col_indices=s.op_div_cols.astype(np.int32),
                 op_div_matrix_row_indices=s.op_div_rows.astype(np.int32),
                 op_div_matrix_shape=np.array([s.num_nodes, 2 * s.num_nodes]), node_labels=s.node_types)
        rows.append((mesh.as_posix(), data.as_posix()))
    df = pd.DataFrame({"mesh_filename": [r[0] for r in rows], "data_filename": [r[1] for r in rows]})
    host = datasets.MeshStressFieldDatasetInMemory(df, periodic_graph=periodic)
    dev = datasets.MeshStressFieldDatasetInMemory(df, periodic_graph=periodic, device="cuda")
    for a, b in zip(host.graphs, dev.graphs):
        assert torch.equal(a.edge_index, b.edge_index)
        assert torch.equal(a.edge_attr, b.edge_attr)
        assert torch.equal(a.pos, b.pos)
    assert float(host.mean_edge_weight) == float(dev.mean_edge_weight)
