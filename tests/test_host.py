"""Host-side logic on CPU: synthetic mesh format, PyG-compatible batching, the
device graph plan (CSR) and the divergence operator layout."""
import numpy as np
import pytest
import torch

from pdg import graph, meshgen
from pdg.plan import GraphPlan
from pdg.dist import shard_graphs


def test_periodic_mesh_format():
    s = meshgen.hole_plate(71)
    assert s.num_nodes == 5041 and s.num_edges == 29968        # SURVEY §8d config 2 numbers
    ei = s.edge_index
    key = ei[0] * s.num_nodes + ei[1]
    assert np.all(np.diff(key) > 0)                            # coalesced: sorted, unique
    pairs = set(zip(ei[0].tolist(), ei[1].tolist()))
    assert all((b, a) in pairs for a, b in pairs)              # symmetric (to_undirected + both directions)
    assert int((s.edge_attr == 0).sum()) == 2 * 71 * 2 + 4     # periodic edges carry 0
    assert set(np.unique(s.node_types)) <= {-1, 0, 1}


def test_hole_plate_node_types_and_divergence_operator():
    s = meshgen.hole_plate(25, hole_radius=0.2)
    assert (s.node_types == -1).sum() > 0 and (s.node_types == 1).sum() > 0
    n = s.num_nodes
    A = np.zeros((n, 2 * n))
    np.add.at(A, (s.op_div_rows, s.op_div_cols), s.op_div_vals)
    # A = [Dx | Dy]: exact on linear fields
    x, y = s.pos[:, 0].astype(np.float64), s.pos[:, 1].astype(np.float64)
    assert np.abs(A[:, :n] @ x - 1).max() < 1e-4 and np.abs(A[:, n:] @ x).max() < 1e-4
    assert np.abs(A[:, n:] @ y - 1).max() < 1e-4


def test_batch_collate_and_slicing():
    samples = meshgen.make_dataset(3, n=9, hole_radius=(0.1, 0.2), seed=1)
    datas = [graph.sample_to_data(s) for s in samples]
    b = graph.Batch.from_data_list(datas)
    assert b.batch_size == 3 and len(b) == 3
    counts = [d.num_nodes for d in datas]
    assert b.ptr.tolist() == list(np.cumsum([0] + counts))
    assert b.edge_index.max() < sum(counts)
    b.local_stress = b.local_stress * 2              # slicing sees the batch's current attributes
    d1 = b[1]
    assert torch.equal(d1.local_stress, datas[1].local_stress * 2)
    assert torch.equal(d1.edge_index, datas[1].edge_index)


def test_graph_plan_csr():
    samples = meshgen.make_dataset(2, n=8, seed=2)
    b = graph.Batch.from_data_list([graph.sample_to_data(s) for s in samples])
    p = GraphPlan(b.edge_index, b.num_nodes, b.ptr, b.op_div_rows, b.op_div_cols, b.op_div_vals)
    src, dst = b.edge_index
    # dst-sorted order, stable -> sources ascending within a destination
    ps, pd = p.src.long(), p.dst.long()
    key = pd * p.n_nodes + ps
    assert torch.all(key[1:] > key[:-1])
    assert torch.equal(src[p.perm.long()], ps) and torch.equal(dst[p.perm.long()], pd)
    rp = p.rowptr_dst.long()
    for v in range(p.n_nodes):
        assert torch.all(pd[rp[v]:rp[v + 1]] == v)
    # src grouping of the sorted edges
    rps = p.rowptr_src.long()
    for v in range(p.n_nodes):
        assert torch.all(ps[p.perm_src.long()[rps[v]:rps[v + 1]]] == v)
    # divergence operator: A and A^T hold the same entries
    assert p.a_val.numel() == p.at_val.numel()
    assert torch.equal(torch.sort(p.a_val).values, torch.sort(p.at_val).values)


def test_shard_graphs_balanced_and_deterministic():
    counts = [5041, 300, 4000, 1200, 2500, 2500, 100, 999]
    sh = shard_graphs(counts, 3)
    assert sorted(i for s in sh for i in s) == list(range(len(counts)))
    loads = [sum(counts[i] for i in s) for s in sh]
    assert max(loads) - min(loads) <= max(counts)
    assert sh == shard_graphs(counts, 3)
    with pytest.raises(ValueError):
        shard_graphs(counts, 0)


def test_kernel_variants_need_explicit_ab_opt_in(monkeypatch):
    """Kernel selection is not taken from a stray environment variable: the
    shipped defaults unless PDG_AB=1; a non-default value without it is refused, malformed values
    always are, explicit overrides (tests, tools) are validated by name."""
    import pytest
    from pdg.engine import VARIANTS, kernel_variants
    for _, (env, _) in VARIANTS.items():
        monkeypatch.delenv(env, raising=False)
    monkeypatch.delenv("PDG_AB", raising=False)
    base = kernel_variants()
    assert base == {k: d for k, (_, d) in VARIANTS.items()}
    monkeypatch.setenv("PDG_FUSED_EDGE_WGRAD", "1")          # equal to the default: allowed
    assert kernel_variants() == base
    monkeypatch.setenv("PDG_FUSED_EDGE_WGRAD", "0")
    with pytest.raises(RuntimeError, match="PDG_AB=1"):
        kernel_variants()
    monkeypatch.setenv("PDG_AB", "1")
    assert kernel_variants()["fused_edge_wgrad"] is False
    monkeypatch.setenv("PDG_PAIR_BLOCKS_PER_CU", "x")
    with pytest.raises(ValueError):
        kernel_variants()
    monkeypatch.delenv("PDG_PAIR_BLOCKS_PER_CU")
    assert kernel_variants({"nbwd_coop": False})["nbwd_coop"] is False
    with pytest.raises(KeyError):
        kernel_variants({"no_such_variant": 1})
