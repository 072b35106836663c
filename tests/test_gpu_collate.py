"""Device-side collate: DeviceGraphStore.batch(indices) equals
Batch.from_data_list(...).to(dev) + plan_for bitwise, attribute by attribute, and a
training step on it equals the host-collated one."""
import pytest
import torch

from gpu_common import dev, make_batch
from pdg import graph, meshgen
from pdg.plan import plan_for

pytestmark = pytest.mark.gpu

PLAN_KEYS = ("perm", "src", "dst", "rowptr_dst", "perm_src", "rowptr_src", "ptr", "a_rowptr", "a_col", "a_val",
             "at_rowptr", "at_row", "at_comp", "at_val")


def _datasets():
    s1 = meshgen.make_dataset(3, n=13, hole_radius=(0.1, 0.2), seed=5)
    s2 = meshgen.make_dataset(2, n=9, hole_radius=(0.0, 0.0), seed=6)
    return [graph.sample_to_data(s) for s in s1 + s2] + [graph.sample_to_data(s2[0], periodic=False)]


@pytest.mark.parametrize("idx", [[0], [3, 0, 4], [5, 1, 2, 4, 3, 0]])
def test_device_batch_equals_host_batch(idx):
    from pdg.collate import DeviceGraphStore
    datas = _datasets()
    store = DeviceGraphStore(datas, dev())
    b_dev = store.batch(idx)
    b_host = graph.Batch.from_data_list([datas[i] for i in idx]).to(dev())
    for k in ("pos", "mean_stress", "local_stress", "nodes_types", "surfaces_nodes_for_div", "edge_attr",
              "edge_index", "batch", "ptr", "_eptr"):
        a, b = b_dev.__dict__[k], b_host.__dict__[k]
        assert a.dtype == b.dtype and a.shape == b.shape, k
        assert torch.equal(a, b), k
    p_dev, p_host = plan_for(b_dev), plan_for(b_host)
    assert (p_dev.n_nodes, p_dev.n_edges, p_dev.n_graphs, p_dev.has_div) == \
        (p_host.n_nodes, p_host.n_edges, p_host.n_graphs, p_host.has_div)
    for k in PLAN_KEYS:
        a, b = getattr(p_dev, k), getattr(p_host, k)
        assert a.dtype == b.dtype and a.shape == b.shape, k
        assert torch.equal(a, b), k
    # per-graph slicing (data_utils.py:25-33) works on the device batch
    g = b_dev[len(idx) - 1]
    assert torch.equal(g.pos, datas[idx[-1]].pos.to(dev()))


def test_training_step_on_device_batch_matches_host_batch():
    from gnn_local_stress.models import EncodeProcessDecode
    from gpu_common import dataset_stats
    from pdg.collate import DeviceGraphStore
    from pdg.trainer import Trainer
    datas = _datasets()
    idx = [4, 1, 2]
    store = DeviceGraphStore(datas, dev())
    b_dev = store.batch(idx)
    b_host = graph.Batch.from_data_list([datas[i] for i in idx]).to(dev())
    stats = {k: float(v) for k, v in dataset_stats(b_host).items()}
    res = []
    for b in (b_dev, b_host):
        torch.manual_seed(69)
        model = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=3, latent_size=128,
                                    input_nodes_features_size=6, output_nodes_features_size=3,
                                    **{k: torch.tensor(v) for k, v in stats.items()}).to(dev())
        tr = Trainer(model, lr=1e-3, divergence=True, divergence_penalty=10.0)
        out = tr.step(b)
        torch.cuda.synchronize()
        res.append((float(out["total"]), tr.flat_p.clone()))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])
