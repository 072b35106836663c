"""The training harness visits the graphs in the reference's order.

The reference seeds torch (scripts/gnn_train.py:360), builds PyG DataLoaders (:387-394; a
torch.utils.data.DataLoader subclass), builds the model (Linear inits draw from the RNG), calls
print_model, which takes one batch from a fresh train iterator (gnn_local_stress/models.py:38),
and then, every epoch, iterates the train loader (shuffle=True: one base-seed draw per iterator
plus the RandomSampler's own seed) and the test loader (one base-seed draw).  Here that sequence
is replayed with plain torch DataLoaders over dataset items and compared with what
gnn_local_stress.train's loaders yield under the same seed and the same calls.  CPU only.
"""
import torch

from gnn_local_stress import models, train
from pdg import graph

SEED = 69


def _model():
    return models.EncodeProcessDecode(input_edges_features_size=1, input_nodes_features_size=6,
                                      message_passing_steps=2, latent_size=128, output_nodes_features_size=3)


class _Store:
    def __init__(self, n):
        self.num_graphs = n


def _reference_orders(n_train, n_test, bs, epochs):
    torch.manual_seed(SEED)
    train_ds = [f"train{i}" for i in range(n_train)]
    test_ds = [f"test{i}" for i in range(n_test)]
    tl = torch.utils.data.DataLoader(train_ds, batch_size=bs, shuffle=True, collate_fn=list)
    vl = torch.utils.data.DataLoader(test_ds, batch_size=bs, shuffle=False, collate_fn=list)
    _model()
    next(iter(tl))                                   # print_model (models.py:38)
    out = []
    for _ in range(epochs):
        out.append(([int(x[5:]) for b in tl for x in b], [int(x[4:]) for b in vl for x in b]))
    return out


def _harness_orders(n_train, n_test, bs, epochs):
    torch.manual_seed(SEED)
    model = _model()
    loaders = train.make_loaders(_Store(n_train), _Store(n_test), bs)
    models.print_model(model, loaders[0], "cpu")
    out = []
    for _ in range(epochs):
        out.append(([i for idx in loaders[0] for i in idx], [i for idx in loaders[1] for i in idx]))
    return out


def test_harness_epoch_order_equals_reference_loaders():
    for n_train, n_test, bs in ((10, 4, 3), (37, 9, 8), (5, 3, 2)):
        ref = _reference_orders(n_train, n_test, bs, 4)
        got = _harness_orders(n_train, n_test, bs, 4)
        assert got == ref
        # the shuffles are real (and differ per epoch), the test order is sequential
        assert len({tuple(o[0]) for o in ref}) > 1
        assert all(o[1] == list(range(n_test)) for o in ref)


def test_naive_sampler_order_differs():
    """Why the replay matters: one RandomSampler per epoch without the loader's base-seed draw and
    without print_model's iterator (the round-2 harness) gives other orders."""
    ref = _reference_orders(10, 4, 3, 2)
    torch.manual_seed(SEED)
    _model()
    naive = [list(torch.utils.data.RandomSampler(range(10))) for _ in range(2)]
    assert [o[0] for o in ref] != naive


def test_graph_dataloader_is_the_torch_loader():
    """pdg.graph.DataLoader draws like PyG's DataLoader: it is the torch loader with a graph collate."""
    from pdg import meshgen
    samples = meshgen.make_dataset(5, n=5, seed=3)
    datas = [graph.sample_to_data(s) for s in samples]
    for i, d in enumerate(datas):
        d.mean_stress = torch.full_like(d.mean_stress, float(i))     # tag each graph
    torch.manual_seed(SEED)
    got = [[int(b.mean_stress[int(b.ptr[k]), 0].item()) for k in range(b.num_graphs)]
           for b in graph.DataLoader(datas, batch_size=2, shuffle=True)]
    torch.manual_seed(SEED)
    ref = list(torch.utils.data.DataLoader(list(range(5)), batch_size=2, shuffle=True, collate_fn=list))
    assert got == ref
