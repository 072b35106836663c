"""Trainer(capture=True): forward + loss + backward replayed from one captured HIP graph
gives bit-identical losses and parameters to eager launches, step after step, with and
without the divergence loss; a new batch object is captured afresh."""
import pytest
import torch

from gpu_common import dataset_stats, dev
from pdg import graph, meshgen

pytestmark = pytest.mark.gpu


def _batch(seed, n_graphs=3):
    samples = meshgen.make_dataset(n_graphs, n=13, hole_radius=(0.1, 0.2), seed=seed)
    return graph.Batch.from_data_list([graph.sample_to_data(s) for s in samples]).to(dev())


def _trainer(batch, divergence, capture):
    from gnn_local_stress.models import EncodeProcessDecode
    from pdg.trainer import Trainer
    stats = {k: torch.tensor(float(v)) for k, v in dataset_stats(batch).items()}
    torch.manual_seed(69)
    model = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=3, latent_size=128,
                                input_nodes_features_size=6, output_nodes_features_size=3, **stats).to(dev())
    return Trainer(model, lr=1e-3, divergence=divergence, divergence_penalty=10.0, capture=capture)


@pytest.mark.parametrize("divergence", [False, True])
def test_graph_replay_equals_eager(divergence):
    b1, b2 = _batch(11), _batch(12)
    runs = []
    for capture in (False, True):
        tr = _trainer(b1, divergence, capture)
        losses = []
        for b in (b1, b1, b1, b2, b2, b1):        # re-capture on each change of batch object
            out = tr.step(b)
            losses.append(float(out["total"]))    # read before the next replay overwrites it
        torch.cuda.synchronize()
        runs.append((losses, tr.flat_p.clone(), tr.flat_g.clone()))
    (l0, p0, g0), (l1, p1, g1) = runs
    assert l0 == l1
    assert torch.equal(g0, g1)
    assert torch.equal(p0, p1)
    assert len(set(l0)) > 1                       # the parameters moved between steps


def test_graph_recaptured_when_the_loss_normaliser_changes():
    """A captured step holds 1/B_global as a constant: stepping the same batch object with another
    n_global_graphs records a new graph instead of replaying the old normaliser (world-1 gloo group,
    replica mode), so captured and eager runs stay bit-identical."""
    import os
    import socket
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(s.getsockname()[1]))
    s.close()
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        b = _batch(13)
        runs = []
        for capture in (False, True):
            tr = _trainer(b, True, capture)
            tr.pg = dist.group.WORLD
            tr.capture = capture
            gs = []
            for bn in (3, 3, 6, 6, 3):
                tr.step(b, n_global_graphs=bn)
                gs.append(tr.flat_g.clone())
            torch.cuda.synchronize()
            runs.append((gs, tr.flat_p.clone()))
        (g0, p0), (g1, p1) = runs
        assert all(torch.equal(a, c) for a, c in zip(g0, g1))
        assert torch.equal(p0, p1)
    finally:
        dist.destroy_process_group()
