"""Graph-batch DP on CPU with gloo, world_size 2: every rank's shard loss is divided
by the GLOBAL minibatch's graph count and the flat gradient buckets are summed, so on an odd
minibatch of unequal graphs (shards of 2 and 1 graphs) every graph still weighs 1/B
(gnn_train.py:193/196).  The per-shard gradients come from the CPU oracle (test infrastructure);
the DP logic under test is pdg.dist (sharding, the flat-bucket all-reduce), the same code the GPU
Trainer and the training harness use.  Also: the harness's per-rank share of every reference
minibatch (pdg.dist.shard_minibatch) partitions it in the loader's order."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_grads(samples, idx, b_global=None):
    from oracle import epd_oracle as O
    from pdg import graph
    from pdg.engine import PARAM_NAMES
    datas = [graph.sample_to_data(samples[i]) for i in idx]
    b = graph.Batch.from_data_list(datas)
    st = {"mean_pos": torch.tensor(50.0), "std_pos": torch.tensor(29.0), "mean_mean_stress": torch.tensor(0.0),
          "std_mean_stress": torch.tensor(60.0), "mean_local_stress": torch.tensor(0.0),
          "std_local_stress": torch.tensor(60.0), "mean_edge_weight": torch.tensor(9.0),
          "std_edge_weight": torch.tensor(4.0)}
    P = {k: v.double().requires_grad_(True) for k, v in O.init_params().items()}
    st = {k: v.double() for k, v in st.items()}
    pred = O.epd_forward(P, st, b.pos.double(), b.mean_stress.double(), b.nodes_types, b.edge_index,
                         b.edge_attr.double(), 2, scale_output=False)
    gt = (b.local_stress.double() - st["mean_local_stress"]) / st["std_local_stress"]
    total, _, _ = O.batch_loss(pred, gt, b.ptr, [d.op_div_matrix.double() for d in datas], b.nodes_types,
                               True, 10.0)
    if b_global is not None:        # / B_global instead of / B_shard
        total = total * (len(idx) / b_global)
    total.backward()
    return torch.cat([P[n].grad.reshape(-1) for n in PARAM_NAMES])


def _worker(rank, world, port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "p-div-gnn_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pdg import meshgen
    from pdg.dist import allreduce_sum_, shard_graphs
    samples = meshgen.make_dataset(3, n=7, hole_radius=(0.1, 0.3), seed=9)
    B = len(samples)
    shards = shard_graphs([s.num_nodes for s in samples], world)
    assert sorted(len(s) for s in shards) == [1, 2]
    flat = _shard_grads(samples, shards[rank], B)
    allreduce_sum_(flat)
    if rank == 0:
        ref = sum(_shard_grads(samples, s, B) for s in shards)
        q.put(float((flat - ref).abs().max() / ref.abs().max()))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_allreduce_sums_shard_gradients_over_global_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    err = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert err < 1e-12


def test_shard_minibatch_partitions_reference_batches():
    """Every rank's graphs of every minibatch the reference's loader yields (the seeded torch
    DataLoader order, gnn_train.py:387-394): disjoint, together the whole minibatch, each in the
    loader's order, balanced by node count (max shard within the largest graph of the mean)."""
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "p-div-gnn_amd")]
    from pdg.dist import shard_minibatch
    from pdg.graph import index_loader
    gen = torch.Generator().manual_seed(5)
    counts = [int(c) for c in torch.randint(300, 2000, (23,), generator=gen)]
    for world in (1, 2, 3, 4, 8):
        torch.manual_seed(69)
        for idx in index_loader(len(counts), 7, shuffle=True):
            parts = [shard_minibatch(idx, counts, world, r) for r in range(world)]
            assert sorted(i for p in parts for i in p) == sorted(idx)
            for p in parts:
                assert p == [i for i in idx if i in p]          # the loader's relative order
            loads = [sum(counts[i] for i in p) for p in parts]
            assert max(loads) <= sum(loads) / world + max(counts[i] for i in idx)


def test_sync_shardable_detects_empty_and_edgeless_shards():
    """dp_mode "sync" needs every rank's share to hold edges (every rank joins every LayerNorm
    statistic collective); a minibatch failing that (fewer graphs than ranks, or a shard of edgeless
    graphs) is stepped whole on one rank (gnn_local_stress/train.py, Trainer.step solo)."""
    import numpy as np
    from pdg.dist import shard_graphs, sync_shardable

    class Store:
        n = np.array([10, 20, 30, 5])
        e = np.array([40, 0, 90, 12])
    assert sync_shardable([0, 1, 2, 3], Store, 2)
    assert not sync_shardable([2], Store, 2)            # one graph, two ranks
    assert shard_graphs([20, 5], 2) == [[0], [1]]
    assert not sync_shardable([1, 3], Store, 2)         # rank 0's shard is the edgeless graph 1
    assert sync_shardable([1, 3], Store, 1)
