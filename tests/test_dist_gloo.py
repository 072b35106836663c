"""Graph-batch DP on CPU with gloo, world_size 2: the all-reduced
flat gradient bucket equals the mean of the per-shard gradients, each shard
computed as its own batch (replica semantics).  The per-shard gradients come
from the CPU oracle (test infrastructure); the DP logic under test is
pdg.dist (sharding + flat-bucket all-reduce), the same code the GPU Trainer uses."""
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


def _shard_grads(samples, idx):
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
    from pdg.dist import allreduce_mean_, shard_graphs
    samples = meshgen.make_dataset(4, n=7, hole_radius=(0.0, 0.0), seed=9)
    shards = shard_graphs([s.num_nodes for s in samples], world)
    flat = _shard_grads(samples, shards[rank])
    allreduce_mean_(flat)
    if rank == 0:
        ref = sum(_shard_grads(samples, s) for s in shards) / world
        q.put(float((flat - ref).abs().max() / ref.abs().max()))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_allreduce_equals_mean_of_shard_gradients():
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
