"""Graph-batch DP through the GPU Trainer, world_size 2 on one GPU.

Both ranks run pdg.trainer.Trainer on cuda:0 with a gloo process group (RCCL
refuses two ranks on one device; the Trainer's collective is the same
`all_reduce` either way).  Checked: the all-reduced flat gradient bucket equals
the sum over shards of the fp64 oracle's shard gradients with every shard's loss
divided by the GLOBAL graph count (dp_mode "replica": each graph weighs 1/B as in
gnn_train.py:193/196, also for the odd 3-graph minibatch of unequal graphs whose
shards hold 2 and 1 graphs) or the fp64 oracle gradient of the whole global
minibatch on one device (dp_mode "sync", graph-LayerNorm statistics exchanged);
the reported loss is the global minibatch's; the parameters stay bit-identical
across ranks after several Adam steps.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

STEPS_MP = 4
STATS = {"mean_pos": 50.0, "std_pos": 29.0, "mean_mean_stress": 0.0, "std_mean_stress": 60.0,
         "mean_local_stress": 0.0, "std_local_stress": 60.0, "mean_edge_weight": 9.0, "std_edge_weight": 4.0}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_grads(P0, samples, idx):
    from oracle import epd_oracle as O
    from pdg import graph
    from pdg.engine import PARAM_NAMES
    datas = [graph.sample_to_data(samples[i]) for i in idx]
    b = graph.Batch.from_data_list(datas)
    P = {k: v.detach().cpu().double().requires_grad_(True) for k, v in P0.items()}
    st = {k: torch.tensor(v, dtype=torch.float64) for k, v in STATS.items()}
    pred = O.epd_forward(P, st, b.pos.double(), b.mean_stress.double(), b.nodes_types, b.edge_index,
                         b.edge_attr.double(), STEPS_MP, scale_output=False)
    gt = (b.local_stress.double() - st["mean_local_stress"]) / st["std_local_stress"]
    total, _, _ = O.batch_loss(pred, gt, b.ptr, [d.op_div_matrix.double() for d in datas], b.nodes_types,
                               True, 10.0)
    total.backward()
    return torch.cat([P[n].grad.reshape(-1) for n in PARAM_NAMES]), float(total.detach())


def _worker(rank, world, port, q, mode):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "p-div-gnn_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gnn_local_stress.models import EncodeProcessDecode
        from pdg import graph, meshgen
        from pdg.dist import shard_graphs
        from pdg.trainer import Trainer
        if mode == "replica_unequal":   # three hole plates of different sizes: shards of 2 and 1 graphs
            samples = meshgen.make_dataset(3, n=9, hole_radius=(0.1, 0.3), seed=11)
        else:
            samples = meshgen.make_dataset(4, n=9, hole_radius=(0.0, 0.0), seed=11)
        shards = shard_graphs([s.num_nodes for s in samples], world)
        B = len(samples)
        batch = graph.Batch.from_data_list([graph.sample_to_data(samples[i]) for i in shards[rank]]).to(dev)
        torch.manual_seed(69)
        model = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=STEPS_MP, latent_size=128,
                                    input_nodes_features_size=6, output_nodes_features_size=3,
                                    **{k: torch.tensor(v) for k, v in STATS.items()}).to(dev)
        P0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
        tr = Trainer(model, lr=1e-3, divergence=True, divergence_penalty=10.0, process_group=dist.group.WORLD,
                     dp_mode="sync" if mode == "sync" else "replica")
        out = tr.step(batch, n_global_graphs=B)
        torch.cuda.synchronize()
        g = tr.flat_g.detach().double().cpu()
        loss = float(out["total"])
        for _ in range(3):
            tr.step(batch, n_global_graphs=B)
        torch.cuda.synchronize()
        p = tr.flat_p.detach().cpu()
        ps = [torch.empty_like(p) for _ in range(world)]
        dist.all_gather(ps, p)
        if rank == 0:
            if mode == "sync":
                ref, ref_loss = _oracle_grads(P0, samples, sorted(i for s in shards for i in s))
            else:   # every shard's loss / B_global: its batch_loss (/ B_shard) scaled by B_shard / B
                assert len({len(s) for s in shards}) == (2 if mode == "replica_unequal" else 1), shards
                rs = [_oracle_grads(P0, samples, s) for s in shards]
                ref = sum(r[0] * (len(s) / B) for r, s in zip(rs, shards))
                ref_loss = sum(r[1] * (len(s) / B) for r, s in zip(rs, shards))
            q.put((float((g - ref).norm() / ref.norm()), max(float((x - ps[0]).abs().max()) for x in ps),
                   abs(loss - ref_loss) / abs(ref_loss)))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["replica", "replica_unequal", "sync"])
def test_trainer_dp_world2_on_one_gpu(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, mode)) for r in range(2)]
    for p in procs:
        p.start()
    gerr, pdiff, lerr = q.get(timeout=400)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert gerr < 1e-4, gerr
    assert lerr < 1e-5, lerr
    assert pdiff == 0.0, pdiff
