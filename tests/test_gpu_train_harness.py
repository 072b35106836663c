"""The training harness (gnn_local_stress.train, mirroring scripts/gnn_train.py:95-442) on the
HIP path: a config with the reference's YAML keys (configs_train/config_train_div.yml) runs
end to end over device-resident datasets and writes what the reference writes.

Checked: the best / last checkpoints exist in the reference's format and reload; the config is
copied; early stopping follows the reference's rule; and the epoch losses equal an independent
replay of the same loop (same seed, torch DataLoaders drawing from the RNG as PyG's do, one
Trainer step per minibatch, losses averaged over batches) — the bookkeeping of
gnn_train.py:154-207 / :258-275."""
import pandas as pd
import pytest
import torch
import yaml

from gpu_common import dev
from test_dataset_io import _write_sample

pytestmark = pytest.mark.gpu


def _dataset(tmp, name, n_graphs, seed):
    from pdg import meshgen
    d = tmp / name
    d.mkdir()
    samples = meshgen.make_dataset(n_graphs, n=11, hole_radius=(0.1, 0.2), seed=seed)
    rows = [_write_sample(d, i, s) for i, s in enumerate(samples)]
    csv = d / "dataset.csv"
    pd.DataFrame({"mesh_filename": [r[0] for r in rows], "data_filename": [r[1] for r in rows]}).to_csv(csv, index=False)
    return csv


def _config(tmp, **kw):
    cfg = dict(dataset_train_csv=_dataset(tmp, "train", 5, 31).as_posix(),
               dataset_test_csv=_dataset(tmp, "test", 3, 32).as_posix(),
               results_folder=(tmp / "res").as_posix(), epochs=3, batch_size=2, learning_rate=0.001,
               early_stopping_limit=20, divergence=True, divergence_penalty=10, latent_size=128,
               message_passing_steps=3, train_all_epochs=True, monitor_divergence_in_test=True, periodic_graph=True)
    cfg.update(kw)
    p = tmp / "config_train_div.yml"
    p.write_text(yaml.safe_dump(cfg))
    return p, cfg


def test_harness_end_to_end(tmp_path):
    from gnn_local_stress import datasets, losses, models, train
    from pdg.collate import DeviceGraphStore
    from pdg.trainer import Trainer
    cfg_path, cfg = _config(tmp_path)
    logs = []
    tr_losses, te_losses = train.main(cfg_path.as_posix(), device="cuda:0", log=logs.append)
    res = tmp_path / "res"
    assert (res / "config_train_div.yml").is_file()
    assert (res / "weights" / "model_weights.pth").is_file()
    assert (res / "weights" / "last_epoch_model_weights.pth").is_file()
    assert len(tr_losses) == 3 and len(te_losses) == 3
    m = models.EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=3, latent_size=128,
                                   input_nodes_features_size=6, output_nodes_features_size=3)
    assert models.load_model_checkpoint(m, (res / "weights" / "last_epoch_model_weights.pth").as_posix()) == 3
    best_epoch = 1 + min(range(3), key=lambda i: te_losses[i])
    assert models.load_model_checkpoint(m, (res / "weights" / "model_weights.pth").as_posix()) == best_epoch

    # independent replay of the same loop
    torch.manual_seed(train.SEED)
    tr_ds = datasets.MeshStressFieldDatasetInMemory(pd.read_csv(cfg["dataset_train_csv"]))
    te_ds = datasets.MeshStressFieldDatasetInMemory(pd.read_csv(cfg["dataset_test_csv"]))
    store, tstore = DeviceGraphStore(tr_ds.graphs, dev()), DeviceGraphStore(te_ds.graphs, dev())
    model = models.EncodeProcessDecode(input_edges_features_size=1, input_nodes_features_size=6,
                                       message_passing_steps=3, latent_size=128, output_nodes_features_size=3,
                                       **{k: v.to(dev()) for k, v in tr_ds.stats().items()}).to(dev())
    t = Trainer(model, lr=1e-3, divergence=True, divergence_penalty=10.0)
    # the reference's loaders (gnn_train.py:387-394) and print_model's extra iterator (models.py:38)
    tl = torch.utils.data.DataLoader(range(5), batch_size=2, shuffle=True, collate_fn=list)
    vl = torch.utils.data.DataLoader(range(3), batch_size=2, shuffle=False, collate_fn=list)
    next(iter(tl))
    for epoch in range(3):
        tot = [float(t.step(store.batch(idx))["total"]) for idx in tl]
        assert abs(sum(tot) / len(tot) - tr_losses[epoch]) <= 1e-6 * abs(tr_losses[epoch])
        with torch.no_grad():
            te = []
            for idx in vl:
                b = tstore.batch(idx)
                pred = model(b, scale_output=False).local_stress
                gt = ((b.local_stress - model.mean_local_stress) / model.std_local_stress).float().contiguous()
                te.append(float(losses.batch_loss(pred, b, gt, divergence=True, divergence_penalty=1.0)[0]))
        assert abs(sum(te) / len(te) - te_losses[epoch]) <= 1e-6 * abs(te_losses[epoch])


def test_harness_early_stopping(tmp_path):
    from gnn_local_stress import train
    cfg_path, _ = _config(tmp_path, epochs=6, early_stopping_limit=1, train_all_epochs=False, learning_rate=0.5)
    logs = []
    tr_losses, te_losses = train.main(cfg_path.as_posix(), device="cuda:0", log=logs.append)
    # the reference rule (gnn_train.py:140-146): stop once the test loss failed to improve
    # early_stopping_limit times in a row
    best, bad = float("inf"), 0
    for i, v in enumerate(te_losses):
        bad = 0 if v < best else bad + 1
        best = min(best, v)
        if bad >= 1 and i + 1 < 6:
            assert len(te_losses) == i + 1 and "Training early stopped" in logs
            break


# ------------------------------------------------------------------ graph-batch DP in the harness
def _harness_worker(rank, world, port, cfg_path, mode, res_dir, q):
    import os
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "p-div-gnn_amd")]
    # what torchrun exports; gloo because RCCL refuses two ranks on one device
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), PDG_DIST_BACKEND="gloo")
    torch.set_num_threads(2)
    import torch.distributed as dist
    from gnn_local_stress import train
    try:
        logs = []
        tr, te = train.main(cfg_path, device="cuda:0", log=logs.append, dp_mode=mode, results_folder=res_dir)
        q.put((rank, tr, te, len(logs)))
        dist.barrier()
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run_world2(cfg_path, mode, res_dir):
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_harness_worker, args=(r, 2, port, cfg_path, mode, res_dir, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    return got


def test_harness_dp_sync_world2_equals_one_device(tmp_path):
    """torchrun-style 2-rank run of the harness (gloo, one GPU) in dp_mode "sync": each rank trains
    on its share of every reference-ordered minibatch, yet the epoch losses equal the one-device run
    (the exact mode: LayerNorm statistics exchanged, losses / B_global, gradients summed); only
    rank 0 logs and writes.  5 training graphs at batch size 2: every epoch ends with a one-graph
    minibatch, which cannot give both ranks a shard (rank 0 steps on it whole, Trainer.step solo)."""
    from gnn_local_stress import train
    cfg_path, cfg = _config(tmp_path, epochs=2)
    tr1, te1 = train.main(cfg_path.as_posix(), device="cuda:0", log=lambda *a: None,
                          results_folder=(tmp_path / "one").as_posix())
    got = _run_world2(cfg_path.as_posix(), "sync", (tmp_path / "two").as_posix())
    (_, tr_a, te_a, logs_a), (_, tr_b, te_b, logs_b) = got
    assert tr_a == tr_b and te_a == te_b            # every rank reports the global losses
    assert logs_a > 0 and logs_b == 0               # rank 0 logs, rank 1 is quiet
    for x, y in zip(tr_a + te_a, tr1 + te1):
        assert abs(x - y) <= 1e-4 * abs(y), (tr_a, te_a, tr1, te1)
    assert (tmp_path / "two" / "weights" / "last_epoch_model_weights.pth").is_file()


def test_harness_dp_replica_world2_odd_minibatches(tmp_path):
    """dp_mode "replica" over minibatches of 2, 2 and 1 graphs (the last leaves rank 1 without a
    graph: it contributes zeros and takes the same Adam step): the run completes with the same
    global losses on both ranks, finite, and rank 0's checkpoints."""
    cfg_path, _ = _config(tmp_path, epochs=2)
    got = _run_world2(cfg_path.as_posix(), "replica", (tmp_path / "rep").as_posix())
    (_, tr_a, te_a, _), (_, tr_b, te_b, _) = got
    assert tr_a == tr_b and te_a == te_b
    assert all(v == v and abs(v) < 1e6 for v in tr_a + te_a)
    assert (tmp_path / "rep" / "weights" / "model_weights.pth").is_file()
