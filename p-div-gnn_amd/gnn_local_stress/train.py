"""Training harness of the reference (``scripts/gnn_train.py``) on the HIP path.

Mirrors ``run_experience`` (gnn_train.py:331-435), ``train`` (:95-305) and ``main``
(:438-...): the same YAML keys (``configs_train/config_train_*.yml``), the same epoch loop
with early stopping, the same train / test loss bookkeeping (per-batch losses summed on the
device, divided by the number of batches once per epoch), the best-test-loss checkpoint
``weights/model_weights.pth`` and the last-epoch checkpoint
``weights/last_epoch_model_weights.pth`` in the reference's checkpoint format, and a copy of
the config in the results folder.  What runs underneath is MI355X-native:

* the datasets are uploaded once into HBM (``pdg.collate.DeviceGraphStore``) and every
  minibatch is collated on the device in one launch;
* each training step is ``pdg.trainer.Trainer.step`` (HIP forward, fused NMSE + divergence
  loss, HIP backward, Adam stepped with GradScaler's skip semantics) with no host sync;
* the test pass runs the HIP forward under ``no_grad`` and the fused batch loss;
* under ``torchrun`` (WORLD_SIZE > 1) it trains with graph-batch data parallelism, one process per
  GPU: every rank draws the same reference-ordered global minibatches, takes its
  ``pdg.dist.shard_minibatch`` share of each (whole graphs, balanced by node count), divides its
  losses by the GLOBAL minibatch's graph count and the gradients are summed over RCCL, so every
  graph weighs 1/B as in gnn_train.py:193/196.  Rank 0 logs and writes the checkpoints.

Minibatches come from ``torch.utils.data.DataLoader`` objects over the graph indices
(``pdg.graph.index_loader``; PyG's ``DataLoader`` is that same torch loader with a graph collate),
created where the reference creates its loaders (gnn_train.py:387-394) and iterated where it
iterates them: ``print_model`` takes one batch from a fresh train iterator (models.py:38), every
epoch iterates the train loader (one base-seed draw plus the RandomSampler's seed) and the test
loader (one base-seed draw).  After ``torch.manual_seed(69)`` the harness therefore visits the
graphs in the reference's order (tests/test_train_order.py).  TensorBoard logging, dataset histograms and the tqdm bars are out of scope
(SURVEY §8); the losses they would log are printed and returned.

    python -m gnn_local_stress.train configs_train/config_train_div.yml
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m gnn_local_stress.train configs_train/config_train_div.yml
"""
from __future__ import annotations

import os
import random
import shutil
import sys
from pathlib import Path
from typing import Any

import numpy as np
import torch

import torch.distributed as dist

from pdg.collate import DeviceGraphStore
from pdg.dist import shard_minibatch, sync_shardable
from pdg.graph import index_loader
from pdg.trainer import Trainer

from . import data_utils, datasets, losses, models

SEED = 69   # gnn_train.py:38


def make_loaders(train_store: DeviceGraphStore, test_store: DeviceGraphStore, batch_size: int):
    """The reference's two loaders (gnn_train.py:387-394) over the stores' graph indices."""
    return (index_loader(train_store.num_graphs, batch_size, shuffle=True),
            index_loader(test_store.num_graphs, batch_size, shuffle=False))


def evaluate(model, store: DeviceGraphStore, loader, monitor_divergence: bool, process_group=None,
             shard: bool = True):
    """The test pass of gnn_train.py:208-252: sum over batches of (NMSE/B [+ div/B]) and of the
    divergence term (unpenalised, as the reference monitors it), as device scalars.  ``loader``
    yields graph-index lists (an int batch size builds an unshuffled one).

    With a process group and ``shard`` (replica data parallelism), every rank evaluates its
    ``shard_minibatch`` share of each test minibatch with its losses scaled to / B_global and the
    two sums are all-reduced once at the end; without ``shard`` (dp_mode "sync") every rank
    evaluates the whole minibatches, so the test loss is the one-device value on every rank."""
    if isinstance(loader, int):
        loader = index_loader(store.num_graphs, loader, shuffle=False)
    total = torch.zeros((), dtype=torch.float32, device=store.device)
    div_sum = torch.zeros((), dtype=torch.float32, device=store.device)
    nb = 0
    world = dist.get_world_size(process_group) if process_group is not None else 1
    rank = dist.get_rank(process_group) if process_group is not None else 0
    with torch.no_grad():
        for idx in loader:
            nb += 1
            mine = shard_minibatch(idx, store.n, world, rank) if (world > 1 and shard) else list(idx)
            if not mine:
                continue
            batch = store.batch(mine)
            pred = model.forward(batch, scale_output=False, scale_input=True).local_stress
            gt = data_utils.standardize(batch.local_stress, model.mean_local_stress, model.std_local_stress)
            t, _, d = losses.batch_loss(pred, batch, gt.float().contiguous(), divergence=monitor_divergence,
                                        divergence_penalty=1.0)
            w = len(mine) / len(idx)        # / B_local -> / B_global (1 without sharding)
            total = total + (t * w if w != 1 else t)
            if monitor_divergence:
                div_sum = div_sum + (d * w if w != 1 else d)
    if world > 1 and shard:
        sums = torch.stack([total, div_sum])
        dist.all_reduce(sums, group=process_group)
        total, div_sum = sums[0], sums[1]
    return total, div_sum, nb


def train(model: models.EncodeProcessDecode, train_store: DeviceGraphStore, test_store: DeviceGraphStore,
          epochs: int, batch_size: int, learning_rate: float = 0.001, weights_folder: str = "",
          early_stopping_limit: int = 10, optimize_divergence: bool = True, divergence_penalty: float = 1.0,
          train_all_epochs: bool = False, monitor_divergence_in_test: bool = False,
          log=print, loaders=None, process_group=None, dp_mode: str = "replica") -> tuple[list[float], list[float]]:
    """gnn_train.py:95-305 (without TensorBoard).  ``loaders``: the (train, test) index loaders
    (make_loaders; built here when omitted).  ``process_group``: graph-batch data parallelism over
    its ranks (module docstring; every rank calls this with the same arguments, rank 0 writes)."""
    train_loader, test_loader = loaders if loaders is not None else make_loaders(train_store, test_store, batch_size)
    pg = process_group
    world = dist.get_world_size(pg) if pg is not None else 1
    rank = dist.get_rank(pg) if pg is not None else 0
    writer = rank == 0
    trainer = Trainer(model, lr=learning_rate, divergence=optimize_divergence,
                      divergence_penalty=divergence_penalty, process_group=pg, dp_mode=dp_mode)
    folder = Path(weights_folder)
    if writer:
        folder.mkdir(parents=True, exist_ok=False)
    best_path = folder / "model_weights.pth"
    last_path = folder / "last_epoch_model_weights.pth"
    log(f"Device = {train_store.device};\nBatch size = {batch_size};\nLearning rate = {learning_rate};\n"
        f"Epochs = {epochs};\nWeights path = {best_path.absolute()};\nOptimize divergence = {optimize_divergence};\n"
        f"Divergence lamba = {divergence_penalty};\nEarly stopping limit = {early_stopping_limit};")
    best_loss = sys.float_info.max
    train_losses: list[float] = []
    test_losses: list[float] = []
    early_stopping_counter = 0
    epoch = -1
    dev = train_store.device
    for epoch in range(epochs):
        if not train_all_epochs and early_stopping_counter >= early_stopping_limit:
            log("Training early stopped")
            break
        model.train()
        nmse_sum = torch.zeros((), dtype=torch.float32, device=dev)
        div_sum = torch.zeros((), dtype=torch.float32, device=dev)
        total_sum = torch.zeros((), dtype=torch.float32, device=dev)
        n_train = 0
        for idx in train_loader:
            if world == 1:
                out = trainer.step(train_store.batch(idx))
            elif dp_mode == "sync" and not sync_shardable(idx, train_store, world):
                # a shard would be empty or edgeless (e.g. the epoch's last minibatch holds fewer graphs than
                # ranks): rank 0 steps on the whole minibatch, the others contribute zeros (Trainer.step solo)
                out = trainer.step(train_store.batch(idx) if rank == 0 else None, n_global_graphs=len(idx),
                                   solo=True)
            else:   # this rank's share of the reference-ordered global minibatch, losses / B_global
                mine = shard_minibatch(idx, train_store.n, world, rank)
                out = trainer.step(train_store.batch(mine) if mine else None, n_global_graphs=len(idx))
            nmse_sum = nmse_sum + out["nmse"]
            total_sum = total_sum + out["total"]
            if optimize_divergence:
                div_sum = div_sum + out["div"]
            n_train += 1
        model.eval()
        test_total, test_div, n_test = evaluate(model, test_store, test_loader, monitor_divergence_in_test,
                                                process_group=pg, shard=dp_mode == "replica")
        # one host sync per epoch (the reference's .item() calls, gnn_train.py:258-275)
        vals = torch.stack([nmse_sum, total_sum, div_sum, test_total, test_div]).tolist()
        train_mse_loss = vals[0] / n_train
        total_loss = vals[1] / n_train
        test_loss = vals[3] / n_test
        if test_loss < best_loss:   # the same decision on every rank: the losses are global
            if writer:
                models.save_model_checkpoint(model, trainer, epoch + 1, best_path.as_posix())
                log(f"Checkpoint saved at {best_path}")
            best_loss = test_loss
            early_stopping_counter = 0
        else:
            early_stopping_counter += 1
        msg = (f"Epoch: {epoch + 1} / {epochs}, \nTotal train Loss : {total_loss}\nMSE train Loss : "
               f"{train_mse_loss} \nTest Loss : {test_loss}")
        if optimize_divergence:
            msg += f"\nDivergence term train {vals[2] / n_train}"
        if monitor_divergence_in_test:
            msg += f"\nDivergence test value {vals[4] / n_test}"
        log(msg)
        train_losses.append(total_loss)
        test_losses.append(test_loss)
    if writer:
        models.save_model_checkpoint(model, trainer, epoch + 1, last_path.as_posix())
        log(f"Last checkpoint at epoch {epoch + 1} saved at {last_path}")
    return train_losses, test_losses


def run_experience(dataset_train_csv: str, dataset_test_csv: str, results_folder: str, epochs: int,
                   batch_size: int, divergence: bool, latent_size: int, divergence_penalty: float,
                   early_stopping_limit: int, learning_rate: float, message_passing_steps: int,
                   train_all_epochs: bool = False, device: str = "cuda", periodic_graph: bool = True,
                   monitor_divergence_in_test: bool = False, config_path: Path = Path(""), *args: Any,
                   log=print, process_group=None, dp_mode: str = "replica",
                   **kwargs: Any) -> tuple[list[float], list[float]]:
    """gnn_train.py:331-435.  ``process_group``: graph-batch data parallelism (module docstring);
    every rank builds the same datasets and loaders, only rank 0 logs and writes."""
    import pandas as pd
    if process_group is not None and dist.get_rank(process_group) != 0:
        log = _quiet
    log(f"DATASET TRAIN CSV {dataset_train_csv}\nDATASET TEST CSV {dataset_test_csv}\nEPOCHS {epochs}\n"
        f"BATCH SIZE {batch_size}\nLEARNING RATE {learning_rate}\nPeriodic graph {periodic_graph}")
    torch.manual_seed(SEED)
    random.seed(SEED)
    np.random.seed(SEED)
    train_df = pd.read_csv(dataset_train_csv)
    test_df = pd.read_csv(dataset_test_csv)
    log(f"Size train dataset {len(train_df)}\nSize test dataset {len(test_df)}\nLoading datasets...")
    train_dataset = datasets.MeshStressFieldDatasetInMemory(train_df, periodic_graph=periodic_graph)
    # the reference builds the test set with the default periodic_graph=True (gnn_train.py:386;
    # reproduced, not "fixed")
    test_dataset = datasets.MeshStressFieldDatasetInMemory(test_df)
    train_store = DeviceGraphStore(train_dataset.graphs, device)
    test_store = DeviceGraphStore(test_dataset.graphs, device)
    model = models.EncodeProcessDecode(
        input_edges_features_size=1, input_nodes_features_size=6, message_passing_steps=message_passing_steps,
        latent_size=latent_size, output_nodes_features_size=3,
        **{k: v.to(device) for k, v in train_dataset.stats().items()})
    loaders = make_loaders(train_store, test_store, batch_size)
    log(models.print_model(model, loaders[0], device))   # every rank: it draws from the loader's RNG
    model.to(device)
    results = Path(results_folder)
    writer = process_group is None or dist.get_rank(process_group) == 0
    if writer:
        results.mkdir(parents=True, exist_ok=True)
        if config_path and Path(config_path).is_file():
            shutil.copyfile(config_path, results / Path(config_path).name)
    return train(model=model, train_store=train_store, test_store=test_store, epochs=epochs,
                 batch_size=batch_size, learning_rate=learning_rate,
                 weights_folder=(results / "weights").as_posix(), early_stopping_limit=early_stopping_limit,
                 optimize_divergence=divergence, divergence_penalty=divergence_penalty,
                 train_all_epochs=train_all_epochs, monitor_divergence_in_test=monitor_divergence_in_test,
                 log=log, loaders=loaders, process_group=process_group, dp_mode=dp_mode)


def _quiet(*_a, **_k) -> None:
    """The log of ranks other than 0."""


def init_distributed(device: str = "cuda"):
    """(process group, device) for a torchrun launch (WORLD_SIZE > 1): one process per GPU,
    ``cuda:LOCAL_RANK``, backend RCCL ("nccl") unless PDG_DIST_BACKEND names another (gloo rehearses
    several ranks on one GPU).  (None, device) for a single process."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return None, device
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    local = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    idx = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(idx)
    dev = torch.device("cuda", idx)
    backend = os.environ.get("PDG_DIST_BACKEND", "nccl")
    if not dist.is_initialized():
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    return dist.group.WORLD, dev


def main(config_path: str, **overrides: Any):
    """gnn_train.py:438-...: read the YAML config and run the experience (under torchrun: graph-batch
    data parallelism over the launched ranks; ``dp_mode`` "replica" or "sync" may be given as an
    override or a config key)."""
    import yaml
    with open(config_path) as f:
        params = yaml.safe_load(f)
    params.update(overrides)
    params["config_path"] = Path(config_path)
    if "process_group" not in params:
        pg, dev = init_distributed(params.get("device", "cuda"))
        if pg is not None:
            params["process_group"], params["device"] = pg, dev
    return run_experience(**params)


if __name__ == "__main__":
    main(sys.argv[1])
