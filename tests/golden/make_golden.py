"""Generate the golden fixtures in tests/golden/*.npz from the REFERENCE code.

Run in the build container only (needs /root/reference, never shipped):

    python tests/golden/make_golden.py

torch_geometric, pyvista, fedoo, fire and tensorboard are not installed, so a
minimal stand-in is registered in ``sys.modules`` before the reference is
imported.  The stand-in implements only what the hot path touches, following
PyG's documented semantics:

* ``MessagePassing.propagate`` (flow source->target, aggr="add"):
  x_i = x.index_select(0, edge_index[1]), x_j = x.index_select(0, edge_index[0]),
  message(...), zeros(N, C).scatter_add_(0, edge_index[1], msgs), update(aggr, x=x);
* ``nn.LayerNorm(C)`` mode="graph", batch=None: (x - x.mean()) / (x.std(unbiased=False) + eps) * w + b,
  weight=1 / bias=0 at init;
* ``data.Data`` attribute bag with ``coalesce()`` (sort by (row, col), sum duplicates);
* a ``Batch`` with ``batch``, ``__len__`` and ``__getitem__`` slicing.

The reference's own ``models.EncodeProcessDecode``, ``data_utils``,
``datasets.compute_periodic_graph``, ``datasets._compute_node_distances_as_edge_weights``
and ``gnn_train.normalized_mse_loss_single`` / ``compute_divergence`` are then run
unchanged on synthetic meshes (p-div-gnn_amd/pdg/meshgen.py) and their inputs,
parameters, outputs, losses and gradients are saved.  What these fixtures pin:
the reference's own glue (feature order, concat orders, weight sharing, residuals,
init order, loss formulas, periodic-edge construction).  What they do NOT pin:
PyG internals beyond the stand-in above ("Parity").
"""
from __future__ import annotations

import os
import sys
import types
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
REF = Path("/root/reference")
sys.path.insert(0, str(REPO / "p-div-gnn_amd"))

from pdg import meshgen  # noqa: E402  (input generator: data, not reference code)


# --------------------------------------------------------------------------- stand-ins
def _module(name: str) -> types.ModuleType:
    m = types.ModuleType(name)
    sys.modules[name] = m
    return m


class StubData:
    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)

    def __getattr__(self, k):
        if k.startswith("__"):
            raise AttributeError(k)
        return None

    @property
    def num_nodes(self):
        return self.pos.shape[0]

    @property
    def num_edges(self):
        return self.edge_index.shape[1]

    def coalesce(self):
        ei = self.edge_index
        n = self.num_nodes
        key = ei[0] * n + ei[1]
        uniq, inv = torch.unique(key, sorted=True, return_inverse=True)
        if self.edge_attr is not None:
            ea = torch.zeros(len(uniq), dtype=self.edge_attr.dtype)
            ea.index_add_(0, inv, self.edge_attr)
            self.edge_attr = ea
        self.edge_index = torch.stack([uniq // n, uniq % n])
        return self


class StubBatch(StubData):
    @classmethod
    def from_list(cls, graphs):
        b = cls()
        counts = [g.num_nodes for g in graphs]
        off = np.concatenate([[0], np.cumsum(counts)])
        for k in ("pos", "mean_stress", "local_stress", "nodes_types", "surfaces_nodes_for_div"):
            setattr(b, k, torch.cat([getattr(g, k) for g in graphs]))
        b.edge_attr = torch.cat([g.edge_attr for g in graphs])
        b.edge_index = torch.cat([g.edge_index + int(off[i]) for i, g in enumerate(graphs)], 1)
        b.batch = torch.repeat_interleave(torch.arange(len(graphs)), torch.tensor(counts))
        b._graphs = graphs
        b._off = off
        return b

    @property
    def batch_size(self):
        return len(self._graphs)

    def __len__(self):
        return len(self._graphs)

    def __getitem__(self, i):
        s, t = int(self._off[i]), int(self._off[i + 1])
        g = self._graphs[i]
        return StubData(local_stress=self.local_stress[s:t], op_div_matrix=g.op_div_matrix,
                        surfaces_nodes_for_div=self.surfaces_nodes_for_div[s:t])


class MessagePassing(torch.nn.Module):
    def __init__(self, aggr: str = "add"):
        super().__init__()
        assert aggr == "add"

    def propagate(self, edge_index, x, edge_attr):
        x_i = x.index_select(0, edge_index[1])
        x_j = x.index_select(0, edge_index[0])
        msg = self.message(x_i=x_i, x_j=x_j, edge_attr=edge_attr)
        out = msg.new_zeros(x.size(0), msg.size(1))
        out.scatter_add_(0, edge_index[1].view(-1, 1).expand_as(msg), msg)
        return self.update(out, x=x)


class LayerNorm(torch.nn.Module):
    def __init__(self, in_channels, eps=1e-5, affine=True, mode="graph"):
        super().__init__()
        self.eps = eps
        self.weight = torch.nn.Parameter(torch.ones(in_channels))
        self.bias = torch.nn.Parameter(torch.zeros(in_channels))

    def forward(self, x, batch=None):
        x = x - x.mean()
        out = x / (x.std(unbiased=False) + self.eps)
        return out * self.weight + self.bias


def install_stubs():
    pyg = _module("torch_geometric")
    for sub in ("data", "nn", "loader", "transforms", "utils"):
        m = _module(f"torch_geometric.{sub}")
        setattr(pyg, sub, m)
    pyg.data.Data = StubData
    pyg.data.Batch = StubBatch
    pyg.data.InMemoryDataset = type("InMemoryDataset", (), {})
    pyg.nn.MessagePassing = MessagePassing
    pyg.nn.LayerNorm = LayerNorm
    pyg.nn.summary = lambda *a, **k: ""
    pyg.loader.DataLoader = object
    pyg.transforms.BaseTransform = object
    pv = _module("pyvista")
    pv.start_xvfb = lambda: None
    pv.PolyData = pv.UnstructuredGrid = object
    _module("fedoo").Mesh = object
    fire = _module("fire")
    fire.Fire = lambda f: None
    tb = _module("torch.utils.tensorboard")
    tb.SummaryWriter = object


# --------------------------------------------------------------------------- generation
def reference_graph(sample: meshgen.MeshSample, periodic: bool, datasets):
    """Build one graph the way datasets.py:249-281 does, on a synthetic mesh."""
    n = sample.num_nodes
    e = np.concatenate([sample.faces[:, [0, 1]], sample.faces[:, [1, 2]], sample.faces[:, [0, 2]]], 0).T
    e = np.concatenate([e, e[::-1]], 1)
    g = StubData(pos=torch.from_numpy(np.concatenate([sample.pos, np.zeros((n, 1), np.float32)], 1)),
                 edge_index=torch.from_numpy(e), face=torch.from_numpy(sample.faces.T.copy()))
    g.coalesce()  # FaceToEdge + to_undirected coalesce
    g.edge_attr = datasets._compute_node_distances_as_edge_weights(g).float()
    if periodic:
        g = datasets.compute_periodic_graph(g)
    g.pos = g.pos[:, :2].float()
    g.mean_stress = torch.ones(n, 3) * torch.from_numpy(sample.mean_stress)
    g.local_stress = torch.from_numpy(sample.local_stress)
    g.op_div_matrix = datasets._init_op_div_matrix({
        "op_div_matrix_data": sample.op_div_vals, "op_div_matrix_col_indices": sample.op_div_cols,
        "op_div_matrix_row_indices": sample.op_div_rows, "op_div_matrix_shape": (n, 2 * n)})
    g.surfaces_nodes_for_div = torch.from_numpy(sample.node_types).unsqueeze(1)
    g.nodes_types = g.surfaces_nodes_for_div
    return g


def run_case(name: str, samples, periodic: bool, steps: int, divergence: bool, penalty: float,
             save_latents: bool, models, datasets, data_utils, gnn_train):
    graphs = [reference_graph(s, periodic, datasets) for s in samples]
    # generator's own graph construction must agree with the reference's
    for s, g in zip(samples, graphs):
        ei = s.edge_index if periodic else meshgen.faces_to_edges(s.faces, s.num_nodes)
        assert np.array_equal(g.edge_index.numpy(), ei), "periodic/coalesce mismatch"
        if periodic:
            assert np.array_equal(g.edge_attr.numpy(), s.edge_attr), "edge_attr mismatch"
    batch = StubBatch.from_list(graphs)
    # scalar standardisation constants, datasets.py:283-291 (over this "dataset")
    st = {
        "mean_pos": batch.pos.mean(), "std_pos": batch.pos.std(),
        "mean_mean_stress": batch.mean_stress.mean(), "std_mean_stress": batch.mean_stress.std(),
        "mean_local_stress": batch.local_stress.mean(), "std_local_stress": batch.local_stress.std(),
        "mean_edge_weight": batch.edge_attr.mean(), "std_edge_weight": batch.edge_attr.std(),
    }
    torch.manual_seed(gnn_train.SEED)
    model = models.EncodeProcessDecode(input_edges_features_size=1, input_nodes_features_size=6,
                                       message_passing_steps=steps, latent_size=128,
                                       output_nodes_features_size=3, **st)
    params = {k: v.detach().clone() for k, v in model.state_dict().items()}
    lat = []
    hook = model.processor.register_forward_hook(lambda m, i, o: lat.append((o.x.detach(), o.edge_attr.detach())))
    with torch.no_grad():
        out_scaled = model.forward(batch, scale_output=True, scale_input=True).local_stress
    hook.remove()
    # train-step body, scripts/gnn_train.py:159-205
    pred = model.forward(batch, scale_output=False, scale_input=True).local_stress
    gt = data_utils.standardize(batch.local_stress, model.mean_local_stress, model.std_local_stress)
    batch.local_stress = gt
    loss = 0
    div_loss = 0
    for sample_i, pred_i in data_utils.slice_batch_gt_and_predictions(batch, pred):
        loss = loss + gnn_train.normalized_mse_loss_single(
            ground_truth_local_stress=sample_i.local_stress, predicted_local_stress=pred_i)
        if divergence:
            div_loss = div_loss + gnn_train.compute_divergence(
                pred_i, sample_i.op_div_matrix, sample_i.surfaces_nodes_for_div,
                reduce_strategy="square") * penalty
    loss = loss / batch.batch_size
    nmse = loss.detach().clone()
    if divergence:
        div_loss = div_loss / batch.batch_size
        loss = loss + div_loss
    model.zero_grad()
    loss.backward()
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters()}

    counts = [g.num_nodes for g in graphs]
    ptr = np.concatenate([[0], np.cumsum(counts)])
    rec = {
        "steps": np.array(steps), "divergence": np.array(divergence), "penalty": np.array(penalty),
        "periodic": np.array(periodic), "ptr": ptr,
        "pos": batch.pos.numpy(), "mean_stress": batch.mean_stress.numpy(),
        "nodes_types": batch.nodes_types.numpy(), "edge_index": batch.edge_index.numpy(),
        "edge_attr": batch.edge_attr.numpy(), "local_stress": np.concatenate([s.local_stress for s in samples]),
        "out_scaled": out_scaled.numpy(), "pred": pred.detach().numpy(), "gt_std": gt.numpy(),
        "loss_total": loss.detach().numpy(), "loss_nmse": nmse.numpy(),
        "loss_div": (div_loss.detach().numpy() if divergence else np.array(0.0, np.float32)),
    }
    for i, g in enumerate(graphs):
        op = g.op_div_matrix.coalesce()
        rec[f"op_div_idx_{i}"] = op.indices().numpy()
        rec[f"op_div_val_{i}"] = op.values().numpy()
    for k, v in st.items():
        rec[f"stat.{k}"] = v.numpy()
    for k, v in params.items():
        rec[f"param.{k}"] = v.numpy()
    for k, v in grads.items():
        rec[f"grad.{k}"] = v.numpy()
    if save_latents:
        for t, (x, e) in enumerate(lat):
            rec[f"latent_x_{t}"] = x.numpy()
            rec[f"latent_e_{t}"] = e.numpy()
    np.savez_compressed(HERE / f"{name}.npz", **rec)
    print(f"{name}: N={batch.pos.shape[0]} E={batch.edge_index.shape[1]} B={len(graphs)} "
          f"loss={float(loss):.6f} nmse={float(nmse):.6f}")


def run_checkpoint_case(models, datasets, data_utils, gnn_train):
    """A checkpoint written by the reference's own save_model_checkpoint (models.py:44-63) after
    one training step of gnn_train.py:154-207 (Adam lr=1e-3; GradScaler is inactive on the CPU),
    plus what the reference computes from it: the forward after that step and the parameters
    after a second step on the same batch (the resume path of load_model_checkpoint /
    load_optimizer_checkpoint, models.py:66-95)."""
    samples = meshgen.make_dataset(3, n=13, hole_radius=(0.15, 0.3), seed=7)
    graphs = [reference_graph(s, True, datasets) for s in samples]
    batch = StubBatch.from_list(graphs)
    st = {
        "mean_pos": batch.pos.mean(), "std_pos": batch.pos.std(),
        "mean_mean_stress": batch.mean_stress.mean(), "std_mean_stress": batch.mean_stress.std(),
        "mean_local_stress": batch.local_stress.mean(), "std_local_stress": batch.local_stress.std(),
        "mean_edge_weight": batch.edge_attr.mean(), "std_edge_weight": batch.edge_attr.std(),
    }
    torch.manual_seed(gnn_train.SEED)
    model = models.EncodeProcessDecode(input_edges_features_size=1, input_nodes_features_size=6,
                                       message_passing_steps=3, latent_size=128,
                                       output_nodes_features_size=3, **st)
    optimizer = torch.optim.Adam(model.parameters(), lr=1e-3)
    gt_raw = batch.local_stress.clone()

    def train_step():
        pred = model.forward(batch, scale_output=False, scale_input=True).local_stress
        batch.local_stress = data_utils.standardize(gt_raw, model.mean_local_stress, model.std_local_stress)
        loss = 0
        div_loss = 0
        for sample_i, pred_i in data_utils.slice_batch_gt_and_predictions(batch, pred):
            loss = loss + gnn_train.normalized_mse_loss_single(
                ground_truth_local_stress=sample_i.local_stress, predicted_local_stress=pred_i)
            div_loss = div_loss + gnn_train.compute_divergence(
                pred_i, sample_i.op_div_matrix, sample_i.surfaces_nodes_for_div, reduce_strategy="square") * 10.0
        loss = loss / batch.batch_size + div_loss / batch.batch_size
        optimizer.zero_grad()
        loss.backward()
        optimizer.step()
        return float(loss)

    loss1 = train_step()
    models.save_model_checkpoint(model, optimizer, 1, str(HERE / "ref_checkpoint.pth"))
    with torch.no_grad():
        out1 = model.forward(batch, scale_output=True, scale_input=True).local_stress
    loss2 = train_step()
    rec = {"loss_step1": np.array(loss1), "loss_step2": np.array(loss2), "out_scaled_after_step1": out1.numpy()}
    for k, v in model.state_dict().items():
        rec[f"param_after_step2.{k}"] = v.numpy()
    np.savez_compressed(HERE / "ref_checkpoint_case.npz", **rec)
    print(f"ref_checkpoint: loss step1={loss1:.6f} step2={loss2:.6f}")


def main():
    install_stubs()
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
    sys.path.insert(0, str(REF))
    sys.path.insert(0, str(REF / "scripts"))
    torch.set_num_threads(1)
    from gnn_local_stress import data_utils, datasets, models  # reference package
    import gnn_train  # reference script module (scripts/gnn_train.py)

    mods = dict(models=models, datasets=datasets, data_utils=data_utils, gnn_train=gnn_train)
    run_case("tiny_periodic", [meshgen.hole_plate(9, seed=1)], True, 2, False, 10.0, True, **mods)
    run_case("batch3_div", meshgen.make_dataset(3, n=13, hole_radius=(0.15, 0.3), seed=7),
             True, 3, True, 10.0, False, **mods)
    run_case("single_no_periodic", [meshgen.hole_plate(12, hole_radius=0.25, periodic=False, seed=3)],
             False, 10, False, 10.0, False, **mods)
    run_case("batch2_div_s10", meshgen.make_dataset(2, n=11, hole_radius=(0.2, 0.3), seed=11),
             True, 10, True, 10.0, False, **mods)
    run_checkpoint_case(**mods)


if __name__ == "__main__":
    main()
