"""Drop-in ``gnn_local_stress.models`` backed by the MI355X HIP kernels.

Mirrors the reference module's public surface (gnn_local_stress/models.py):

* ``StressFieldBaseModel`` (:98-179): same constructor keywords, the 8 scalar
  standardisation statistics as plain attributes moved by ``.to()`` (:164-179),
  ``format_node_features`` / ``format_edge_features`` (:140-162);
* ``Processor`` (:182-243): ``edge_net`` / ``node_net`` Sequentials with the
  same parameter names, so ``state_dict`` keys match and reference ``.pth``
  checkpoints load unchanged;
* ``EncodeProcessDecode`` (:246-326): same constructor and
  ``forward(mesh_graph, scale_output=True, scale_input=True) -> Data`` with
  ``local_stress``, ``edge_index``, ``pos``;
* checkpoint helpers (:44-95) with the same dict keys.

``forward`` on a HIP device runs the whole stack through libpdivgnn_hip.so
(pdg.engine) as the ``torch.ops.pdivgnn.epd_forward`` custom op (pdg.ops), whose
registered autograd backward is the HIP backward.  There is no silent fallback:
on a CPU tensor the call raises (the CPU path of this repo is the test oracle,
not product).
"""
from __future__ import annotations

from abc import ABC
from typing import Optional

import torch
from torch.nn import Linear, Sequential

from pdg import ops
from pdg.engine import PARAM_NAMES, EPDEngine
from pdg.graph import Data
from pdg.plan import plan_for

_STAT_ORDER = ("mean_pos", "std_pos", "mean_mean_stress", "std_mean_stress", "mean_local_stress",
               "std_local_stress", "mean_edge_weight", "std_edge_weight")


class GraphLayerNorm(torch.nn.Module):
    """torch_geometric ``LayerNorm(C)`` in its default ``mode="graph"`` with ``batch=None``:
    ``(x - x.mean()) / (x.std(unbiased=False) + eps) * weight + bias`` over the whole input.
    Parameters ``weight`` (ones) and ``bias`` (zeros) as in PyG, so state_dict keys match."""

    def __init__(self, in_channels: int, eps: float = 1e-5) -> None:
        super().__init__()
        self.in_channels = in_channels
        self.eps = eps
        self.weight = torch.nn.Parameter(torch.ones(in_channels))
        self.bias = torch.nn.Parameter(torch.zeros(in_channels))

    def forward(self, x: torch.Tensor, batch: Optional[torch.Tensor] = None) -> torch.Tensor:
        if batch is not None:
            raise NotImplementedError("per-graph LayerNorm (batch=...) is not used by the reference model")
        x = x - x.mean()
        out = x / (x.std(unbiased=False) + self.eps)
        return out * self.weight + self.bias

    def extra_repr(self) -> str:
        return f"{self.in_channels}, mode=graph"


def print_model(model: torch.nn.Module, data_loader, device: str) -> str:
    """models.py:33-41 (PyG ``summary`` is unavailable): a parameter table.  Like the reference it
    takes one minibatch from a fresh iterator of ``data_loader`` (when given), so the global-RNG
    draws of that iterator (base seed, sampler seed) happen here too and the training epochs that
    follow see the reference's shuffles."""
    if data_loader is not None:
        next(iter(data_loader))
    lines = [f"{type(model).__name__}  (parameters: {sum(p.numel() for p in model.parameters()):,})"]
    for name, p in model.named_parameters():
        lines.append(f"  {name:40s} {tuple(p.shape)}")
    return "\n".join(lines)


def save_model_checkpoint(model: torch.nn.Module, optimizer: torch.optim.Optimizer, epoch: int,
                          filename: str) -> None:
    """models.py:44-63 — identical checkpoint dict."""
    ckpt = {"model_state_dict": model.state_dict(), "optimizer_state_dict": optimizer.state_dict(),
            "epoch": epoch}
    for k in ("mean_pos", "mean_mean_stress", "std_mean_stress", "mean_local_stress", "std_pos",
              "std_local_stress", "mean_edge_weight", "std_edge_weight"):
        ckpt[k] = getattr(model, k)
    torch.save(ckpt, filename)


def load_model_checkpoint(model: torch.nn.Module, filename: str,
                          optimizer: Optional[torch.optim.Optimizer] = None) -> int:
    """models.py:66-87.  Loads with ``weights_only=True`` (the checkpoint holds only
    tensors, ints and optimizer state)."""
    map_location = None if torch.cuda.is_available() else torch.device("cpu")
    ckpt = torch.load(filename, map_location=map_location, weights_only=True)
    model.load_state_dict(ckpt["model_state_dict"])
    if optimizer:
        optimizer.load_state_dict(ckpt["optimizer_state_dict"])
    for k in _STAT_ORDER:
        setattr(model, k, ckpt[k])
    return ckpt["epoch"]


def load_optimizer_checkpoint(optimizer: torch.optim.Optimizer, filename: str) -> torch.optim.Optimizer:
    """models.py:90-95."""
    ckpt = torch.load(filename, weights_only=True)
    optimizer.load_state_dict(ckpt["optimizer_state_dict"])
    return optimizer


class StressFieldBaseModel(torch.nn.Module, ABC):
    """models.py:98-179."""

    def __init__(self, latent_size: int, input_nodes_features_size: int, output_nodes_features_size: int,
                 mean_pos=torch.Tensor(1), std_pos=torch.Tensor(1), mean_mean_stress=torch.Tensor(1),
                 std_mean_stress=torch.Tensor(1), mean_local_stress=torch.Tensor(1),
                 std_local_stress=torch.Tensor(1), mean_edge_weight=torch.Tensor(1),
                 std_edge_weight=torch.Tensor(1)):
        super().__init__()
        self.latent_size = latent_size
        self.input_nodes_features_size = input_nodes_features_size
        self.output_nodes_features_size = output_nodes_features_size
        self.mean_pos = mean_pos
        self.std_pos = std_pos
        self.mean_mean_stress = mean_mean_stress
        self.std_mean_stress = std_mean_stress
        self.mean_local_stress = mean_local_stress
        self.std_local_stress = std_local_stress
        self.mean_edge_weight = mean_edge_weight
        self.std_edge_weight = std_edge_weight

    def format_node_features(self, mesh_graph, scale_data: bool) -> torch.Tensor:
        pos, mean_stress, nodes_types = mesh_graph.pos, mesh_graph.mean_stress, mesh_graph.nodes_types
        if scale_data:
            mean_stress = (mean_stress - self.mean_mean_stress) / self.std_mean_stress
            pos = (pos - self.mean_pos) / self.std_pos
        return torch.hstack([mean_stress, pos, nodes_types])

    def format_edge_features(self, mesh_graph, scale_data: bool) -> torch.Tensor:
        edge_attr = mesh_graph.edge_attr
        if scale_data:
            edge_attr = (edge_attr - self.mean_edge_weight) / self.std_edge_weight
        return edge_attr

    def to(self, device, *args, **kwargs) -> torch.nn.Module:
        for attr in _STAT_ORDER:
            value = getattr(self, attr)
            if value is not None:
                setattr(self, attr, value.to(device))
        return super().to(device, *args, **kwargs)


class Processor(torch.nn.Module):
    """models.py:182-243: the weight-shared message-passing block (parameters only;
    the fused HIP step in pdg.engine executes it)."""

    def __init__(self, latent_size: int, input_nodes_features_size: int, input_edges_features_size: int):
        super().__init__()
        self.latent_size = latent_size
        self.edge_net = Sequential(Linear(input_edges_features_size, latent_size), torch.nn.ReLU(),
                                   Linear(latent_size, latent_size), torch.nn.ReLU(), GraphLayerNorm(latent_size))
        self.node_net = Sequential(Linear(input_nodes_features_size, latent_size), torch.nn.ReLU(),
                                   Linear(latent_size, latent_size), torch.nn.ReLU(), GraphLayerNorm(latent_size))


class EncodeProcessDecode(StressFieldBaseModel):
    """models.py:246-326."""

    def __init__(self, input_edges_features_size: int, message_passing_steps: int, *args, **kwargs):
        super().__init__(*args, **kwargs)
        if self.latent_size != 128:
            raise ValueError("the HIP kernels are specialised for latent_size=128 (all reference configs)")
        self.message_passing_steps = message_passing_steps
        self.input_edges_features_size = input_edges_features_size
        L = self.latent_size
        self.node_encoder = Sequential(Linear(self.input_nodes_features_size, L), torch.nn.ReLU(), Linear(L, L),
                                       torch.nn.ReLU(), GraphLayerNorm(L))
        self.edge_encoder = Sequential(Linear(self.input_edges_features_size, L), torch.nn.ReLU(), Linear(L, L),
                                       torch.nn.ReLU(), GraphLayerNorm(L))
        self.processor = Processor(L, input_nodes_features_size=L * 2, input_edges_features_size=L * 3)
        self.node_decoder = Sequential(Linear(L, L), torch.nn.ReLU(), Linear(L, self.output_nodes_features_size))
        self._engines: dict = {}

    def _engine_for(self, device) -> EPDEngine:
        """This model's executor on ``device`` (its own scratch and data-parallel settings; the custom
        op finds it by the key ops.register_engine returns)."""
        key = str(device)
        if key not in self._engines:
            eng = EPDEngine(device)
            self._engines[key] = (ops.register_engine(eng, owner=self), eng)
        return self._engines[key][1]

    def stats_tensor(self, device) -> torch.Tensor:
        """The 8 dataset statistics as one fp32 tensor on `device` (pdg_format_inputs' operand).

        Cached while the statistics are unchanged (the same tensor objects at the same version
        counter, or equal Python scalars): rebuilding it took 8 host-to-device copies per training
        step.  Callers only read it."""
        key = [("d", str(device))]
        for k in _STAT_ORDER:
            v = getattr(self, k)
            key.append(("t", v, v._version) if isinstance(v, torch.Tensor) else ("s", float(v)))

        def same(a, b):
            if a[0] != b[0]:
                return False
            return (a[1] is b[1] and a[2] == b[2]) if a[0] == "t" else a[1] == b[1]

        c = self.__dict__.get("_stats_cache")
        if c is not None and all(same(a, b) for a, b in zip(c[0], key)):
            return c[1]
        out = self._build_stats_tensor(device)
        self.__dict__["_stats_cache"] = (key, out)
        return out

    def _build_stats_tensor(self, device) -> torch.Tensor:
        vals = []
        for k in _STAT_ORDER:
            v = torch.as_tensor(getattr(self, k), dtype=torch.float32)
            if v.numel() != 1:
                # the reference's datasets compute scalar statistics (datasets.py:283-291); the HIP
                # input formatting takes one scalar per statistic, never a silently truncated vector
                raise ValueError(f"{k} must be a scalar (got {tuple(v.shape)}); per-axis statistics are "
                                 "not supported by the HIP path")
            vals.append(v.reshape(1).to(device))
        return torch.cat(vals).contiguous()

    def forward(self, mesh_graph, scale_output: bool = True, scale_input: bool = True):
        dev = mesh_graph.pos.device
        if dev.type != "cuda":
            raise RuntimeError("EncodeProcessDecode runs on the MI355X HIP path only; move the batch to a HIP "
                               "device (the CPU restatement lives in oracle/ and is test-only)")
        if self.input_nodes_features_size != 6 or self.input_edges_features_size != 1 \
                or self.output_nodes_features_size != 3:
            raise ValueError("HIP path supports the reference feature sizes (6 node, 1 edge, 3 outputs)")
        ms = mesh_graph.mean_stress
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        from pdg.lib import lib, stream_handle
        lib.pdg_any_nonzero(ms.data_ptr(), ms.numel(), flag.data_ptr(), stream_handle(dev))
        if not bool(flag.item()):   # models.py:294-299 (same host sync as the reference's torch.any)
            return Data(local_stress=torch.zeros_like(ms), edge_index=mesh_graph.edge_index, pos=mesh_graph.pos)
        plan = plan_for(mesh_graph)
        ops.register_plan(mesh_graph.edge_index, plan)
        params = [self.get_parameter(n) for n in PARAM_NAMES]
        need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        if torch.is_grad_enabled() and any(t.requires_grad for t in (mesh_graph.pos, mesh_graph.mean_stress,
                                                                      mesh_graph.edge_attr)):
            # the reference never differentiates w.r.t. the mesh inputs (gnn_train.py:159-205); the
            # HIP backward produces parameter gradients only, so refuse rather than return None
            raise NotImplementedError("EncodeProcessDecode (HIP path): gradients w.r.t. pos / mean_stress / "
                                      "edge_attr are not supported; detach the inputs")
        # inference (gnn_inference.py runs under no_grad) keeps nothing for a backward
        self._engine_for(dev)
        y, _handle = torch.ops.pdivgnn.epd_forward(params, self.stats_tensor(dev), mesh_graph.pos, ms,
                                                   mesh_graph.nodes_types, mesh_graph.edge_attr,
                                                   mesh_graph.edge_index, plan.n_nodes, self.message_passing_steps,
                                                   bool(scale_input), bool(scale_output), need_grad,
                                                   self._engines[str(dev)][0])
        return Data(local_stress=y, edge_index=mesh_graph.edge_index, pos=mesh_graph.pos)
