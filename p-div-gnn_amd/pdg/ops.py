"""torch.library registration of the HIP path (the autograd entry points of the
boundary as ``torch.library`` custom ops).

    torch.ops.pdivgnn.epd_forward(params, stats8, pos, mean_stress, nodes_types, edge_attr,
                                  edge_index, num_nodes, steps, scale_input, scale_output,
                                  need_grad, engine) -> (local_stress, handle)
    torch.ops.pdivgnn.epd_backward(handle, grad_local_stress, params, std_local_stress)
                                  -> [grad of each parameter]
    torch.ops.pdivgnn.batch_loss(pred, gt, ptr, types, a_rowptr, a_col, a_val, at_rowptr,
                                 at_row, at_comp, at_val, with_nmse, divergence, penalty,
                                 reduce_abs) -> (total, nmse, div)

``epd_forward`` is ``EncodeProcessDecode.forward`` (gnn_local_stress/models.py:288-326) on the
tensors of a (batched) mesh graph, ``params`` in state_dict order (pdg.engine.PARAM_NAMES),
``stats8`` the eight standardisation scalars (models.py:99-138), ``engine`` the key of the
executor to run on (ops.register_engine; 0 = a shared executor per device).  With ``need_grad`` the
activations the backward needs stay on the device behind ``handle`` (an int64 key); autograd
(registered below) hands it to ``epd_backward``, and the activations are released when the
handle tensor dies (after the backward, or with the graph when no backward runs).
``batch_loss`` is gnn_train.py:168-197 fused (normalized_mse_loss_single summed over the
graphs / B, plus penalty * compute_divergence summed / B), with the divergence operator in the
CSR / CSR^T form of pdg.plan.GraphPlan.  ``register_fake`` gives both ops shapes for tracing.

``EncodeProcessDecode.forward`` and ``gnn_local_stress.losses.batch_loss`` call these ops, so
the reference's training loop reaches the kernels through the torch dispatcher.
"""
from __future__ import annotations

import itertools
import weakref
from typing import List, Optional

import torch
from torch import Tensor

from .engine import PARAM_NAMES, EPDEngine
from .lib import lib, stream_handle
from .plan import GraphPlan

_engines: dict = {}              # engine key -> EPDEngine (0: the shared engine of a device, by name)
_ctx: dict = {}                  # handle key -> (engine, forward context: activations on the device)
_keys = itertools.count(1)
_engine_keys = itertools.count(1)
_plans: dict = {}                # id(edge_index) -> (weakref, num_nodes, version, GraphPlan)


def register_engine(engine: EPDEngine, owner=None) -> int:
    """Key under which the ops find ``engine`` (a model's own executor: its scratch buffers and
    data-parallel settings stay its own).  With ``owner`` (the model) the registration ends when
    the owner is garbage collected, so the engine's device scratch is freed with the model; a
    pending backward keeps its engine alive through its saved context."""
    key = next(_engine_keys)
    _engines[key] = engine
    if owner is not None:
        weakref.finalize(owner, unregister_engine, key)
    return key


def unregister_engine(key: int) -> None:
    _engines.pop(key, None)


def engine_for(device, key: int = 0) -> EPDEngine:
    if key:
        return _engines[key]
    name = str(torch.device(device))
    if name not in _engines:
        _engines[name] = EPDEngine(torch.device(device))
    return _engines[name]


def plan_of(edge_index: Tensor, num_nodes: int) -> GraphPlan:
    """The edge plan of ``edge_index``, built once per tensor object and dropped with it (a
    freed tensor's address or id can be reused by the next batch, its weakref cannot)."""
    k = id(edge_index)
    hit = _plans.get(k)
    if hit is not None and hit[0]() is edge_index and hit[1] == num_nodes and hit[2] == edge_index._version:
        return hit[3]
    plan = GraphPlan(edge_index, num_nodes)
    ref = weakref.ref(edge_index, lambda _r, k=k: _plans.pop(k, None))
    _plans[k] = (ref, num_nodes, edge_index._version, plan)
    return plan


def register_plan(edge_index: Tensor, plan: GraphPlan) -> None:
    """Seed the cache with a plan built elsewhere (pdg.plan.plan_for on the batch object)."""
    k = id(edge_index)
    ref = weakref.ref(edge_index, lambda _r, k=k: _plans.pop(k, None))
    _plans[k] = (ref, plan.n_nodes, edge_index._version, plan)


def _release(key: int) -> None:
    _ctx.pop(key, None)


# ----------------------------------------------------------------------------- model
@torch.library.custom_op("pdivgnn::epd_forward", mutates_args=())
def epd_forward(params: List[Tensor], stats8: Tensor, pos: Tensor, mean_stress: Tensor, nodes_types: Tensor,
                edge_attr: Tensor, edge_index: Tensor, num_nodes: int, steps: int, scale_input: bool,
                scale_output: bool, need_grad: bool, engine: int) -> tuple[Tensor, Tensor]:
    dev = pos.device
    if dev.type != "cuda":
        raise RuntimeError("pdivgnn::epd_forward runs on a HIP device only (the CPU restatement is oracle/)")
    plan = plan_of(edge_index, num_nodes)
    P = dict(zip(PARAM_NAMES, params))
    eng = engine_for(dev, engine)
    y, fctx = eng.forward(P, stats8, plan, pos.float().contiguous(), mean_stress.float().contiguous(),
                                      nodes_types.reshape(-1).to(torch.int64).contiguous(),
                                      edge_attr.reshape(-1).float().contiguous(), steps, scale_input, scale_output,
                                      need_grad)
    key = next(_keys) if need_grad else 0
    handle = torch.tensor([key], dtype=torch.int64)
    if need_grad:
        _ctx[key] = (eng, fctx)
        weakref.finalize(handle, _release, key)
    return y, handle


@epd_forward.register_fake
def _(params, stats8, pos, mean_stress, nodes_types, edge_attr, edge_index, num_nodes, steps, scale_input,
      scale_output, need_grad, engine):
    return pos.new_empty((num_nodes, 3)), torch.empty(1, dtype=torch.int64)


@torch.library.custom_op("pdivgnn::epd_backward", mutates_args=())
def epd_backward(handle: Tensor, grad_local_stress: Tensor, params: List[Tensor],
                 std_local_stress: Tensor) -> List[Tensor]:
    key = int(handle[0])
    eng, fctx = _ctx.pop(key, (None, None))
    if fctx is None:
        raise RuntimeError("pdivgnn::epd_backward: no saved forward for this handle (forward ran without "
                           "need_grad, or its backward already ran)")
    P = dict(zip(PARAM_NAMES, params))
    if fctx.scale_output:
        P["_std_local_stress"] = std_local_stress
    G = {n: torch.zeros_like(p) for n, p in zip(PARAM_NAMES, params)}
    eng.backward(P, fctx, grad_local_stress, G)
    return [G[n] for n in PARAM_NAMES]


@epd_backward.register_fake
def _(handle, grad_local_stress, params, std_local_stress):
    return [torch.empty_like(p) for p in params]


def _epd_setup(ctx, inputs, output):
    params = inputs[0]
    ctx.save_for_backward(output[1], inputs[1], *params)


def _epd_bwd(ctx, g_y, _g_handle):
    handle, stats8, *params = ctx.saved_tensors
    grads = torch.ops.pdivgnn.epd_backward(handle, g_y.contiguous(), list(params), stats8[5:6])
    return (list(grads),) + (None,) * 12


torch.library.register_autograd("pdivgnn::epd_forward", _epd_bwd, setup_context=_epd_setup)


# ----------------------------------------------------------------------------- losses
@torch.library.custom_op("pdivgnn::batch_loss", mutates_args=())
def batch_loss_op(pred: Tensor, gt: Optional[Tensor], ptr: Tensor, types: Optional[Tensor],
                  a_rowptr: Optional[Tensor], a_col: Optional[Tensor], a_val: Optional[Tensor],
                  at_rowptr: Optional[Tensor], at_row: Optional[Tensor], at_comp: Optional[Tensor],
                  at_val: Optional[Tensor], with_nmse: bool, divergence: bool, penalty: float,
                  reduce_abs: bool) -> tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """Returns (total, nmse, div, den, divf): den (B, 3) and divf (N, 2) are the residuals the
    backward needs (empty when unused).  at_* (the operator transposed, grouped by node) are
    read by the backward only."""
    if pred.device.type != "cuda":
        raise RuntimeError("pdivgnn::batch_loss runs on a HIP device only (the CPU restatement is oracle/)")
    s = stream_handle(pred.device)
    B, N = ptr.numel() - 1, pred.shape[0]
    pred = pred.float().contiguous()
    f32 = dict(dtype=torch.float32, device=pred.device)
    nmse = torch.zeros((), **f32)
    den = torch.empty(0, **f32)
    if with_nmse:
        gt = gt.float().contiguous()
        loss_g, den = torch.empty(B, **f32), torch.empty(B, 3, **f32)
        lib.pdg_nmse_fwd(B, ptr.data_ptr(), gt.data_ptr(), pred.data_ptr(), loss_g.data_ptr(), den.data_ptr(), s)
        nmse = loss_g.sum() / B
    div_tot = torch.zeros((), **f32)
    divf = torch.empty(0, **f32)
    if divergence:
        if a_rowptr is None:
            raise ValueError("batch has no divergence operator")
        types = types.reshape(-1).to(torch.int64).contiguous()
        divf = torch.empty(N, 2, **f32)
        loss_d = torch.empty(B, **f32)
        lib.pdg_div_fwd(B, ptr.data_ptr(), a_rowptr.data_ptr(), a_col.data_ptr(), a_val.data_ptr(),
                        types.data_ptr(), pred.data_ptr(), int(reduce_abs), divf.data_ptr(), loss_d.data_ptr(), s)
        div_tot = (loss_d * penalty).sum() / B
    return nmse + div_tot, nmse.clone(), div_tot.clone(), den, divf


@batch_loss_op.register_fake
def _(pred, gt, ptr, types, a_rowptr, a_col, a_val, at_rowptr, at_row, at_comp, at_val, with_nmse, divergence,
      penalty, reduce_abs):
    B, N = ptr.shape[0] - 1, pred.shape[0]
    return (pred.new_empty(()), pred.new_empty(()), pred.new_empty(()),
            pred.new_empty((B, 3) if with_nmse else (0,)), pred.new_empty((N, 2) if divergence else (0,)))


@torch.library.custom_op("pdivgnn::batch_loss_backward", mutates_args=())
def batch_loss_backward(g_total: Tensor, g_nmse: Tensor, g_div: Tensor, pred: Tensor, gt: Optional[Tensor],
                        ptr: Tensor, den: Tensor, divf: Tensor, at_rowptr: Optional[Tensor],
                        at_row: Optional[Tensor], at_comp: Optional[Tensor], at_val: Optional[Tensor],
                        penalty: float, reduce_abs: bool) -> Tensor:
    """d(loss)/d(pred) for upstream gradients of all three scalar outputs: total = nmse + div, so
    the NMSE term's gradient is scaled by g_total + g_nmse and the divergence term's by
    g_total + g_div (a caller may back-propagate nmse and div separately, as the reference's
    batch_loss and batch_divergence_loss are separate tensors, gnn_train.py:168-197)."""
    s = stream_handle(pred.device)
    B, N = ptr.numel() - 1, pred.shape[0]
    pred = pred.float().contiguous()
    gt_all = g_total.float().reshape(1)
    gp = torch.zeros_like(pred)
    if den.numel():
        gt = gt.float().contiguous()
        scale = ((gt_all + g_nmse.float().reshape(1)) / B).contiguous()
        lib.pdg_nmse_bwd(B, ptr.data_ptr(), N, gt.data_ptr(), pred.data_ptr(), den.data_ptr(), scale.data_ptr(), 0,
                         gp.data_ptr(), s)
    if divf.numel():
        sd = ((gt_all + g_div.float().reshape(1)) * (penalty / B)).contiguous()
        lib.pdg_div_bwd(B, ptr.data_ptr(), N, at_rowptr.data_ptr(), at_row.data_ptr(), at_comp.data_ptr(),
                        at_val.data_ptr(), divf.data_ptr(), sd.data_ptr(), int(reduce_abs), 1, gp.data_ptr(), s)
    return gp


@batch_loss_backward.register_fake
def _(g_total, g_nmse, g_div, pred, gt, ptr, den, divf, at_rowptr, at_row, at_comp, at_val, penalty, reduce_abs):
    return torch.empty_like(pred)


def _loss_setup(ctx, inputs, output):
    pred, gt, ptr = inputs[0], inputs[1], inputs[2]
    ctx.penalty, ctx.reduce_abs = inputs[13], inputs[14]
    ctx.has_gt = gt is not None
    ctx.has_at = inputs[7] is not None
    at = tuple(inputs[7:11]) if ctx.has_at else ()
    ctx.save_for_backward(pred, ptr, output[3], output[4], *((gt,) if ctx.has_gt else ()), *at)


def _loss_bwd(ctx, g_total, g_nmse, g_div, _g_den, _g_divf):
    pred, ptr, den, divf, *rest = ctx.saved_tensors
    gt = rest.pop(0) if ctx.has_gt else None
    at = rest if ctx.has_at else [None, None, None, None]
    zero = torch.zeros((), dtype=torch.float32, device=pred.device)
    g_total, g_nmse, g_div = (zero if g is None else g for g in (g_total, g_nmse, g_div))
    gp = torch.ops.pdivgnn.batch_loss_backward(g_total, g_nmse, g_div, pred, gt, ptr, den, divf, *at, ctx.penalty,
                                               ctx.reduce_abs)
    return (gp,) + (None,) * 14


torch.library.register_autograd("pdivgnn::batch_loss", _loss_bwd, setup_context=_loss_setup)
