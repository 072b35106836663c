"""Training losses of scripts/gnn_train.py:41-92 on the HIP kernels.

* ``normalized_mse_loss_single`` / ``compute_divergence``: the reference's
  per-graph functions, same signatures and error behaviour;
* ``batch_loss``: the whole per-graph loop of gnn_train.py:168-197 fused into
  two segmented kernels over the batch's ``ptr`` (no Python loop, no dense
  operator), returning (total, nmse, div) with nmse/div already / batch_size.
"""
from __future__ import annotations

import torch

from pdg.lib import lib, stream_handle
from pdg.plan import GraphPlan, plan_for


def _check_dev(t: torch.Tensor) -> None:
    if t.device.type != "cuda":
        raise RuntimeError("HIP losses need tensors on a HIP device (the CPU restatement is test-only, oracle/)")


class _BatchLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, gt, plan: GraphPlan, types, with_nmse: bool, divergence: bool, penalty: float,
                reduce_abs: bool):
        _check_dev(pred)
        s = stream_handle(pred.device)
        B, N = plan.n_graphs, plan.n_nodes
        pred = pred.float().contiguous()
        f32 = dict(dtype=torch.float32, device=pred.device)
        nmse = torch.zeros((), **f32)
        den = None
        if with_nmse:
            gt = gt.float().contiguous()
            loss_g, den = torch.empty(B, **f32), torch.empty(B, 3, **f32)
            lib.pdg_nmse_fwd(B, plan.ptr.data_ptr(), gt.data_ptr(), pred.data_ptr(), loss_g.data_ptr(),
                             den.data_ptr(), s)
            nmse = loss_g.sum() / B
        div_tot = torch.zeros((), **f32)
        div = None
        if divergence:
            if not plan.has_div:
                raise ValueError("batch has no divergence operator")
            types = types.reshape(-1).to(torch.int64).contiguous()
            div = torch.empty(N, 2, **f32)
            loss_d = torch.empty(B, **f32)
            lib.pdg_div_fwd(B, plan.ptr.data_ptr(), plan.a_rowptr.data_ptr(), plan.a_col.data_ptr(),
                            plan.a_val.data_ptr(), types.data_ptr(), pred.data_ptr(), int(reduce_abs),
                            div.data_ptr(), loss_d.data_ptr(), s)
            div_tot = (loss_d * penalty).sum() / B
        ctx.save_for_backward(pred)
        ctx.gt, ctx.den = gt, den
        ctx.div = div
        ctx.plan, ctx.penalty, ctx.reduce_abs = plan, penalty, reduce_abs
        nd, dd = nmse.detach().clone(), div_tot.detach().clone()
        ctx.mark_non_differentiable(nd, dd)
        return nmse + div_tot, nd, dd

    @staticmethod
    def backward(ctx, g_total, _g1, _g2):
        (pred,) = ctx.saved_tensors
        gt, den = ctx.gt, ctx.den
        plan = ctx.plan
        s = stream_handle(pred.device)
        B, N = plan.n_graphs, plan.n_nodes
        scale = (g_total.float() / B).reshape(1).contiguous()
        gp = torch.zeros_like(pred)
        if den is not None:
            lib.pdg_nmse_bwd(B, plan.ptr.data_ptr(), N, gt.data_ptr(), pred.data_ptr(), den.data_ptr(),
                             scale.data_ptr(), 0, gp.data_ptr(), s)
        if ctx.div is not None:
            sd = (scale * ctx.penalty).contiguous()
            lib.pdg_div_bwd(B, plan.ptr.data_ptr(), N, plan.at_rowptr.data_ptr(), plan.at_row.data_ptr(),
                            plan.at_comp.data_ptr(), plan.at_val.data_ptr(), ctx.div.data_ptr(), sd.data_ptr(),
                            int(ctx.reduce_abs), 1, gp.data_ptr(), s)
        return gp, None, None, None, None, None, None, None


def batch_loss(pred: torch.Tensor, batch, gt_std: torch.Tensor, divergence: bool = False,
               divergence_penalty: float = 1.0, reduce_strategy: str = "square"):
    """Fused gnn_train.py:168-197: returns (total, nmse/B, lambda*div/B)."""
    if reduce_strategy not in ("abs", "square"):
        raise AttributeError("reduce_strategy must be 'abs' or 'square'")
    plan = plan_for(batch)
    types = batch.surfaces_nodes_for_div if batch.surfaces_nodes_for_div is not None else batch.nodes_types
    return _BatchLoss.apply(pred, gt_std, plan, types, True, bool(divergence), float(divergence_penalty),
                            reduce_strategy == "abs")


def normalized_mse_loss_single(ground_truth_local_stress: torch.Tensor,
                               predicted_local_stress: torch.Tensor) -> torch.Tensor:
    """gnn_train.py:41-57 on one graph."""
    n = predicted_local_stress.shape[0]
    plan = _SinglePlan.get(n, predicted_local_stress.device)
    total, _, _ = _BatchLoss.apply(predicted_local_stress, ground_truth_local_stress, plan, None, True, False, 1.0,
                                   False)
    return total


class _SinglePlan:
    """Minimal plan for single-graph loss calls (ptr = [0, n], optional operator)."""

    _cache: dict = {}

    @classmethod
    def get(cls, n: int, device, op=None) -> GraphPlan:
        p = GraphPlan.__new__(GraphPlan)
        p.n_nodes, p.n_edges, p.n_graphs = n, 0, 1
        p.ptr = torch.tensor([0, n], dtype=torch.int32, device=device)
        p.has_div = False
        if op is not None:
            op = op.coalesce()
            idx = op.indices().to(device)
            p.has_div = True
            GraphPlan._build_div(p, idx[0], idx[1], op.values().to(device).float())
        return p


def compute_divergence(local_stress_field: torch.Tensor, op_div_matrix: torch.Tensor,
                       surface_nodes_ids: torch.Tensor, reduce_strategy: str = "square") -> torch.Tensor:
    """gnn_train.py:60-92 on one graph: mean over rows of |A[:, :2N] S|^2 (boundary rows
    zeroed), summed over the 2 components.  Sparse CSR instead of ``to_dense``."""
    if reduce_strategy not in ("abs", "square"):
        raise AttributeError("reduce_strategy must be 'abs' or 'square'")
    n = local_stress_field.shape[0]
    plan = _SinglePlan.get(n, local_stress_field.device, op_div_matrix)
    total, _, _ = _BatchLoss.apply(local_stress_field, None, plan, surface_nodes_ids, False, True, 1.0,
                                   reduce_strategy == "abs")
    return total
