"""Training losses of scripts/gnn_train.py:41-92 on the HIP kernels.

* ``normalized_mse_loss_single`` / ``compute_divergence``: the reference's
  per-graph functions, same signatures and error behaviour;
* ``batch_loss``: the whole per-graph loop of gnn_train.py:168-197 fused into
  two segmented kernels over the batch's ``ptr`` (no Python loop, no dense
  operator), returning (total, nmse, div) with nmse/div already / batch_size.
  All three are differentiable: total = nmse + div, and back-propagating nmse
  and div separately (or their sum) gives the reference's gradients.

All three run through the ``torch.ops.pdivgnn.batch_loss`` custom op (pdg.ops).
"""
from __future__ import annotations

import torch

from pdg import ops  # noqa: F401  (registers torch.ops.pdivgnn.*)
from pdg.plan import GraphPlan, plan_for


def _check_dev(t: torch.Tensor) -> None:
    if t.device.type != "cuda":
        raise RuntimeError("HIP losses need tensors on a HIP device (the CPU restatement is test-only, oracle/)")


def _loss(pred, gt, plan: GraphPlan, types, with_nmse: bool, divergence: bool, penalty: float,
          reduce_abs: bool):
    """(total, nmse / B, penalty * div / B) through the torch.ops.pdivgnn.batch_loss custom op (pdg.ops)."""
    _check_dev(pred)
    if divergence and not plan.has_div:
        raise ValueError("batch has no divergence operator")
    d = plan.has_div and divergence
    total, nmse, div, _den, _divf = torch.ops.pdivgnn.batch_loss(
        pred, gt if with_nmse else None, plan.ptr, types if divergence else None,
        plan.a_rowptr if d else None, plan.a_col if d else None, plan.a_val if d else None,
        plan.at_rowptr if d else None, plan.at_row if d else None, plan.at_comp if d else None,
        plan.at_val if d else None, bool(with_nmse), bool(divergence), float(penalty), bool(reduce_abs))
    return total, nmse, div


def batch_loss(pred: torch.Tensor, batch, gt_std: torch.Tensor, divergence: bool = False,
               divergence_penalty: float = 1.0, reduce_strategy: str = "square"):
    """Fused gnn_train.py:168-197: returns (total, nmse/B, lambda*div/B)."""
    if reduce_strategy not in ("abs", "square"):
        raise AttributeError("reduce_strategy must be 'abs' or 'square'")
    plan = plan_for(batch)
    types = batch.surfaces_nodes_for_div if batch.surfaces_nodes_for_div is not None else batch.nodes_types
    return _loss(pred, gt_std, plan, types, True, bool(divergence), float(divergence_penalty),
                 reduce_strategy == "abs")


def normalized_mse_loss_single(ground_truth_local_stress: torch.Tensor,
                               predicted_local_stress: torch.Tensor) -> torch.Tensor:
    """gnn_train.py:41-57 on one graph."""
    n = predicted_local_stress.shape[0]
    plan = _SinglePlan.get(n, predicted_local_stress.device)
    total, _, _ = _loss(predicted_local_stress, ground_truth_local_stress, plan, None, True, False, 1.0, False)
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
    total, _, _ = _loss(local_stress_field, None, plan, surface_nodes_ids, False, True, 1.0,
                        reduce_strategy == "abs")
    return total
