"""Gradients at the reference checkpoint on the batch3_div golden batch (tests/test_gpu_checkpoint.py's
inputs) with the default edge-encoder forward and with the knot-table variant: per-tensor relative difference
and gradient norm, largest differences first."""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, "p-div-gnn_amd")
from gpu_common import golden_batch, rel  # noqa: E402
from test_gpu_checkpoint import _loaded_model  # noqa: E402


def grads(over):
    from gnn_local_stress import losses
    _, batch = golden_batch("batch3_div")
    m, _ = _loaded_model()
    for k, v in over.items():
        setattr(m._engine_for(batch.pos.device), k, v)
    pred = m(batch, scale_output=False).local_stress
    gt = (batch.local_stress - m.mean_local_stress) / m.std_local_stress
    total, _, _ = losses.batch_loss(pred, batch, gt, divergence=True, divergence_penalty=10.0)
    total.backward()
    return {n: p.grad.detach().clone() for n, p in m.named_parameters()}


if __name__ == "__main__":
    a = grads({})
    b = grads({"edge_enc_knots": True})
    rows = sorted(((rel(b[n], a[n]), n, float(a[n].norm())) for n in a), reverse=True)
    for r, n, nrm in rows[:8]:
        print(f"{n:40s} rel diff {r:.3e}   |g| {nrm:.3e}")
