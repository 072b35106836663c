"""Per-parameter gradient error vs the fp64 oracle on a golden case, for several engine variants side by
side (which kernels' arithmetic the error comes from), next to the fp32 oracle's and the golden fp32
reference's own errors.  GPU box only.   python tools/grad_err_golden.py [case]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-div-gnn_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import test_gpu_model as T  # noqa: E402
from gpu_common import golden_batch, rel  # noqa: E402

VARIANTS = {"default": {}, "node_bwd_fp32": {"nbwd_coop": False}, "gsum2_fp32": {"gsum2_coop": False},
            "both_fp32": {"nbwd_coop": False, "gsum2_coop": False}}


def grads(g, batch, steps, var):
    from gnn_local_stress import losses
    model = T._model(steps, g["stats"], g["params"])
    eng = model._engine_for(batch.pos.device)
    for k, v in var.items():
        setattr(eng, k, v)
    pred = model(batch, scale_output=False).local_stress
    gt = (batch.local_stress - model.mean_local_stress) / model.std_local_stress
    total, _, _ = losses.batch_loss(pred, batch, gt, divergence=bool(g["divergence"]),
                                    divergence_penalty=float(g["penalty"]))
    model.zero_grad()
    total.backward()
    return {n: p.grad.detach().clone() for n, p in model.named_parameters()}


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "batch2_div_s10"
    g, batch = golden_batch(case)
    steps = int(g["steps"])
    st = {k: float(v) for k, v in g["stats"].items()}
    _, _, g64 = T._oracle_grads(g["params"], st, batch, steps, torch.float64, bool(g["divergence"]), float(g["penalty"]))
    _, _, g32 = T._oracle_grads(g["params"], st, batch, steps, torch.float32, bool(g["divergence"]), float(g["penalty"]))
    res = {k: grads(g, batch, steps, v) for k, v in VARIANTS.items()}
    print(f"{case}: relative L2 error vs fp64")
    print(f"{'tensor':32s} {'golden32':>9s} {'oracle32':>9s} " + " ".join(f"{k:>13s}" for k in VARIANTS))
    for n in g64:
        print(f"{n:32s} {rel(g['grads'][n], g64[n]):9.2e} {rel(g32[n], g64[n]):9.2e} "
              + " ".join(f"{rel(res[k][n], g64[n]):13.2e}" for k in VARIANTS))


if __name__ == "__main__":
    main()
