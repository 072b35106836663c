"""Per-parameter gradient error of the HIP path against the fp64 oracle, next to the fp32
oracle's own error (the parity test's criterion, tests/test_gpu_model.py), for the library
selected by PDG_LIB.  GPU box only.   python tools/grad_err.py [nmesh ngraph steps div]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-div-gnn_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402

import test_gpu_model as T  # noqa: E402
from gpu_common import dataset_stats, make_batch, rel  # noqa: E402


def main():
    nmesh, ngraph, steps, div = (int(a) for a in (sys.argv[1:5] if len(sys.argv) > 4 else (21, 2, 10, 1)))
    from gnn_local_stress import losses
    from pdg import meshgen
    samples = meshgen.make_dataset(ngraph, n=nmesh, hole_radius=(0.15, 0.3), seed=5)
    batch = make_batch(samples)
    stats = {k: float(v) for k, v in dataset_stats(batch).items()}
    model = T._model(steps, stats)
    params = {k: v.detach().clone() for k, v in model.state_dict().items()}
    pred = model(batch, scale_output=False).local_stress
    gt = (batch.local_stress - model.mean_local_stress) / model.std_local_stress
    total, _, _ = losses.batch_loss(pred, batch, gt, divergence=bool(div), divergence_penalty=10.0)
    model.zero_grad()
    total.backward()
    p32, t32, g32 = T._oracle_grads(params, stats, batch, steps, torch.float32, bool(div), 10.0)
    p64, t64, g64 = T._oracle_grads(params, stats, batch, steps, torch.float64, bool(div), 10.0)
    print(f"out: hip {rel(pred.detach(), p64):.2e}  fp32 {rel(p32, p64):.2e}")
    for name, p in model.named_parameters():
        print(f"{name:34s} hip {rel(p.grad, g64[name]):.2e}  fp32 {rel(g32[name], g64[name]):.2e}")


if __name__ == "__main__":
    main()
