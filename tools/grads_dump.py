"""Dump one training step's loss, output and every parameter gradient (library chosen by PDG_LIB)
to a .pt file, for bitwise A/B of two library builds.  GPU box only.
    python tools/grads_dump.py OUT.pt [nmesh ngraph steps div]
    python tools/grads_dump.py --compare A.pt B.pt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-div-gnn_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402


def dump(out, nmesh=41, ngraph=3, steps=4, div=1):
    import test_gpu_model as T
    from gpu_common import dataset_stats, make_batch
    from gnn_local_stress import losses
    from pdg import meshgen
    samples = meshgen.make_dataset(ngraph, n=nmesh, hole_radius=(0.15, 0.3), seed=5)
    batch = make_batch(samples)
    stats = {k: float(v) for k, v in dataset_stats(batch).items()}
    model = T._model(steps, stats)
    pred = model(batch, scale_output=False).local_stress
    gt = (batch.local_stress - model.mean_local_stress) / model.std_local_stress
    total, _, _ = losses.batch_loss(pred, batch, gt, divergence=bool(div), divergence_penalty=10.0)
    model.zero_grad()
    total.backward()
    res = {"loss": total.detach().cpu(), "out": pred.detach().cpu()}
    res.update({n: p.grad.detach().cpu() for n, p in model.named_parameters()})
    torch.save(res, out)


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = [k for k in A if not torch.equal(A[k], B[k])]
    for k in bad:
        d = (A[k].double() - B[k].double()).norm() / B[k].double().norm().clamp_min(1e-30)
        print(f"DIFF {k}: rel {float(d):.3e}")
    print(f"{len(A) - len(bad)}/{len(A)} tensors bitwise equal")
    return not bad


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    dump(sys.argv[1], *(int(a) for a in sys.argv[2:6]))
