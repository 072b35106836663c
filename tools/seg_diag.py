"""Diagnostic (GPU box): gradients of the golden case with the fused message sums, bisected by
swapping the backward's per-step inputs for the unfused path's."""
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-div-gnn_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402


def run(g, batch, seg, patch=None):
    import test_gpu_model as T
    from gnn_local_stress import losses
    steps = int(g["steps"])
    model = T._model(steps, g["stats"], g["params"])
    eng = model._engine_for(batch.pos.device)
    eng.seg_sums = seg
    keep = {}
    orig = eng.forward

    def fwd(*a, **k):
        y, ctx = orig(*a, **k)
        keep["ctx"] = ctx
        return y, ctx
    eng.forward = fwd
    pred = model(batch, scale_output=False).local_stress
    gt = (batch.local_stress - model.mean_local_stress) / model.std_local_stress
    total, _, _ = losses.batch_loss(pred, batch, gt, divergence=bool(g["divergence"]),
                                    divergence_penalty=float(g["penalty"]))
    ctx = keep["ctx"]
    if patch:
        patch(ctx)
    per = [dict(d) for d in ctx.per_step]
    ctx._keep = per
    model.zero_grad()
    total.backward()
    torch.cuda.synchronize()
    return per, {n: p.grad.clone() for n, p in model.named_parameters()}, ctx


def main(case="tiny_periodic"):
    from gpu_common import golden_batch, rel
    g, batch = golden_batch(case)
    per0, g0, _ = run(g, batch, False)

    def xs_from_sums(ctx):
        deg = (ctx.plan.rowptr_dst[1:] - ctx.plan.rowptr_dst[:-1]).double()[:, None]
        for d in ctx.per_step:
            i = d["i_m"] * ctx.stats.nbytes
            mean, den = struct.unpack("ff", bytes(ctx.stats.buf[i:i + 8].cpu().numpy().tobytes()))
            d["xs"] = torch.where(deg > 0, (d["sums"].double() - deg * mean) / den, torch.zeros_like(deg)).float()
            d["sums"] = None

    def plus_aggr(ctx):
        xs_from_sums(ctx)
        for d, d0 in zip(ctx.per_step, per0):
            d["aggr"] = d0["aggr"]

    def plus_all(ctx):
        for d, d0 in zip(ctx.per_step, per0):
            for k in d:
                if k not in ("sums",):
                    d[k] = d0[k]
            d["sums"] = None
    per1, _, _ = run(g, batch, True)
    for t, (d0, d1) in enumerate(zip(per0, per1)):
        print(t, " ".join(f"{k}={rel(d1[k], d0[k]):.2e}" for k in d0
                          if torch.is_tensor(d0[k]) and torch.is_tensor(d1.get(k))))
    for t, (d0, d1) in enumerate(zip(per0, per1)):
        for k in ("a1n", "a2n", "a1m", "a2m"):
            f = ((d0[k] > 0) != (d1[k] > 0))
            if int(f.sum()):
                idx = f.nonzero()[:4].tolist()
                print(f"step {t} {k}: {int(f.sum())} relu flips, e.g.", [(i, float(d0[k][i[0], i[1]]), float(d1[k][i[0], i[1]])) for i in idx])
    def self_clone(ctx):
        for d in ctx.per_step:
            d["a2n"] = d["a2n"].clone()
    def snap(ctx):
        ctx._snap = [d["a2n"].clone() for d in ctx.per_step]
    _, g1, c1 = run(g, batch, True, snap)
    print("a2n changed during backward:", [float((d["a2n"] - s0).abs().max()) for d, s0 in zip(c1._keep, c1._snap)])
    _, g1, _ = run(g, batch, True, self_clone)
    worst = max(g0, key=lambda n: rel(g1[n], g0[n]))
    print(f"a2n self-clone worst {worst} {rel(g1[worst], g0[worst]):.3e}")
    for key in ("a2n",):
        def only(ctx, key=key):
            plus_aggr(ctx)
            for d, d0 in zip(ctx.per_step, per0):
                if torch.is_tensor(d0.get(key)):
                    d[key] = d0[key]
        _, g1, _ = run(g, batch, True, only)
        worst = max(g0, key=lambda n: rel(g1[n], g0[n]))
        print(f"+{key:6s} worst {worst} {rel(g1[worst], g0[worst]):.3e}")
    for name, patch in (("seg", None), ("seg+xs(torch)", xs_from_sums), ("seg+xs+aggr", plus_aggr),
                        ("seg+all", plus_all)):
        _, g1, _ = run(g, batch, True, patch)
        worst = max(g0, key=lambda n: rel(g1[n], g0[n]))
        print(f"{name:16s} worst {worst} {rel(g1[worst], g0[worst]):.3e}  "
              f"node_net.2.weight {rel(g1['processor.node_net.2.weight'], g0['processor.node_net.2.weight']):.3e}")


if __name__ == "__main__":
    main(*sys.argv[1:])
