"""Per-stage error table of the HIP path on a golden case: for every
message-passing step, the GPU's forward latents / activations and backward input gradients against
the fp64 restatement, beside two fp32 CPU evaluations of the same math (the reference's op order,
and the GPU's re-associated first layer P[dst] + Q[src] + C), the relu mask bits each one flips
against fp64, and the GPU's gradients against an fp64 evaluation that uses the GPU's own relu
masks (the exact gradient of the piecewise-linear region the GPU's forward landed in).  GPU box only.

    python tools/grad_err_stages.py [case] [--json OUT]

Test infrastructure (it imports oracle/); the restated step follows oracle.epd_oracle.processor_step
(models.py:210-243) op for op, with the intermediates kept.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-div-gnn_amd"), os.path.join(ROOT, "tests")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import epd_oracle as O  # noqa: E402

L = 128


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def _relu(h, key, masks, keep):
    keep[key] = h
    if masks is not None and key in masks:
        return h * masks[key].to(h.dtype)
    return torch.relu(h)


def oracle_run(params, stats, batch, steps, dtype, divergence, penalty, reassoc=False, masks=None):
    """fp32/fp64 forward + backward with every intermediate kept (pre-activations h*, latents x_t / e_t,
    aggr_t with their gradients).  ``reassoc``: the edge MLP's first layer as the GPU forms it,
    (Wa x)[dst] + (Wb x)[src] + (Wc e + b1).  ``masks``: (t, name) -> relu mask replacing relu(h)."""
    P = {k: v.detach().cpu().to(dtype).clone().requires_grad_(True) for k, v in params.items()}
    st = {k: torch.as_tensor(v).cpu().to(dtype) for k, v in stats.items()}
    b = batch
    x, e = O.format_inputs(st, b.pos.cpu().to(dtype), b.mean_stress.cpu().to(dtype), b.nodes_types.cpu(),
                           b.edge_attr.cpu().to(dtype), True)
    x = O._mlp(x, P, "node_encoder")
    e = O._mlp(e, P, "edge_encoder")
    ei = b.edge_index.cpu()
    src, dst = ei[0], ei[1]
    W1, b1 = P["processor.edge_net.0.weight"], P["processor.edge_net.0.bias"]
    W2, b2 = P["processor.edge_net.2.weight"], P["processor.edge_net.2.bias"]
    ge, be = P["processor.edge_net.4.weight"], P["processor.edge_net.4.bias"]
    Wn1, bn1 = P["processor.node_net.0.weight"], P["processor.node_net.0.bias"]
    Wn2, bn2 = P["processor.node_net.2.weight"], P["processor.node_net.2.bias"]
    gn, bnn = P["processor.node_net.4.weight"], P["processor.node_net.4.bias"]
    keep, lat = {}, []

    def edge_mlp(xa, xb, ia, ib, e, t, tag):
        if reassoc:
            Pm, Qm = F.linear(x, W1[:, :L]), F.linear(x, W1[:, L:2 * L])
            C = F.linear(e, W1[:, 2 * L:], b1)
            h1 = (C + Pm.index_select(0, ia)) + Qm.index_select(0, ib)
        else:
            h1 = F.linear(torch.cat([xa, xb, e], dim=-1), W1, b1)
        a1 = _relu(h1, (t, "h1" + tag), masks, keep)
        h2 = F.linear(a1, W2, b2)
        a2 = _relu(h2, (t, "h2" + tag), masks, keep)
        return O.graph_layer_norm(a2, ge, be)

    for t in range(steps):
        x.retain_grad()
        e.retain_grad()
        lat.append((x, e))
        msg = edge_mlp(x.index_select(0, dst), x.index_select(0, src), dst, src, e, t, "m")
        aggr = x.new_zeros(x.shape[0], L)
        aggr.scatter_add_(0, dst.unsqueeze(-1).expand_as(msg), msg)
        aggr.retain_grad()
        keep[(t, "aggr")] = aggr
        h1n = F.linear(torch.cat([aggr, x], dim=-1), Wn1, bn1)
        a1n = _relu(h1n, (t, "h1n"), masks, keep)
        a2n = _relu(F.linear(a1n, Wn2, bn2), (t, "h2n"), masks, keep)
        upd = O.graph_layer_norm(a2n, gn, bnn)
        new_e = edge_mlp(x[src], x[dst], src, dst, e, t, "e")
        x, e = upd + x, new_e + e
    y = O._mlp(x, P, "node_decoder", layer_norm=False)
    gt = (b.local_stress.cpu().to(dtype) - st["mean_local_stress"]) / st["std_local_stress"]
    ops = [d.op_div_matrix.to(dtype) for d in b._data_list]
    total, _, _ = O.batch_loss(y, gt, b.ptr, ops, b.nodes_types.cpu(), divergence, penalty)
    total.backward()
    return dict(P=P, keep=keep, lat=lat, y=y.detach(), grads={k: v.grad for k, v in P.items()})


def gpu_run(g, batch, steps):
    import test_gpu_model as T
    from gnn_local_stress import losses
    model = T._model(steps, g["stats"], g["params"])
    eng = model._engine_for(batch.pos.device)
    cap = {}
    fwd = eng.forward

    def fwd_keep(*a, **k):
        y, ctx = fwd(*a, **k)
        cap["ctx"] = ctx
        return y, ctx
    eng.forward = fwd_keep
    eng.probe = {}
    pred = model(batch, scale_output=False).local_stress
    gt = (batch.local_stress - model.mean_local_stress) / model.std_local_stress
    total, _, _ = losses.batch_loss(pred, batch, gt, divergence=bool(g["divergence"]),
                                    divergence_penalty=float(g["penalty"]))
    model.zero_grad()
    total.backward()
    torch.cuda.synchronize()
    ctx = cap["ctx"]
    out = dict(y=pred.detach().cpu(), perm=ctx.plan.perm.long().cpu(), per_step=[], probe={},
               grads={n: p.grad.detach().cpu() for n, p in model.named_parameters()})
    for d in ctx.per_step:
        out["per_step"].append({k: (v.detach().cpu() if isinstance(v, torch.Tensor) else v) for k, v in d.items()})
    for t, d in eng.probe.items():
        out["probe"][t] = {k: (None if v is None else v.cpu()) for k, v in d.items()}
    eng.probe = None
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    case = args[0] if args else "batch2_div_s10"
    jpath = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
    from gpu_common import golden_batch
    g, batch = golden_batch(case)
    steps = int(g["steps"])
    st = {k: float(v) for k, v in g["stats"].items()}
    div, pen = bool(g["divergence"]), float(g["penalty"])
    G = gpu_run(g, batch, steps)
    perm = G["perm"]
    r64 = oracle_run(g["params"], st, batch, steps, torch.float64, div, pen)
    r32 = oracle_run(g["params"], st, batch, steps, torch.float32, div, pen)
    r32r = oracle_run(g["params"], st, batch, steps, torch.float32, div, pen, reassoc=True)
    # the GPU's relu masks in the oracle's edge order (GPU rows are dst-sorted: row r = edge perm[r])
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel())
    masks = {}
    for t, d in enumerate(G["per_step"]):
        for name, key, edge in (("a1m", "h1m", True), ("a2m", "h2m", True), ("a1e", "h1e", True),
                                ("a2e", "h2e", True), ("a1n", "h1n", False), ("a2n", "h2n", False)):
            v = d.get(name)
            if v is None:
                continue
            m = v > 0
            masks[(t, key)] = m[inv] if edge else m
    r64m = oracle_run(g["params"], st, batch, steps, torch.float64, div, pen, masks=masks)

    def flips(keep, t, key):
        h64 = r64["keep"][(t, key)]
        return int(((keep[(t, key)] > 0) != (h64 > 0)).sum())

    rows = []
    print(f"{case}: {steps} steps, N = {batch.num_nodes}, E = {batch.num_edges}")
    print("forward, relative L2 vs fp64 (GPU | fp32 | fp32 re-associated); relu mask bits flipped vs fp64")
    hdr = f"{'t':>2s} {'x_t':>26s} {'e_t':>26s} {'aggr_t':>26s}   flips GPU / fp32 / fp32r (h1m h2m h1e h2e h1n h2n)"
    print(hdr)
    for t in range(steps):
        d = G["per_step"][t]
        xg, eg = d["x"], d["e"][inv] if d["e"] is not None else None
        x64, e64 = r64["lat"][t]
        x32, e32 = r32["lat"][t]
        x32r, e32r = r32r["lat"][t]
        a64 = r64["keep"][(t, "aggr")]
        row = dict(t=t, x=[rel(xg, x64), rel(x32, x64), rel(x32r, x64)],
                   e=[rel(eg, e64), rel(e32, e64), rel(e32r, e64)],
                   aggr=[rel(d["aggr"], a64), rel(r32["keep"][(t, "aggr")], a64), rel(r32r["keep"][(t, "aggr")], a64)])
        fl = {}
        for key in ("h1m", "h2m", "h1e", "h2e", "h1n", "h2n"):
            if (t, key) not in masks:
                continue
            h64 = r64["keep"][(t, key)]
            fl[key] = [int((masks[(t, key)] != (h64 > 0)).sum()), flips(r32["keep"], t, key), flips(r32r["keep"], t, key)]
        row["flips"] = fl
        pr = G["probe"][t]
        gx64, ge64 = x64.grad, e64.grad
        row["gx"] = [rel(pr["gx"], gx64), rel(x32.grad, gx64), rel(x32r.grad, gx64), rel(pr["gx"], r64m["lat"][t][0].grad)]
        row["ge"] = ([rel(pr["ge"][inv], ge64), rel(e32.grad, ge64), rel(e32r.grad, ge64),
                      rel(pr["ge"][inv], r64m["lat"][t][1].grad)] if pr["ge"] is not None else None)
        row["gaggr"] = [rel(pr["gaggr"], a64.grad), rel(r32["keep"][(t, "aggr")].grad, a64.grad),
                        rel(r32r["keep"][(t, "aggr")].grad, a64.grad), rel(pr["gaggr"], r64m["keep"][(t, "aggr")].grad)]
        rows.append(row)
        f3 = lambda v: " ".join(f"{u:8.1e}" for u in v)  # noqa: E731
        print(f"{t:2d} {f3(row['x'])} {f3(row['e'])} {f3(row['aggr'])}   "
              + " ".join(f"{k}:{'/'.join(map(str, v))}" for k, v in fl.items()))
    print("\nbackward input gradients, relative L2 vs fp64 (GPU | fp32 | fp32r | GPU vs fp64 with the GPU's masks)")
    print(f"{'t':>2s} {'d/dx_t':>36s} {'d/de_t':>36s} {'d/daggr_t':>36s}")
    for row in rows:
        f4 = lambda v: " ".join(f"{u:8.1e}" for u in v) if v else " " * 35  # noqa: E731
        print(f"{row['t']:2d} {f4(row['gx'])} {f4(row['ge'])} {f4(row['gaggr'])}")
    print("\nparameter gradients, relative L2 vs fp64")
    print(f"{'tensor':30s} {'GPU':>9s} {'golden32':>9s} {'fp32':>9s} {'fp32r':>9s} {'GPU|mask':>9s} {'fp32|msk':>9s}")
    g64 = r64["grads"]
    # the fp32 oracle again with the GPU's masks: the fp32 noise floor inside the GPU's relu region
    r32m = oracle_run(g["params"], st, batch, steps, torch.float32, div, pen, masks=masks)
    prow = {}
    for n in g64:
        v = [rel(G["grads"][n], g64[n]), rel(g["grads"][n], g64[n]), rel(r32["grads"][n], g64[n]),
             rel(r32r["grads"][n], g64[n]), rel(G["grads"][n], r64m["grads"][n]), rel(r32m["grads"][n], r64m["grads"][n])]
        prow[n] = v
        print(f"{n:30s} " + " ".join(f"{u:9.2e}" for u in v))
    print(f"\noutput: GPU {rel(G['y'], r64['y']):.2e}  fp32 {rel(r32['y'], r64['y']):.2e}  "
          f"fp32r {rel(r32r['y'], r64['y']):.2e}")
    if jpath:
        with open(jpath, "w") as f:
            json.dump(dict(case=case, steps=rows, params=prow, lib=os.environ.get("PDG_LIB", "shipped")), f)


if __name__ == "__main__":
    main()
