"""pdg_edge_fwd_coop against pdg_edge_fwd_p2 alone over a sweep of edge counts E (training variants: with
and without the edge update), median of `reps` launches each (HIP events), and the fit t(E) = fixed + E *
per_row of each: where the pipelined kernel gains (per row) and loses (fixed).  Mesh-like gathers: dst
sorted, src within +-64 nodes of dst.

    python tools/diag/efwd_sweep.py [--reps 20]"""
import ctypes
import struct
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "p-div-gnn_amd")]

import torch  # noqa: E402

from pdg import hiptimer  # noqa: E402
from pdg.lib import lib, stream_handle  # noqa: E402

L = 128
ES = [2520, 11088, 27136, 58808, 151864, 245760, 401408, 614400]


def rnd(*shape):
    return torch.randn(*shape, device="cuda")


def time_launch(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = hiptimer.Event(), hiptimer.Event()
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main(argv):
    reps = int(argv[argv.index("--reps") + 1]) if "--reps" in argv else 20
    torch.manual_seed(0)
    s = stream_handle(torch.device("cuda:0"))
    P = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    res = {}
    for E in ES:
        N = max(E // 6, 64)
        dst = torch.sort(torch.randint(0, N, (E,), device="cuda")).values
        src = (dst + torch.randint(-64, 65, (E,), device="cuda")).clamp(0, N - 1)
        dst, src = dst.int().contiguous(), src.int().contiguous()
        a2p, eres, eout = torch.relu(rnd(E, L)), rnd(E, L), torch.empty(E, L, device="cuda")
        pq = rnd(N, 2 * L)
        W1, b1 = (rnd(L, 3 * L) * 0.05).contiguous(), rnd(L) * 0.1
        W2, b2 = (rnd(L, L) * 0.08).contiguous(), rnd(L) * 0.1
        lg, lb = rnd(L) * 0.3 + 1.0, rnd(L) * 0.1
        mean, sd = float(a2p.double().mean()), float(a2p.double().std(unbiased=False))
        den = float(torch.tensor(sd, dtype=torch.float32) + 1e-5)
        st = torch.frombuffer(bytearray(struct.pack("ffffddd", mean, den, 1.0 / den, sd, mean, sd, a2p.numel())),
                              dtype=torch.uint8).cuda()
        outs = [torch.empty(E, L, device="cuda") for _ in range(4)]
        pm, pe = (torch.zeros(2 * 256, dtype=torch.float64, device="cuda") for _ in range(2))
        qp = pq.data_ptr() + (64 if lib.pdg_pq_layout() else 0)
        for tr in (1, 0):
            for eu in (1, 0):
                for name, fn in (("coop", lib.pdg_edge_fwd_coop), ("p2", lib.pdg_edge_fwd_p2)):
                    call = lambda: fn(E, P(a2p), P(st), P(lg), P(lb), P(eres), P(eout), P(src), P(dst),  # noqa
                                      pq.data_ptr(), qp, P(W1), P(b1), P(W2), P(b2), P(outs[0]) if tr else None,
                                      P(outs[1]), P(outs[2]) if (eu and tr) else None, P(outs[3]) if eu else None,
                                      P(pm), P(pe) if eu else None, eu, 256, s)
                    res.setdefault((name, tr, eu), {})[E] = time_launch(call, reps)
        torch.cuda.synchronize()
        del a2p, eres, eout, pq, outs
        torch.cuda.empty_cache()
    print(f"edge forward alone, median of {reps} launches (us), 256 blocks")
    print(f"{'kernel':16s} " + " ".join(f"{e:>8d}" for e in ES) + f" {'fixed':>7s} {'ns/row':>7s}")
    for (name, tr, eu), r in res.items():
        pts = [(e, r[e]) for e in ES]
        mx, my = sum(e for e, _ in pts) / len(pts), sum(t for _, t in pts) / len(pts)
        sl = sum((e - mx) * (t - my) for e, t in pts) / sum((e - mx) ** 2 for e, _ in pts)
        print(f"{name + (' train' if tr else ' infer') + ' eu' + str(eu):16s} " + " ".join(f"{r[e]:8.1f}" for e in ES) +
              f" {my - sl * mx:7.1f} {sl * 1e3:7.4f}")


if __name__ == "__main__":
    main(sys.argv[1:])
