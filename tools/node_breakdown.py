"""Where the node chain's time goes: each node-sized kernel of the training step timed
on its own over a sweep of row counts N, with HIP events around `reps` back-to-back launches (median per
launch), and the time fitted as  t(N) = fixed + N * per_row  over the sizes with at least two tiles per CU.

  fixed     launch + the per-block preamble (weights staged into registers from L2, LayerNorm statistics,
            the first tile's fill) + the drain of the last tile: what a block pays whatever its row count
  per_row   the marginal cost of one more row, beside the bytes that row moves (marginal TB/s)

and the split of the config-2 call (N = 40,328) into the two.  Also timed: the same kernel at N = 16 x grid
(exactly one 16-row tile per block) -- the weight-staging preamble plus one tile.

    python tools/node_breakdown.py [--reps 20] [--json OUT]"""
import ctypes
import json
import struct
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "p-div-gnn_amd")]

import torch  # noqa: E402

from pdg import hiptimer  # noqa: E402
from pdg.lib import lib, stream_handle  # noqa: E402

L = 128
NS = [4096, 8192, 16384, 24576, 32768, 40328, 49152, 65536, 81920]
ROW = 512


def rnd(*shape):
    return torch.randn(*shape, device="cuda")


def stat(a2):
    mean, sd = float(a2.double().mean()), float(a2.double().std(unbiased=False))
    den = float(torch.tensor(sd, dtype=torch.float32) + 1e-5)
    return torch.frombuffer(bytearray(struct.pack("ffffddd", mean, den, 1.0 / den, sd, mean, sd, a2.numel())),
                            dtype=torch.uint8).cuda()


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


def kernels(N, s, cus):
    """name -> (launch closure, bytes per row moved)."""
    W = {k: (rnd(L, L) * 0.08).contiguous() for k in ("W2T", "WaT", "WbT", "Wn2")}
    W1 = (rnd(L, 3 * L) * 0.05).contiguous()
    Wn1 = (rnd(L, 2 * L) * 0.06).contiguous()
    b = rnd(L) * 0.1
    g = rnd(L) * 0.3 + 1.0
    a2, a1, x, gy, aggr = (torch.relu(rnd(N, L)) for _ in range(5))
    st = stat(a2)
    outs = [torch.empty(N, L, device="cuda") for _ in range(4)]
    pq = torch.empty(N, 2 * L, device="cuda")
    part = torch.zeros(lib.pdg_max_blocks() * 2, dtype=torch.float64, device="cuda")
    part[0::2] = float(a2.double().sum()) / cus
    part[1::2] = float((a2.double() ** 2).sum()) / cus
    st_out = torch.zeros(40, dtype=torch.uint8, device="cuda")
    acc = torch.zeros(2 * cus * 256, dtype=torch.float64, device="cuda")
    pairs = torch.tensor([[1.5, -0.5]] * 3, dtype=torch.float64, device="cuda")
    pairs_out = torch.zeros(cus * 2, dtype=torch.float64, device="cuda")
    n = ctypes.c_int(0)
    P = lambda t: t.data_ptr()  # noqa: E731
    return {
        # training node_net: reads aggr, x; writes a1n, a2n
        "node_net_x6": (lambda: lib.pdg_node_net(N, P(aggr), P(x), P(Wn1), P(b), P(W["Wn2"]), P(b), P(outs[0]),
                                                 P(outs[1]), P(part), ctypes.byref(n), s), 4 * ROW),
        # node pre-pass with the previous step's statistics reduced in-kernel: reads a2, x_prev; writes x, P|Q
        "node_pq_x6": (lambda: lib.pdg_node_pq_rw_fin(N, P(a2), P(part), cus, float(N * L), P(st_out), P(g), P(b),
                                                      P(x), P(outs[2]), P(W1), P(pq), pq.data_ptr() + 64, s), 5 * ROW),
        # node_net backward: reads gy, a2n, a1n; writes gz2n, gz1n, gaggr, gx_part
        "node_bwd_coop": (lambda: lib.pdg_node_bwd_coop(N, P(gy), P(a2), P(a1), P(st), None, P(g), P(W["W2T"]),
                                                        P(W["WaT"]), P(W["WbT"]), *[P(o) for o in outs], P(pairs), 3,
                                                        cus, s), 7 * ROW),
        # input gradient of x: reads gP, gQ, gx_part, a2n_prev; writes gx_t (+ LayerNorm column sums)
        "gemm_sum2_coop": (lambda: lib.pdg_gemm_sum2_coop(N, P(gy), P(a1), P(W["WaT"]), P(W["WbT"]), P(x),
                                                          P(outs[3]), P(a2), P(st), P(acc), P(g), P(pairs_out), 1, cus,
                                                          s), 5 * ROW),
    }


def main(argv):
    reps = int(argv[argv.index("--reps") + 1]) if "--reps" in argv else 20
    out = argv[argv.index("--json") + 1] if "--json" in argv else None
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    s = stream_handle(dev)
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    res = {}
    for N in NS + [16 * cus]:
        ks = kernels(N, s, cus)
        for name, (fn, bpr) in ks.items():
            res.setdefault(name, {"bytes_per_row": bpr, "t_us": {}})["t_us"][N] = time_launch(fn, reps)
        del ks
        torch.cuda.empty_cache()
    print(f"node-sized kernels alone, median of {reps} launches (HIP events), {cus} CUs")
    print(f"{'kernel':16s} {'1 tile/CU':>9s} " + " ".join(f"{n:>7d}" for n in NS))
    for name, r in res.items():
        print(f"{name:16s} {r['t_us'][16 * cus]:9.1f} " + " ".join(f"{r['t_us'][n]:7.1f}" for n in NS))
    print()
    print(f"{'kernel':16s} {'fixed_us':>8s} {'ns/row':>7s} {'marg TB/s':>9s} {'t(40328)':>8s} {'fixed %':>7s} "
          f"{'avg TB/s':>8s}")
    for name, r in res.items():
        pts = [(n, r["t_us"][n]) for n in NS if n >= 16384]
        mx = sum(n for n, _ in pts) / len(pts)
        my = sum(t for _, t in pts) / len(pts)
        slope = sum((n - mx) * (t - my) for n, t in pts) / sum((n - mx) ** 2 for n, _ in pts)
        icpt = my - slope * mx
        t2 = r["t_us"][40328]
        r.update(fixed_us=icpt, ns_per_row=slope * 1e3, marginal_tbs=r["bytes_per_row"] / (slope * 1e-6) / 1e12,
                 t_config2_us=t2, fixed_share=icpt / t2, avg_tbs=r["bytes_per_row"] * 40328 / (t2 * 1e-6) / 1e12)
        print(f"{name:16s} {icpt:8.1f} {slope * 1e3:7.3f} {r['marginal_tbs']:9.2f} {t2:8.1f} {100 * icpt / t2:6.1f}% "
              f"{r['avg_tbs']:8.2f}")
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
