"""Bitwise A/B of pdg_edge_bwd_w2 between two library builds on identical random inputs, in one
process (both .so files loaded side by side).  GPU box only.
    python tools/ebw_bitwise.py LIB_A LIB_B [E]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "p-div-gnn_amd")]

import torch  # noqa: E402

from pdg.lib import LN_BWD_BYTES, LN_STAT_BYTES, SIGNATURES, stream_handle  # noqa: E402


def load(path):
    dll = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    f = dll.pdg_edge_bwd_w2
    f.argtypes = SIGNATURES["pdg_edge_bwd_w2"]
    f.restype = ctypes.c_int
    return dll


def main(a, b, E=60001, N=10007):
    torch.manual_seed(1)
    dev = torch.device("cuda:0")
    L = 128
    f = dict(dtype=torch.float32, device=dev)
    dst = torch.sort(torch.randint(0, N, (E,), device=dev))[0].int()
    gaggr, ge = torch.randn(N, L, **f), torch.randn(E, L, **f)
    a2m, a1m, a2e, a1e = (torch.randn(E, L, **f).relu() for _ in range(4))
    st = torch.zeros(2, LN_STAT_BYTES, dtype=torch.uint8, device=dev)
    sv = torch.tensor([0.3, 1.2, 1 / 1.2, 1.19999], dtype=torch.float32)
    dv = torch.tensor([0.3, 1.19999, float(E * L)], dtype=torch.float64)
    for i in range(2):
        st[i, :16] = sv.view(torch.uint8).to(dev)
        st[i, 16:40] = dv.view(torch.uint8).to(dev)
    lb = torch.zeros(2, LN_BWD_BYTES, dtype=torch.uint8, device=dev)
    for i in range(2):
        lb[i, :8] = torch.tensor([0.01, -0.02], dtype=torch.float32).view(torch.uint8).to(dev)
    g = torch.rand(L, **f) + 0.5
    W2T = torch.randn(L, L, **f) * 0.1
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    out = {}
    for name, path in (("a", a), ("b", b)):
        dll = load(path)
        res = {k: torch.full((E, L), 7.0, **f) for k in ("gz1m", "gz1e", "gC")}
        slabs = torch.zeros(cus, L * L + L, **f)
        for eu in (True, False):
            P = lambda t: t.data_ptr()
            rc = dll.pdg_edge_bwd_w2(E, P(dst), P(gaggr), P(ge) if eu else None, P(a2m), P(a1m), P(a2e), P(a1e),
                                     P(st), P(st) + LN_STAT_BYTES, P(lb), P(lb) + LN_BWD_BYTES, P(g), P(W2T),
                                     P(res["gz1m"]), P(res["gz1e"]), P(res["gC"]), P(slabs), cus, None, 0, None, 0,
                                     0, stream_handle(dev))
            assert rc == 0, rc
            torch.cuda.synchronize()
            out[(name, eu)] = {k: v.clone() for k, v in res.items()} | {"slabs": slabs.clone()}
    for eu in (True, False):
        for k in out[("a", eu)]:
            x, y = out[("a", eu)][k], out[("b", eu)][k]
            nd = int((x != y).sum())
            print(f"EU={eu} {k:6s} {'EQUAL' if nd == 0 else 'DIFF'} n={nd} rel={float((x - y).norm() / y.norm()):.2e}")


if __name__ == "__main__":
    main(*sys.argv[1:3], *(int(x) for x in sys.argv[3:]))
