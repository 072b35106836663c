"""How the MFMA accumulation rounds on gfx950 (diagnostic for the bf16x6 / bf16x9 products).
GPU box only:  python tools/mfma_round.py   (builds tools/_mfma_round.so on first use)

For D = A B + C over one 16x16 tile per wave, compares each D element with the fp64 value of
C + sum a b (exact for bf16 products) rounded to fp32 by round-to-nearest-even (RNE) and by
truncation toward zero (RTZ), and reports the mean signed error in fp32 ulps."""
import ctypes
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "_mfma_round.so")


def lib():
    if not os.path.exists(SO):
        subprocess.check_call(["hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC",
                               "-I", os.path.join(HERE, "..", "p-div-gnn_amd", "csrc"),
                               os.path.join(HERE, "mfma_round.hip"), "-o", SO])
    d = ctypes.CDLL(SO)
    for f in (d.mfma_round_bf16, d.mfma_round_f32):
        f.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4
        f.restype = ctypes.c_int
    d.x6_chain.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 3 + [ctypes.c_int]
    d.x6_chain.restype = ctypes.c_int
    return d


def rtz(x64):
    f = x64.float()
    over = f.double().abs() > x64.abs()
    return torch.where(over, torch.nextafter(f, torch.zeros_like(f)), f)


def report(name, D, exact, scale):
    """scale: |C| + sum |a b| per element (the magnitude the accumulation works at)."""
    D = D.double().cpu()
    exact = exact.cpu()
    rne = exact.float().double()
    tz = rtz(exact).double()
    diff = rne != tz
    rel = (D - exact) / scale          # error relative to the accumulation's magnitude
    rel_rne = (rne - exact) / scale
    print(f"{name:36s} ==RNE {float((D == rne).double().mean()):.4f}  where RNE!=RTZ: "
          f"==RNE {float((D[diff] == rne[diff]).double().mean()):.3f} ==RTZ {float((D[diff] == tz[diff]).double().mean()):.3f}"
          f"  err/scale: mean {float(rel.mean()):+.2e} rms {float(rel.pow(2).mean().sqrt()):.2e}"
          f"  (RNE: mean {float(rel_rne.mean()):+.2e} rms {float(rel_rne.pow(2).mean().sqrt()):.2e})")


def main():
    d = lib()
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    T = 4096
    keep = []

    def run_bf16(A, B, C):
        Ag, Bg, Cg = A.to(dev), B.to(dev), C.to(dev)
        keep.extend((Ag, Bg, Cg))
        D = torch.empty_like(Cg)
        assert d.mfma_round_bf16(T, Ag.data_ptr(), Bg.data_ptr(), Cg.data_ptr(), D.data_ptr()) == 0
        exact = C.double() + torch.bmm(A.double(), B.double())
        scale = C.double().abs() + torch.bmm(A.double().abs(), B.double().abs())
        return D, exact, scale

    def run_f32(A, B, C):
        Ag, Bg, Cg = A.to(dev), B.to(dev), C.to(dev)
        keep.extend((Ag, Bg, Cg))
        D = torch.empty_like(Cg)
        assert d.mfma_round_f32(T, Ag.data_ptr(), Bg.data_ptr(), Cg.data_ptr(), D.data_ptr()) == 0
        exact = C.double() + torch.bmm(A.double(), B.double())
        scale = C.double().abs() + torch.bmm(A.double().abs(), B.double().abs())
        return D, exact, scale

    for cscale, label in ((1.0, "C~N(0,1)"), (0.0, "C=0"), (64.0, "C~N(0,64^2)")):
        A = torch.randn(T, 16, 32, generator=g).bfloat16()
        B = torch.randn(T, 32, 16, generator=g).bfloat16()
        C = (torch.randn(T, 16, 16, generator=g) * cscale).float()
        report(f"bf16 16x16x32 {label}", *run_bf16(A, B, C))
        report(f"bf16 16x16x32 positive {label}", *run_bf16(A.abs(), B.abs(), C.abs()))
        report(f"bf16 16x16x32 negative {label}", *run_bf16(-A.abs(), B.abs(), -C.abs()))
        A32 = torch.randn(T, 16, 4, generator=g)
        B32 = torch.randn(T, 4, 16, generator=g)
        report(f"f32 16x16x4 {label}", *run_f32(A32, B32, C))
        report(f"f32 16x16x4 positive {label}", *run_f32(A32.abs(), B32.abs(), C.abs()))
        report(f"f32 16x16x4 negative {label}", *run_f32(-A32.abs(), B32.abs(), -C.abs()))
        keep.clear()
    # fp32-accurate K = 128 products: the accumulation schemes (x6_chain modes)
    names = {0: "bf16x6 one chain", 1: "bf16x6 fresh per chunk + VALU", 2: "bf16x9 one chain", 3: "fp32 MFMA chain"}
    for label, pos in (("signed", False), ("positive", True)):
        A = torch.randn(T, 16, 128, generator=g)
        B = torch.randn(T, 128, 16, generator=g)
        if pos:
            A, B = A.abs(), B.abs()
        exact = torch.bmm(A.double(), B.double())
        scale = torch.bmm(A.double().abs(), B.double().abs())
        Ag, Bg = A.to(dev), B.to(dev)
        for mode in (0, 1, 2, 3):
            D = torch.empty(T, 16, 16, device=dev)
            assert d.x6_chain(T, Ag.data_ptr(), Bg.data_ptr(), D.data_ptr(), mode) == 0
            report(f"K=128 {names[mode]} {label}", D, exact, scale)


if __name__ == "__main__":
    sys.exit(main())
