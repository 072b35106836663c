"""Diagnose eager vs graph-replay differences: per step, which gradient blocks differ."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "p-div-gnn_amd"), str(ROOT / "tests")]

import torch  # noqa: E402

import test_gpu_trainer_graph as t  # noqa: E402
from pdg.engine import PARAM_SHAPES  # noqa: E402


def run(capture, div, seq):
    tr = t._trainer(seq[0], div, capture)
    gs, ls = [], []
    for b in seq:
        out = tr.step(b)
        ls.append(float(out["total"]))
        gs.append(tr.flat_g.clone())
    return ls, gs


def main():
    div = len(sys.argv) > 1 and sys.argv[1] == "div"
    b1, b2 = t._batch(11), t._batch(12)
    seq = (b1, b1, b1, b2, b2, b1)
    runs = {"eagerA": run(False, div, seq), "eagerB": run(False, div, seq), "graph": run(True, div, seq)}
    names = [n for n, _ in PARAM_SHAPES]
    sizes = [int(torch.Size(s).numel()) for _, s in PARAM_SHAPES]
    for other in ("eagerB", "graph"):
        la, ga = runs["eagerA"]
        lb, gb = runs[other]
        print(other, "losses", ["%.6f/%.6f" % (x, y) for x, y in zip(la, lb)])
        for i, (x, y) in enumerate(zip(ga, gb)):
            if torch.equal(x, y):
                continue
            off, bad = 0, []
            for n, k in zip(names, sizes):
                d = (x[off:off + k] - y[off:off + k]).abs().max().item()
                if d > 0:
                    bad.append(f"{n}:{d:.2e}")
                off += k
            print(f"  step {i}: {len(bad)} blocks differ: {' '.join(bad[:12])}")
            break


if __name__ == "__main__":
    main()
