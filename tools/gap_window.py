"""Inter-kernel gaps of the training step from a rocprofv3 kernel trace of bench.py:
every gap start[i+1] - end[i] between consecutive dispatches of a window of W whole steps (steps end at
each adam_kernel dispatch), summed per boundary type (producer kernel -> consumer kernel), beside the
step's span and kernel sum.  The bench brackets the launches of its LAST 3 timed steps with HIP events
(each event record is a queue packet between two kernels), so the window ends --skip 3 steps before the
trace's end: it measures the uninstrumented steps.

    python tools/gap_window.py KERNEL_TRACE.csv [--steps W] [--skip K] [--top N] [--json OUT]"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"^void ", "", name)
    base = name.split("(")[0]
    return base[:48]


def main(argv):
    path = argv[0]
    opt = lambda k, d: int(argv[argv.index(k) + 1]) if k in argv else d  # noqa: E731
    W, skip, top = opt("--steps", 5), opt("--skip", 3), opt("--top", 25)
    out = argv[argv.index("--json") + 1] if "--json" in argv else None
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("adam_kernel")]
    if len(ends) < W + skip + 1:
        raise SystemExit(f"{len(ends)} steps in the trace, need {W + skip + 1}")
    lo, hi = ends[-(W + skip) - 1] + 1, ends[-skip - 1] if skip else ends[-1]
    win = rows[lo:hi + 1]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in win]
    busy = sum(e - s for s, e, _ in ks)
    span = ks[-1][1] - ks[0][0]
    gaps = defaultdict(lambda: [0, 0])
    neg = 0
    for (s0, e0, a), (s1, e1, b) in zip(ks, ks[1:]):
        g = s1 - e0
        if g < 0:
            neg += -g
            continue
        gaps[(a, b)][0] += g
        gaps[(a, b)][1] += 1
    tot = sum(v[0] for v in gaps.values())
    n = len(ks) - 1
    print(f"window: {W} uninstrumented steps ({skip} event-timed steps excluded), {len(ks)} dispatches "
          f"({len(ks) / W:.1f} per step)")
    print(f"per step: span {span / W / 1e6:.3f} ms, kernel sum {busy / W / 1e6:.3f} ms, gaps {tot / W / 1e6:.3f} ms "
          f"(mean {tot / max(n, 1) / 1e3:.2f} us over {n / W:.0f} boundaries; overlap {neg / W / 1e3:.1f} us)")
    print(f"{'gap us/step':>11s} {'count/step':>10s} {'mean us':>8s}  boundary")
    items = sorted(gaps.items(), key=lambda kv: -kv[1][0])
    for (a, b), (g, c) in items[:top]:
        print(f"{g / W / 1e3:11.2f} {c / W:10.1f} {g / c / 1e3:8.2f}  {a} -> {b}")
    # by consumer kernel
    byc = defaultdict(lambda: [0, 0])
    for (a, b), (g, c) in gaps.items():
        byc[b][0] += g
        byc[b][1] += c
    print("\nby consumer (the gap before each launch of it):")
    for b, (g, c) in sorted(byc.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{g / W / 1e3:11.2f} {c / W:10.1f} {g / c / 1e3:8.2f}  {b}")
    if out:
        json.dump({"steps": W, "skip": skip, "span_ms": span / W / 1e6, "kernel_sum_ms": busy / W / 1e6,
                   "gaps_ms": tot / W / 1e6, "dispatches_per_step": len(ks) / W,
                   "boundaries": [{"from": a, "to": b, "gap_us_per_step": g / W / 1e3, "count_per_step": c / W}
                                  for (a, b), (g, c) in items]}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
