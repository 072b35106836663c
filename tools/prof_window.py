"""Per-kernel rocprofv3 averages over the last W training steps of a kernel trace: the dispatches the
bench line's HIP events time (bench.py brackets the launches of the last 3 timed steps), so the two
averages compare the same launches of the same process.  Steps end at each adam_kernel dispatch.
    python tools/prof_window.py KERNEL_TRACE.csv [W] [--json OUT]"""
import csv
import json
import sys
from collections import defaultdict


def main(argv):
    path = argv[0]
    w = int(argv[1]) if len(argv) > 1 and not argv[1].startswith("--") else 3
    out = argv[argv.index("--json") + 1] if "--json" in argv else None
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("adam_kernel")]
    if len(ends) <= w:
        raise SystemExit(f"{len(ends)} steps in the trace, need more than {w}")
    first = ends[-w - 1] + 1
    acc = defaultdict(list)
    for r in rows[first:ends[-1] + 1]:
        acc[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    res = {k: {"calls_per_step": len(v) / w, "avg_us": sum(v) / len(v), "ms_per_step": sum(v) / w * 1e-3}
           for k, v in acc.items()}
    total = sum(r["ms_per_step"] for r in res.values())
    print(f"rocprofv3 kernel trace, the last {w} of {len(ends)} steps (the bench's event window)")
    print(f"{'kernel':60s} {'calls/step':>10s} {'avg_us':>9s} {'ms/step':>8s}")
    for k, r in sorted(res.items(), key=lambda kv: -kv[1]["ms_per_step"])[:30]:
        print(f"{k[:60]:60s} {r['calls_per_step']:10.1f} {r['avg_us']:9.1f} {r['ms_per_step']:8.3f}")
    print(f"total GPU ms/step: {total:.3f}")
    if out:
        json.dump({"window_steps": w, "steps_in_trace": len(ends), "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
