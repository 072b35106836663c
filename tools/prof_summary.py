"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels, per-step share."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'kernel':60s} {'calls/step':>10s} {'avg_us':>9s} {'ms/step':>8s} {'share':>6s}")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f"{r['Name'][:60]:60s} {int(r['Calls'])/steps:10.1f} {float(r['AverageNs'])/1e3:9.1f} "
          f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} {float(r['Percentage']):5.1f}%")
print(f"total GPU ms/step: {tot/1e6/steps:.3f}")
