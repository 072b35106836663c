"""Idle gaps between consecutive kernels in a rocprofv3 kernel_trace.csv (single stream).

    python tools/gaps.py kernel_trace.csv [first_kernel_substring]
Prints total busy time, total gap time and the largest gaps over the traced window
(from the last occurrence of the marker kernel minus one step, if given)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
# keep the last ~third of the trace (steady state)
ks = ks[len(ks) * 2 // 3:]
busy = sum(e - s for s, e, _ in ks)
gaps = [(ks[i + 1][0] - ks[i][1], ks[i][2][:50], ks[i + 1][2][:50]) for i in range(len(ks) - 1)]
tot_gap = sum(g for g, _, _ in gaps if g > 0)
span = ks[-1][1] - ks[0][0]
print(f"kernels {len(ks)}  span {span/1e6:.3f} ms  busy {busy/1e6:.3f} ms  gaps {tot_gap/1e6:.3f} ms "
      f"(mean gap {tot_gap/max(len(gaps),1)/1e3:.2f} us)")
for g, a, b in sorted(gaps, reverse=True)[:8]:
    print(f"  {g/1e3:8.2f} us  {a} -> {b}")
