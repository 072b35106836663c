"""Per-kernel SQ counter breakdown from a rocprofv3 --pmc pass (counter_collection.csv).

Prints, per kernel (mean per dispatch, top kernels by SQ_WAVE_CYCLES): the wave-cycle split
WAIT_ANY (parked on s_waitcnt / barrier), WAIT_INST_ANY (issue stalls), ACTIVE_INST_ANY
(issuing), which add up to WAVE_CYCLES (MI355X_MICROARCH.md §rocprofv3 PMC slots), and the
MFMA busy fraction SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES * 4 SIMDs) when both exist.

    python tools/pmc_sq.py counter_collection.csv [top]
"""
import csv
import sys
from collections import defaultdict


def main(argv):
    path = argv[0]
    top = int(argv[1]) if len(argv) > 1 else 12
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        rows.append((m.get("SQ_WAVE_CYCLES", 0.0), k, m))
    rows.sort(reverse=True)
    for wc, k, m in rows[:top]:
        parts = []
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in m and wc > 0:
                parts.append(f"{c[3:]}={m[c] / wc:5.1%}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("SQ_BUSY_CYCLES", 0) > 0:
            parts.append(f"MFMA_busy={m['SQ_VALU_MFMA_BUSY_CYCLES'] / (4 * m['SQ_BUSY_CYCLES']):5.1%}")
        extra = [f"{c}={v:.3g}" for c, v in sorted(m.items()) if c not in (
            "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")]
        print(f"{k[:60]:60s} wave_cyc={wc:.3g} " + " ".join(parts) + " | " + " ".join(extra))


if __name__ == "__main__":
    main(sys.argv[1:])
