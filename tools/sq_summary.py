"""MFMA utilisation and wave-cycle split per kernel from two rocprofv3 SQ counter passes, each run
with --kernel-trace so every dispatch has its duration (tools/sq_pass.sh).

Pass A: SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
Pass B: SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES

Units (MI355X_MICROARCH.md, 's_memtime tick vs SQ PMC units'): SQ_VALU_MFMA_BUSY_CYCLES counts shader
cycles of matrix-pipe occupancy summed over every SIMD (32 per v_mfma_f32_32x32x16_bf16), the
SQ_WAVE/WAIT/ACTIVE counters count quad-cycles.  So, per dispatch,

    mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x clock x duration)

is the fraction of the chip's matrix-pipe cycles the kernel kept busy.  The clock is the one the
kernel ran at, GRBM_GUI_ACTIVE / duration / 8 XCDs (reported; the nominal 2.4 GHz figure is printed
beside it).  MFMA busy is a time fraction, not a FLOP fraction: an fp32 v_mfma_f32_16x16x4_f32
occupies the pipe for 32 cycles for 2,048 FLOP, a bf16 v_mfma_f32_16x16x32_bf16 for 16 cycles for
16,384; bench.py's frac_mfma prices executed FLOPs against the peak of their instruction, which at
full clock is the same quantity.

    python tools/sq_summary.py DIR_A DIR_B [--tree HASH] [--json OUT] [--top N]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 1024
XCDS = 8
NOMINAL_GHZ = 2.4


def _load(d):
    """{dispatch id: (kernel, {counter: value}, duration_ns)} of one pass directory."""
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc:
        raise SystemExit(f"no counter_collection.csv under {d}")
    dur = {}
    for path in kt:
        for r in csv.DictReader(open(path)):
            dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {}
    for path in cc:
        for r in csv.DictReader(open(path)):
            did = r["Dispatch_Id"]
            k, cs, t = out.get(did, (r["Kernel_Name"], {}, None))
            cs[r["Counter_Name"]] = cs.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if t is None:
                if did in dur:
                    t = dur[did]
                elif r.get("End_Timestamp") and r.get("Start_Timestamp"):
                    t = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            out[did] = (k, cs, t)
    return out


def summarise(da, db):
    per = defaultdict(lambda: defaultdict(list))
    for pas in (_load(da), _load(db)):
        for k, cs, t in pas.values():
            for c, v in cs.items():
                per[k][c].append(v)
            if t:
                per[k]["_dur_ns"].append(t)
    rows = []
    for k, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items() if v}
        m["_calls"] = len(cs.get("_dur_ns", [])) / 2 or len(next(iter(cs.values())))
        t = m.get("_dur_ns")
        r = {"kernel": k, "avg_us": t * 1e-3 if t else None}
        if t and m.get("GRBM_GUI_ACTIVE"):
            r["clock_GHz"] = m["GRBM_GUI_ACTIVE"] / XCDS / t
        if t and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            ghz = r.get("clock_GHz") or NOMINAL_GHZ
            r["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * ghz * t)
            r["mfma_busy_at_2.4GHz"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * NOMINAL_GHZ * t)
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    r[c[3:].lower() + "_frac"] = m[c] / wc
        r["counters"] = {c: v for c, v in m.items() if not c.startswith("_")}
        rows.append(r)
    rows.sort(key=lambda r: -(r["avg_us"] or 0) * 1)
    return rows


def main(argv):
    da, db = argv[0], argv[1]
    tree = argv[argv.index("--tree") + 1] if "--tree" in argv else None
    out = argv[argv.index("--json") + 1] if "--json" in argv else None
    top = int(argv[argv.index("--top") + 1]) if "--top" in argv else 24
    rows = summarise(da, db)
    if tree:
        print(f"tree {tree}")
    print("rocprofv3 SQ counters per dispatch (mean), durations from the same passes' kernel traces")
    print(f"{'kernel':58s} {'us':>7s} {'GHz':>5s} {'mfma':>6s} {'@2.4':>6s} {'wait':>6s} {'stall':>6s} {'issue':>6s}")
    for r in rows[:top]:
        def f(key, fmt="{:6.1%}"):
            v = r.get(key)
            return fmt.format(v) if v is not None else "     -"
        print(f"{r['kernel'][:58]:58s} {r['avg_us'] or 0:7.1f} {f('clock_GHz', '{:5.2f}')} {f('mfma_busy')} "
              f"{f('mfma_busy_at_2.4GHz')} {f('wait_any_frac')} {f('wait_inst_any_frac')} {f('active_inst_any_frac')}")
    if out:
        with open(out, "w") as fh:
            json.dump({"_meta": {"tree": tree}, "kernels": rows[:top]}, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
