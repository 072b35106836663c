"""Kernel sum vs wall of the published-workload sweep from a rocprofv3 kernel trace of
`bench.py --sweep-only` (tools/sweep_pass.sh).

Every forward of the engine starts with format_inputs_kernel and ends with decoder_coop_kernel; per mesh
size bench.published_sweep runs 5 set-up forwards (warm-up fwd, warm-up fwd_prepro, the capture's warm
run, the first replay, the launch count run) and then `reps` x (fwd, fwd_prepro, fwd_replay).  For each
forward this prints the kernel sum (format .. decoder, inclusive), the GPU span (first start to last
end) and the dispatch count, per size and series (medians), beside the wall times of the sweep line.

    python tools/sweep_trace.py KERNEL_TRACE.csv SWEEP_LINE.json [--reps 5]"""
import csv
import json
import statistics
import sys

SETUP = 5


def forwards(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    out, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if name.startswith("format_inputs_kernel") or " format_inputs_kernel" in name:
            cur = {"start": s, "end": e, "busy": e - s, "n": 1}
        elif cur is not None:
            cur["end"] = max(cur["end"], e)
            cur["busy"] += e - s
            cur["n"] += 1
            if "decoder_coop_kernel" in name:
                out.append(cur)
                cur = None
    return out


def main(argv):
    reps = int(argv[argv.index("--reps") + 1]) if "--reps" in argv else 5
    fw = forwards(argv[0])
    line = json.load(open(argv[1]))["published_sweep"]["rows"]
    per = SETUP + 3 * reps
    if len(fw) != per * len(line):
        raise SystemExit(f"{len(fw)} forwards in the trace, expected {per} x {len(line)}")
    print(f"{'nodes':>6s} {'series':>10s} {'kernels':>7s} {'ksum_us':>9s} {'span_us':>9s} {'wall_ms(unprof)':>15s}")
    res = []
    for i, row in enumerate(line):
        blk = fw[i * per + SETUP:(i + 1) * per]
        for j, series in enumerate(("fwd", "fwd_prepro", "fwd_replay")):
            f = blk[j::3]
            ks = statistics.median(x["busy"] for x in f) / 1e3
            sp = statistics.median(x["end"] - x["start"] for x in f) / 1e3
            n = f[0]["n"]
            print(f"{row['nodes']:6d} {series:>10s} {n:7d} {ks:9.1f} {sp:9.1f} {row[series]['median_ms']:15.3f}")
            res.append({"nodes": row["nodes"], "series": series, "dispatches": n, "kernel_sum_us": round(ks, 1),
                        "span_us": round(sp, 1), "wall_ms": row[series]["median_ms"]})
    if "--json" in argv:
        json.dump(res, open(argv[argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
