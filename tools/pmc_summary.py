"""Per-kernel HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (counter_collection.csv).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide
coalesced read -> bytes_read = 2 * FETCH_SIZE * 1024; WRITE_SIZE (KB) is exact for 16-B stores.
Prints the mean per dispatch for each kernel name; --json FILE also writes
{kernel name: {"read": B, "write": B, "total": B, "dispatches": n}}.

    python tools/pmc_summary.py fetch/counter_collection.csv write/counter_collection.csv [--json out.json]
"""
import csv
import json
import sys
from collections import defaultdict


def load(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main(argv):
    out_json = None
    meta = {}
    if "--tree" in argv:        # tree hash of the measured sources (bench.tree_hash), stored under "_meta"
        i = argv.index("--tree")
        meta["tree"] = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    if "--json" in argv:
        i = argv.index("--json")
        out_json = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    fetch = load(argv[0], "FETCH_SIZE")
    write = load(argv[1], "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, (0.0, 0))[0] * 1024 * 2
        w = write.get(k, (0.0, 0))[0] * 1024
        n = max(fetch.get(k, (0, 0))[1], write.get(k, (0, 0))[1])
        res[k] = {"read": f, "write": w, "total": f + w, "dispatches": n}
        print(f"{k[:70]:70s} read {f/1e6:10.1f} MB  write {w/1e6:10.1f} MB  total {(f+w)/1e6:10.1f} MB")
    if meta:
        print(f"tree {meta['tree']}")
    if out_json:
        json.dump({**({"_meta": meta} if meta else {}), **res}, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
