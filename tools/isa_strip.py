"""One character per instruction of a kernel's main loop (gfx950 ISA from hipcc -S), to see how the
compiler interleaved matrix, vector, LDS and memory work:  M mfma  V valu  R ds_read  W ds_write
G global/buffer load  S global/buffer store  B s_barrier  w s_waitcnt  . other scalar.
    python tools/isa_strip.py FILE.hip KERNEL_SUBSTRING [loop-index]"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path


def classify(op: str) -> str:
    if op.startswith("v_mfma"):
        return "M"
    if op.startswith("ds_read") or op.startswith("ds_bpermute"):
        return "R"
    if op.startswith("ds_write"):
        return "W"
    if op.startswith(("global_load", "buffer_load")):
        return "G"
    if op.startswith(("global_store", "buffer_store")):
        return "S"
    if op == "s_barrier":
        return "B"
    if op == "s_waitcnt":
        return "w"
    if op.startswith("v_"):
        return "V"
    return "."


def main():
    src, kname = sys.argv[1], sys.argv[2]
    which = int(sys.argv[3]) if len(sys.argv) > 3 else -1
    with tempfile.TemporaryDirectory() as d:
        out = Path(d) / "k.s"
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", *sys.argv[4:],
                        src, "-o", str(out)], check=True, capture_output=True)
        text = out.read_text()
    m = re.search(r"^(_Z\w*" + re.escape(kname) + r"\w*):", text, re.M)
    body = text[m.end():text.index(".Lfunc_end", m.end())]
    loops, cur = [], None
    for line in body.split("\n"):
        t = line.strip()
        if t.startswith(".LBB"):
            if "Loop Header" in t:
                cur = []
                loops.append(cur)
            elif "in Loop" not in t:
                cur = None
            continue
        if cur is None or not t or t.startswith((";", ".")):
            continue
        cur.append(classify(t.split()[0]))
    for i, lp in enumerate(loops):
        if which >= 0 and i != which:
            continue
        s = "".join(lp)
        print(f"loop {i}: {len(s)} instructions, {s.count('M')} M, {s.count('V')} V, {s.count('R')} R, {s.count('W')} W")
        for k in range(0, len(s), 120):
            print("  " + s[k:k + 120])


if __name__ == "__main__":
    main()
