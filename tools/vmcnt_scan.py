"""List the s_waitcnt vmcnt waits inside loops of every kernel (gfx950 ISA from hipcc -S).

A vmcnt(0) inside a streaming loop usually means the compiler could not count the memory operations in
flight (a conditional load / store on some path into the loop, or a loop-invariant load it sank into the
loop) and waits for every outstanding load AND store there.
    python tools/vmcnt_scan.py [csrc/file.hip ...] [--kernel SUBSTR]"""
import argparse
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "p-div-gnn_amd" / "csrc"


def isa(src: Path) -> str:
    with tempfile.TemporaryDirectory() as d:
        out = Path(d) / (src.stem + ".s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", str(src), "-o", str(out)], check=True, capture_output=True)
        return out.read_text()


def scan(text: str, want: str | None):
    for m in re.finditer(r"^(_Z\w+):\s*(?:;.*)?$", text, re.M):
        name = m.group(1)
        if want and want not in name:
            continue
        body = text[m.end():text.index(".Lfunc_end", m.end())]
        in_loop, waits = False, []
        for line in body.split("\n"):
            t = line.strip()
            if t.startswith(".LBB"):
                in_loop = "in Loop" in t or "Loop Header" in t
            elif t.startswith("s_waitcnt") and "vmcnt" in t and in_loop:
                waits.append(re.search(r"vmcnt\((\d+)\)", t).group(1))
        zeros = waits.count("0")
        print(f"{name[:70]:70s} loop vmcnt waits {len(waits):3d}  vmcnt(0): {zeros}  {' '.join(waits)[:80]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="*")
    ap.add_argument("--kernel")
    a = ap.parse_args()
    files = [Path(f) for f in a.files] or sorted(CSRC.glob("*.hip"))
    for f in files:
        print(f"== {f.name}")
        scan(isa(f), a.kernel)


if __name__ == "__main__":
    sys.exit(main())
