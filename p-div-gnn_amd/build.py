"""Build libpdivgnn_hip.so (all HIP kernels + the C ABI of include/pdivgnn.h) for gfx950.

    python p-div-gnn_amd/build.py [--force] [--report]

Compiles each csrc/*.hip with hipcc in parallel and links one shared library into
pdg/ (in-tree, so it travels to the GPU box with the repo snapshot)."""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = Path(os.environ.get("PDG_CSRC", HERE / "csrc"))
# PDG_OUT / PDG_BUILD_DIR / PDG_EXTRA_FLAGS build side-by-side variants for A/B timing
# (loaded with PDG_LIB=...); the default build is the shipped library, and it is always built
# from csrc/ with the default flags (extra flags are refused for it).
SHIPPED = HERE / "pdg" / "libpdivgnn_hip.so"
OUT = Path(os.environ.get("PDG_OUT", SHIPPED))
BUILD = Path(os.environ.get("PDG_BUILD_DIR", HERE / "build"))
ARCH = os.environ.get("PDG_OFFLOAD_ARCH", "gfx950")
EXTRA = os.environ.get("PDG_EXTRA_FLAGS", "").split()
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function", *EXTRA]


def source_hash(csrc: Path = CSRC) -> str:
    """sha256 (16 hex) of the library's sources; embedded as pdg_source_hash() and checked by pdg.lib
    (same function there)."""
    h = hashlib.sha256()
    for f in sorted(csrc.glob("*.hip")) + sorted(csrc.glob("*.hpp")) + [csrc.parent.parent / "include" / "pdivgnn.h"]:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()[:16]


INFO = "pdg_build_info"   # compiled on every build, with the source hash


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and Path(c).exists():
            return c
    raise RuntimeError("hipcc not found")


def _compile(src: Path, report: bool) -> Path:
    obj = BUILD / (src.stem + ".o")
    deps = [src] + sorted(CSRC.glob("*.hpp")) + [CSRC.parent.parent / "include" / "pdivgnn.h"]
    info = src.stem == INFO
    # an object is reused only when the CONTENT of its sources and the flags match the stamp written
    # beside it (modification times let a source restored with an older mtime link a stale object)
    # (a --report compile embeds its extra flag in the object: its objects are never reused by a normal build)
    h = hashlib.sha256(" ".join(FLAGS + (["--report"] if report else [])).encode())
    for d in deps:
        h.update(d.name.encode())
        h.update(d.read_bytes())
    stamp = obj.with_suffix(".stamp")
    if obj.exists() and stamp.exists() and stamp.read_text() == h.hexdigest() and not info:
        return obj
    stamp.unlink(missing_ok=True)
    cmd = [hipcc(), *FLAGS, "-c", str(src), "-o", str(obj)]
    if info:
        cmd.append(f'-DPDG_SRC_HASH="{source_hash()}"')
    if report:
        cmd.append("-Rpass-analysis=kernel-resource-usage")
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed on {src.name}:\n{r.stderr}")
    if report:
        (BUILD / (src.stem + ".res")).write_text(r.stderr)
    stamp.write_text(h.hexdigest())
    return obj


def build(force: bool = False, report: bool = False) -> Path:
    if OUT.resolve() == SHIPPED.resolve() and (EXTRA or CSRC.resolve() != (HERE / "csrc").resolve()
                                               or ARCH != "gfx950"):
        raise RuntimeError("the shipped library is built from csrc/ for gfx950 with the default flags only; "
                           "set PDG_OUT (and PDG_BUILD_DIR) to build an A/B variant")
    BUILD.mkdir(parents=True, exist_ok=True)
    OUT.parent.mkdir(parents=True, exist_ok=True)
    srcs = sorted(CSRC.glob("*.hip"))
    if force:
        for o in BUILD.glob("*.o"):
            o.unlink()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, report), srcs))
    # always linked: the build-info object is compiled on every build
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(OUT), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--report", action="store_true", help="write per-kernel register/spill report")
    a = ap.parse_args()
    out = build(force=a.force, report=a.report)
    print(out)
    if a.report:
        subprocess.run([sys.executable, str(HERE / "tools" / "regs.py"), *map(str, sorted(BUILD.glob("*.res")))])
