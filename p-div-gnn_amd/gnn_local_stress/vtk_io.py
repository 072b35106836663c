"""Legacy-VTK mesh I/O without pyvista.

The reference stores every sample mesh with ``pv_mesh.save("….vtk")``
(``scripts/generate_dataset.py:556,584``: a ``PolyData`` surface, legacy VTK,
binary by default) and reads it back with ``pv.get_reader(f).read()``
(``datasets.py:247``) before ``mesh_to_graph`` (``convert_utils.py:47-60``).
pyvista/VTK are not available here, so this module parses the legacy format
directly: ASCII and BINARY (big-endian) files, ``DATASET POLYDATA``
(``POLYGONS``) and ``DATASET UNSTRUCTURED_GRID`` (``CELLS``/``CELL_TYPES``),
both the classic cell layout (``n id id id`` per cell, file versions <= 4.2)
and the VTK-9 layout (``OFFSETS`` + ``CONNECTIVITY`` arrays, version 5.1).
Point/cell data sections are skipped.  ``write_legacy_vtk`` writes the same
formats (used to build test fixtures; no real dataset files ship with the
reference).

Parity: unpinned against VTK itself (no reference .vtk file exists to pin it);
the parser follows the published legacy file-format specification and is
round-trip tested on every layout it accepts.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

_DT = {"float": ">f4", "double": ">f8", "int": ">i4", "unsigned_int": ">u4", "long": ">i8",
       "unsigned_long": ">u8", "vtktypeint64": ">i8", "vtktypeint32": ">i4", "short": ">i2",
       "unsigned_short": ">u2", "char": ">i1", "unsigned_char": ">u1"}


class _Reader:
    def __init__(self, data: bytes, binary: bool) -> None:
        self.d = data
        self.p = 0
        self.binary = binary

    def line(self) -> str:
        while True:
            e = self.d.find(b"\n", self.p)
            if e < 0:
                e = len(self.d)
            s = self.d[self.p:e].decode("latin-1").strip()
            self.p = e + 1
            if s or self.p >= len(self.d):
                return s

    def array(self, n: int, dtype: str) -> np.ndarray:
        if n == 0:
            return np.zeros(0, dtype=_DT[dtype].replace(">", "<"))
        if self.binary:
            dt = np.dtype(_DT[dtype])
            nb = n * dt.itemsize
            a = np.frombuffer(self.d, dtype=dt, count=n, offset=self.p)
            self.p += nb
            # skip the newline that follows a binary block
            if self.p < len(self.d) and self.d[self.p:self.p + 1] == b"\n":
                self.p += 1
            return a.astype(dt.newbyteorder("<"))
        vals: list[str] = []
        while len(vals) < n:
            vals.extend(self.line().split())
        if len(vals) != n:
            raise ValueError("malformed ASCII VTK array")
        return np.array(vals, dtype=_DT[dtype].replace(">", "<"))


def read_legacy_vtk(path: str | Path) -> tuple[np.ndarray, np.ndarray]:
    """Return (points (N, 3) in the stored float dtype, faces (F, k) int64) of a legacy VTK mesh.
    All cells must have the same vertex count k (triangles: 3, quads: 4), as mesh_to_graph
    requires (convert_utils.py:28-34)."""
    data = Path(path).read_bytes()
    r = _Reader(data, False)
    if not r.line().startswith("# vtk DataFile"):
        raise ValueError(f"{path}: not a legacy VTK file")
    r.line()   # title
    fmt = r.line().upper()
    if fmt not in ("ASCII", "BINARY"):
        raise ValueError(f"{path}: unknown format {fmt}")
    r.binary = fmt == "BINARY"
    kind = r.line().split()
    if len(kind) != 2 or kind[0].upper() != "DATASET" or kind[1].upper() not in ("POLYDATA", "UNSTRUCTURED_GRID"):
        raise ValueError(f"{path}: unsupported dataset {' '.join(kind)}")
    points = None
    cells = None
    types = None
    while r.p < len(data):
        ln = r.line()
        if not ln:
            break
        tok = ln.split()
        key = tok[0].upper()
        if key == "POINTS":
            n, dt = int(tok[1]), tok[2].lower()
            points = r.array(3 * n, dt).reshape(n, 3)
        elif key in ("POLYGONS", "CELLS", "TRIANGLE_STRIPS", "LINES", "VERTICES"):
            a, b = int(tok[1]), int(tok[2])
            nxt = r.p
            peek = r.line()
            if peek.upper().startswith("OFFSETS"):           # VTK >= 9 layout: a = ncells + 1, b = nconn
                offsets = r.array(a, peek.split()[1].lower()).astype(np.int64)
                conn_hdr = r.line().split()
                conn = r.array(b, conn_hdr[1].lower()).astype(np.int64)
                sizes = np.diff(offsets)
                flat = conn
            else:                                             # classic layout: a = ncells, b = total ints
                r.p = nxt
                raw = r.array(b, "int").astype(np.int64)
                sizes, flat_parts, i = [], [], 0
                for _ in range(a):
                    k = int(raw[i])
                    sizes.append(k)
                    flat_parts.append(raw[i + 1:i + 1 + k])
                    i += 1 + k
                sizes = np.array(sizes, dtype=np.int64)
                flat = np.concatenate(flat_parts) if flat_parts else np.zeros(0, np.int64)
            if key in ("POLYGONS", "CELLS"):
                if len(sizes) and not np.all(sizes == sizes[0]):
                    raise ValueError(f"{path}: mixed cell sizes are not supported")
                k = int(sizes[0]) if len(sizes) else 3
                cells = flat.reshape(-1, k)
        elif key == "CELL_TYPES":
            types = r.array(int(tok[1]), "int")
        elif key in ("POINT_DATA", "CELL_DATA", "FIELD", "METADATA"):
            break   # attributes are not needed by the graph (datasets.py:247-281)
    if points is None or cells is None:
        raise ValueError(f"{path}: no POINTS or no polygon/cell connectivity")
    if types is not None and len(types) and not np.all(np.isin(types, (5, 9))):
        raise ValueError(f"{path}: only triangle (5) and quad (9) cells are supported")
    return points, cells


def write_legacy_vtk(path: str | Path, points: np.ndarray, faces: np.ndarray, binary: bool = True,
                     layout: str = "5.1", dataset: str = "POLYDATA", point_type: str = "double") -> None:
    """Write points (N, 2|3) and faces (F, k) as legacy VTK (layout "5.1": OFFSETS/CONNECTIVITY,
    "4.2": classic cells); point_type "double" or "float"."""
    pts = np.asarray(points, dtype=np.float64 if point_type == "double" else np.float32)
    if pts.shape[1] == 2:
        pts = np.concatenate([pts, np.zeros((len(pts), 1), pts.dtype)], 1)
    faces = np.asarray(faces, dtype=np.int64)
    F, k = faces.shape
    out = bytearray()
    out += f"# vtk DataFile Version {layout}\nmesh\n{'BINARY' if binary else 'ASCII'}\nDATASET {dataset}\n".encode()

    def arr(a: np.ndarray, dt: str) -> None:
        nonlocal out
        if binary:
            out += np.ascontiguousarray(a, dtype=_DT[dt]).tobytes() + b"\n"
        else:
            out += (" ".join(str(x) for x in a.reshape(-1).tolist()) + "\n").encode()

    out += f"POINTS {len(pts)} {point_type}\n".encode()
    arr(pts.reshape(-1), point_type)
    key = "POLYGONS" if dataset == "POLYDATA" else "CELLS"
    if layout.startswith("5"):
        out += f"{key} {F + 1} {F * k}\nOFFSETS vtktypeint64\n".encode()
        arr(np.arange(F + 1, dtype=np.int64) * k, "vtktypeint64")
        out += b"CONNECTIVITY vtktypeint64\n"
        arr(faces.reshape(-1), "vtktypeint64")
    else:
        out += f"{key} {F} {F * (k + 1)}\n".encode()
        arr(np.concatenate([np.full((F, 1), k, np.int64), faces], 1).reshape(-1), "int")
    if dataset != "POLYDATA":
        out += f"CELL_TYPES {F}\n".encode()
        arr(np.full(F, 5 if k == 3 else 9, np.int64), "int")
    Path(path).write_bytes(bytes(out))
