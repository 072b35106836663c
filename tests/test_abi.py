"""CPU-side checks of the drop-in boundary: the C ABI library loads, exports every
entry point include/pdivgnn.h declares, and the ctypes signatures match the header."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "pdivgnn.h"


def _decls():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    out = {}
    for m in re.finditer(r"\b(?:int|long|const char\*)\s+(pdg_\w+)\s*\(([^)]*)\)\s*;", text, re.S):
        args = [a.strip() for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        out[m.group(1)] = args
    return out


def test_header_declares_entry_points():
    d = _decls()
    assert len(d) >= 30
    for name in ("pdg_edge_fwd", "pdg_edge_bwd", "pdg_segment_sum", "pdg_div_fwd", "pdg_nmse_fwd", "pdg_adam"):
        assert name in d


def test_library_exports_every_declared_symbol():
    from pdg.lib import lib
    dll = lib.load()
    for name in _decls():
        assert hasattr(dll, name), name


def test_library_is_built_from_these_sources():
    """The shipped library embeds build.py's hash of csrc/ + the header; pdg.lib refuses a stale one."""
    from pdg.lib import lib, source_hash
    assert lib.pdg_source_hash().decode() == source_hash()


def test_ctypes_signatures_match_header():
    from pdg.lib import SIGNATURES
    d = _decls()
    assert set(SIGNATURES) == set(d), set(SIGNATURES) ^ set(d)
    for name, args in d.items():
        assert len(SIGNATURES[name]) == len(args), (name, len(SIGNATURES[name]), len(args))


def test_library_reports_errors_without_gpu():
    """Argument validation happens before any HIP call, so it runs on a CPU-only host."""
    from pdg.lib import PdgError, lib
    with pytest.raises(PdgError, match="rows must be > 0"):
        lib.pdg_mlp2_fwd(0, None, None, None, None, None, None, None)
    assert lib.pdg_max_blocks() >= 256
    # mesh-graph scratch sizing is host arithmetic; argument checks precede any HIP call
    assert lib.pdg_mesh_graph_scratch_bytes(100, 150) > 4 * (6 * 150)
    assert lib.pdg_mesh_graph_scratch_bytes(0, 1) < 0
    with pytest.raises(PdgError, match="bad sizes"):
        lib.pdg_mesh_graph(10, None, 4, 0, None, 1, None, None, None, 0, None, None, 0, None)


def test_struct_sizes_match_header():
    import ctypes
    from pdg.lib import LN_BWD_BYTES, LN_STAT_BYTES

    class Stat(ctypes.Structure):
        _fields_ = [("mean", ctypes.c_float), ("den", ctypes.c_float), ("rstd", ctypes.c_float),
                    ("std_", ctypes.c_float), ("mean_d", ctypes.c_double), ("std_d", ctypes.c_double),
                    ("count", ctypes.c_double)]

    class Bwd(ctypes.Structure):
        _fields_ = [("c1", ctypes.c_float), ("c2", ctypes.c_float), ("S1", ctypes.c_double), ("S2", ctypes.c_double)]

    assert ctypes.sizeof(Stat) == LN_STAT_BYTES and ctypes.sizeof(Bwd) == LN_BWD_BYTES


def test_model_refuses_cpu_tensors():
    import torch
    from gnn_local_stress.models import EncodeProcessDecode
    from pdg import graph, meshgen
    m = EncodeProcessDecode(1, 2, latent_size=128, input_nodes_features_size=6, output_nodes_features_size=3)
    b = graph.Batch.from_data_list([graph.sample_to_data(meshgen.hole_plate(5))])
    with pytest.raises(RuntimeError, match="HIP"):
        m(b)
    with pytest.raises(ValueError):
        EncodeProcessDecode(1, 2, latent_size=64, input_nodes_features_size=6, output_nodes_features_size=3)


def test_vector_statistics_are_refused():
    """Per-axis statistics would be truncated to their first element by the scalar input
    formatting; the model refuses them (advisor round 1)."""
    import torch
    from gnn_local_stress.models import EncodeProcessDecode
    m = EncodeProcessDecode(1, 2, latent_size=128, input_nodes_features_size=6, output_nodes_features_size=3,
                            mean_pos=torch.tensor([1.0, 2.0]), std_pos=torch.tensor(3.0))
    with pytest.raises(ValueError, match="mean_pos"):
        m.stats_tensor("cpu")
    m.mean_pos = torch.tensor(1.5)
    assert m.stats_tensor("cpu")[0] == 1.5


def test_stats_tensor_cache_follows_the_statistics():
    """stats_tensor is built once per set of statistics (no per-step host-to-device copies) and
    rebuilt when one is reassigned or modified in place."""
    import torch
    from gnn_local_stress.models import EncodeProcessDecode
    m = EncodeProcessDecode(1, 2, latent_size=128, input_nodes_features_size=6, output_nodes_features_size=3,
                            mean_pos=torch.tensor(1.0), std_pos=2.0)
    t0 = m.stats_tensor("cpu")
    assert m.stats_tensor("cpu") is t0
    m.mean_pos.add_(1.0)                      # in place: version counter moves
    t1 = m.stats_tensor("cpu")
    assert t1 is not t0 and float(t1[0]) == 2.0
    m.std_pos = 4.0                           # reassigned Python scalar
    t2 = m.stats_tensor("cpu")
    assert t2 is not t1 and float(t2[1]) == 4.0 and m.stats_tensor("cpu") is t2
    m.std_pos = torch.tensor(4.0)             # same value, now a tensor: rebuilt, equal contents
    t3 = m.stats_tensor("cpu")
    assert t3 is not t2 and torch.equal(t3, t2)


def test_call_sites_match_signatures():
    """Every direct call of a C-ABI entry point in the host code and the tests passes as many
    arguments as the header declares (calls through lib.pdg_x(...) and engine._t(name, lib.pdg_x, ...)
    without star-arguments), so a signature change cannot leave a stale call behind."""
    import ast
    from pdg.lib import SIGNATURES
    files = list((ROOT / "p-div-gnn_amd").rglob("*.py")) + list((ROOT / "tests").glob("*.py")) + [ROOT / "bench.py"]
    bad = []
    for f in files:
        tree = ast.parse(f.read_text())
        for node in ast.walk(tree):
            if not isinstance(node, ast.Call):
                continue
            fn, args = node.func, node.args
            if isinstance(fn, ast.Attribute) and fn.attr == "_t" and len(args) >= 2:
                fn, args = args[1], args[2:]
            if not (isinstance(fn, ast.Attribute) and fn.attr in SIGNATURES):
                continue
            if any(isinstance(a, ast.Starred) for a in args):
                continue
            if len(args) != len(SIGNATURES[fn.attr]):
                bad.append(f"{f.name}:{node.lineno} {fn.attr} {len(args)} != {len(SIGNATURES[fn.attr])}")
    assert not bad, bad


def test_custom_ops_registered_and_refuse_cpu():
    """torch.library boundary (pdg/ops.py): the four ops exist with their schemas, and a CPU
    tensor is refused before any HIP call (no CPU fallback)."""
    import torch
    from pdg import ops  # noqa: F401
    for name in ("epd_forward", "epd_backward", "batch_loss", "batch_loss_backward"):
        assert hasattr(torch.ops.pdivgnn, name), name
    sch = str(torch.ops.pdivgnn.epd_forward.default._schema)
    assert "Tensor[] params" in sch and "bool need_grad" in sch
    z = torch.zeros(4, 2)
    with pytest.raises(RuntimeError, match="HIP device"):
        torch.ops.pdivgnn.epd_forward([z], torch.zeros(8), z, torch.zeros(4, 3), torch.zeros(4, 1, dtype=torch.long),
                                      torch.zeros(2), torch.zeros(2, 2, dtype=torch.long), 4, 1, True, True, False, 0)
    with pytest.raises(RuntimeError, match="HIP device"):
        torch.ops.pdivgnn.batch_loss(torch.zeros(4, 3), torch.zeros(4, 3), torch.tensor([0, 4]), None, None, None,
                                     None, None, None, None, None, True, False, 1.0, False)


def _params(name):
    """(type, name) of every parameter of `name` in include/pdivgnn.h."""
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    m = re.search(rf"\bint\s+{name}\s*\(([^)]*)\)\s*;", text, re.S)
    out = []
    for a in m.group(1).split(","):
        a = a.strip()
        nm = re.findall(r"\w+", a)[-1]
        out.append(("ptr" if "*" in a else "int", nm))
    return out


INTS = {"n_edges": 1000, "n_nodes": 1000, "nslabs": 256, "nblocks": 256, "npairs_m": 1, "npairs_e": 1,
        "with_edge_update": 1, "slab_init": 0, "accumulate": 0, "e_is_sum": 0}


def _args(name, null):
    """Arguments of `name` with every pointer a distinct 16-byte-aligned fake address (never dereferenced:
    the checks run on the host before any HIP call) except `null`, which is NULL."""
    out = []
    for i, (kind, nm) in enumerate(_params(name)):
        if kind == "ptr":
            out.append(None if nm in (null, "stream") else 0x100000 + 0x1000 * i)
        else:
            out.append(INTS[nm])
    return out


@pytest.mark.parametrize("name,outputs", [
    ("pdg_edge_fwd_coop", ["e_out", "a2m", "part_m", "a2_prev", "src", "P"]),
    ("pdg_edge_fwd_infer", ["e_out", "a2m", "part_m", "a2_prev", "src", "Q"]),
    ("pdg_edge_fwd", ["e_out", "a2m", "part_m", "dst", "Q"]),
    ("pdg_edge_bwd", ["gz2m", "gz1m", "gC", "ge_out", "dst"]),
    ("pdg_edge_bwd_w2", ["gz1m", "gC", "slabs", "gaggr"]),
    ("pdg_edge_gout_wc", ["ge_out", "slabs", "gC", "WcT"]),
    ("pdg_pq_scatter_bwd", ["gP", "gQ", "gz1m", "perm_src"]),
])
def test_edge_entry_points_refuse_null_required_arguments(name, outputs):
    """the edge kernels write through their output pointers (buffer stores drop a NULL
    range silently, flat stores fault), so every required input and output is checked on the host and a
    NULL one refused with PdgError before anything is launched (round 5's fault was an engine branch that
    passed NULL gz2m / gz1e outputs to pdg_edge_bwd)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("host-side argument checks only: never called with fake pointers where a GPU is present")
    from pdg.lib import PdgError, lib
    for nm in outputs:
        with pytest.raises(PdgError, match="null argument|bad slabs|required"):
            getattr(lib, name)(*_args(name, nm))
