"""ctypes binding of libpdivgnn_hip.so (C ABI declared in include/pdivgnn.h).

The library is loaded once, after torch (torch ships the HIP runtime whose
SONAME, libamdhip64.so.7, the library links against, so both share one runtime).
There is no fallback: if the library is missing or fails to load, every
hot-path call raises.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
from ctypes import c_double, c_float, c_int, c_int64, c_void_p
from pathlib import Path

import torch  # noqa: F401  (must be loaded before the HIP library)

SHIPPED = Path(__file__).resolve().parent / "libpdivgnn_hip.so"
LIB_PATH = Path(os.environ.get("PDG_LIB", SHIPPED))
CSRC = Path(__file__).resolve().parents[1] / "csrc"


def source_hash(csrc: Path = CSRC) -> str | None:
    """build.py's hash of the library sources beside this package (None when they are absent)."""
    files = sorted(csrc.glob("*.hip")) + sorted(csrc.glob("*.hpp")) + [csrc.parent.parent / "include" / "pdivgnn.h"]
    if not csrc.is_dir() or not files[-1].exists():
        return None
    h = hashlib.sha256()
    for f in files:
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()[:16]

P = c_void_p
I = c_int

# name -> argtypes (restype is int status unless listed in _RESTYPES)
SIGNATURES: dict[str, list] = {
    "pdg_last_error": [],
    "pdg_version": [],
    "pdg_source_hash": [],
    "pdg_max_blocks": [],
    "pdg_pq_layout": [],
    "pdg_format_inputs": [I, I, P, P, P, P, P, P, I, P, P, P],
    "pdg_encoder_fwd": [I, I, P, P, P, P, P, P, P, P, P, P],
    "pdg_ln_finalize": [P, I, c_double, P, P],
    "pdg_ln_finalize2": [P, P, I, c_double, P, P, P],
    "pdg_node_pq_rw_fin": [I, P, P, I, c_double, P, P, P, P, P, P, P, P, P],
    "pdg_ln_partials_sum": [P, I, P, P],
    "pdg_node_pq": [I, P, P, P, P, P, P, P, P, P, P],
    "pdg_node_pq_rw": [I, P, P, P, P, P, P, P, P, P, P],
    "pdg_edge_fwd": [I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, P, P],
    "pdg_segment_sum": [I, P, P, P, P, P, P, P, P],
    "pdg_segment_sum_fin": [I, P, P, P, P, I, c_double, P, P, P, P, P, P, P],
    "pdg_node_mlp1": [I, P, P, P, P, P, P],
    "pdg_mlp2_fwd": [I, P, P, P, P, P, P, P],
    "pdg_node_net": [I, P, P, P, P, P, P, P, P, P, P, P],
    "pdg_decoder_fwd": [I, P, P, P, P, P, P, P, P, P, P, P, P, I, P, P],
    "pdg_decoder_fwd_fin": [I, P, P, I, c_double, P] + [P] * 10 + [I, P, P],
    "pdg_decoder_fwd_coop": [I, P, P, P, I, c_double, P] + [P] * 10 + [I, P, I, P],
    "pdg_any_nonzero": [P, c_int64, P, P],
    "pdg_zero_unless": [P, P, c_int64, P],
    "pdg_decoder_bwd": [I, P, P, P, P, P, P, P],
    "pdg_ln_colsum": [I, P, P, P, P, P, P, P, P, I, P],
    "pdg_ln_colsum_nodes": [I, P, P, P, P, P, P, P, I, P],
    "pdg_ln_colsum_finalize": [P, I, P, P, P, P, P, P],
    "pdg_ln_param_grads": [I, P, P, P, P, P],
    "pdg_mlp2_bwd": [I, P, P, P, P, P, P, P, P, P, P, P, I, P],
    "pdg_node_bwd": [I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, P],
    "pdg_gemm_dual": [I, P, P, P, P, P, P, P, P],
    "pdg_gemm_sum2": [I, P, P, P, P, P, P, P],
    "pdg_gemm_sum2_rw": [I, P, P, P, P, P, P, P, P, P, P, P, P, I, P],
    "pdg_edge_bwd": [I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, P, I, P],
    "pdg_pq_scatter_bwd": [I, P, P, P, P, P, I, P, P, P],
    "pdg_wgrad_accum": [I, P, P, P, P, P, I, P],
    "pdg_wgrad_reduce": [P, I, P, I, I, P, P],
    "pdg_transpose128_batch": [I, P, P, P, P],
    "pdg_wgrad_reduce_batch": [I, P, P, P, P, P, P, P],
    "pdg_wgrad_segments_batch": [I, P, P, P, P, P, I, P],
    "pdg_edge_fwd_coop": [I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, P],
    "pdg_edge_fwd_infer": [I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, I, P],
    "pdg_edge_enc_fwd": [I, P, P, P, P, P, P, P, I, P],
    "pdg_node_enc_fwd": [I, P, P, P, P, P, P, P, P, I, P],
    "pdg_gemm_sum2_coop": [I, P, P, P, P, P, P, P, P, P, P, P, I, I, P],
    "pdg_node_bwd_coop": [I] + [P] * 14 + [I, I, P],
    "pdg_mlp2_bwd_coop": [I] + [P] * 10 + [I, P, P, I, P],
    "pdg_decoder_bwd_coop": [I] + [P] * 11 + [I, P, I, P],
    "pdg_wgrad_narrow_finalize": [P, I, I, I, P, P, P, P],
    "pdg_bwd_epilogue": [I, P, P, P, P, P, P, I, P, P, P, P, I, P, P, P, P, P, P, P, P, I, P, P, P],
    "pdg_wgrad_slabs_per_cu": [],
    "pdg_wgrad_pairs": [I, P, P, P, P, I, P, P, I, P],
    "pdg_edge_enc_bwd": [I, P, P, P, P, P, P, P, P, I, P, P, P, P, I, I, P],
    "pdg_enc_narrow_reduce": [P, I, P, P, P],
    "pdg_edge_bwd_w2": [I, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, P, I, P, I, P, I, I, P],
    "pdg_edge_gout_wc": [I, P, P, P, P, P, P, I, P, P, P, P, P, I, I, P],
    "pdg_mesh_graph": [I, P, I, I, P, I, P, P, P, ctypes.c_long, P, P, ctypes.c_long, P],
    "pdg_mesh_graph_scratch_bytes": [I, I],
    "pdg_wgrad_segments": [I, P, P, P, P, I, P],
    "pdg_wgrad_narrow": [I, P, P, I, I, P, P, P, P, P],
    "pdg_nmse_fwd": [I, P, P, P, P, P, P],
    "pdg_nmse_bwd": [I, P, I, P, P, P, P, I, P, P],
    "pdg_nmse_fwd_bwd": [I, P, P, P, P, P, P, I, P, P],
    "pdg_div_fwd": [I, P, P, P, P, P, P, I, P, P, P],
    "pdg_div_bwd": [I, P, I, P, P, P, P, P, P, I, I, P, P],
    "pdg_transpose": [I, I, I, P, P, P],
    "pdg_nonfinite2": [P, c_int64, P, P, I, P],
    "pdg_loss_reduce": [I, P, P, c_float, c_float, P, P, P],
    "pdg_collate": [P, I, ctypes.c_long, P],
    "pdg_adam": [c_int64, P, P, P, P, P, I, c_float, c_float, c_float, c_float, P, P, I, P],
}
_RESTYPES = {"pdg_last_error": ctypes.c_char_p, "pdg_source_hash": ctypes.c_char_p, "pdg_mesh_graph_scratch_bytes": ctypes.c_long}

LN_STAT_BYTES = 40   # sizeof(pdg_ln_stat)
# PDG_DEBUG_SYNC=1: synchronise after every library call and name it on stderr (locating a faulting kernel)
_DEBUG_SYNC = os.environ.get("PDG_DEBUG_SYNC") == "1"
LN_BWD_BYTES = 24    # sizeof(pdg_ln_bwd)


class PdgError(RuntimeError):
    pass


class _Lib:
    def __init__(self) -> None:
        self._dll = None
        self.calls = 0   # status-returning entry points called (launch counts: pdg/serve.py, bench.py)
        self.hook = None  # optional callable(name) run after every such call (fault localisation tools)

    def load(self) -> ctypes.CDLL:
        if self._dll is None:
            if not LIB_PATH.exists():
                raise PdgError(f"{LIB_PATH} not built: run `python p-div-gnn_amd/build.py` "
                               "(the HIP path has no CPU fallback)")
            dll = ctypes.CDLL(str(LIB_PATH))
            for name, args in SIGNATURES.items():
                fn = getattr(dll, name)
                fn.argtypes = args
                fn.restype = _RESTYPES.get(name, c_int)
            # the shipped library must be the build of the sources beside it (A/B variants loaded
            # through PDG_LIB may come from other revisions)
            if LIB_PATH.resolve() == SHIPPED:
                want, got = source_hash(), dll.pdg_source_hash().decode()
                if want is not None and got != want:
                    raise PdgError(f"{LIB_PATH} was built from other sources (hash {got}, sources {want}): "
                                   "rebuild it with `python p-div-gnn_amd/build.py`")
            self._dll = dll
        return self._dll

    def __getattr__(self, name: str):
        if not name.startswith("pdg_"):
            raise AttributeError(name)
        fn = getattr(self.load(), name)
        if name in _RESTYPES or name in ("pdg_version", "pdg_max_blocks", "pdg_wgrad_slabs_per_cu", "pdg_pq_layout"):
            return fn

        def call(*args):
            self.calls += 1
            rc = fn(*args)
            if rc != 0:
                msg = self.load().pdg_last_error().decode(errors="replace")
                raise PdgError(f"{name} failed ({rc}): {msg}")
            if self.hook is not None:
                self.hook(name)
            if _DEBUG_SYNC:   # fault localisation: every launch completes before the next (stderr names it)
                import sys
                print(f"[pdg] {name}", file=sys.stderr, flush=True)
                torch.cuda.synchronize()
            return rc

        call.__name__ = name
        return call


lib = _Lib()


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
