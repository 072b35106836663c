"""Forward/backward orchestration of EncodeProcessDecode on the HIP kernels.

One call of :meth:`EPDEngine.forward` runs the whole encode-process-decode
stack of ``gnn_local_stress/models.py:288-326`` as a fixed sequence of HIP
launches on the current stream (no host sync, no torch compute ops); with
``need_grad`` it keeps the activations the backward needs.
:meth:`EPDEngine.backward` runs the reverse sequence and accumulates every
parameter gradient into caller-provided fp32 buffers.

Per message-passing step t (weights shared across steps, models.py:313-314):

  forward                                   kernels
  x_t = LN_n(a2n_{t-1}) + x_{t-1}           pdg_node_pq      (also P = Wa x_t, Q = Wb x_t)
  e_t = LN_e(a2e_{t-1}) + e_{t-1}           pdg_edge_fwd     (C = Wc e_t + b1, both edge_net
  a1m,a2m (message), a1e,a2e (edge upd.)                      evaluations, LN partials)
  aggr = sum_dst LN_m(a2m)                  pdg_segment_sum
  a1n = relu(Wn1 [aggr, x_t] + bn1)         pdg_node_mlp1
  a2n = relu(Wn2 a1n + bn2)                 pdg_mlp2_fwd

Graph-global LayerNorm statistics are reduced by pdg_ln_finalize between the
producer and the consumer of each normalised tensor.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import torch

from . import hiptimer
from .lib import LN_BWD_BYTES, LN_STAT_BYTES, lib, stream_handle
from .plan import GraphPlan

L = 128

PARAM_SHAPES = [  # state_dict order of gnn_local_stress/models.py:246-286
    ("node_encoder.0.weight", (L, 6)), ("node_encoder.0.bias", (L,)),
    ("node_encoder.2.weight", (L, L)), ("node_encoder.2.bias", (L,)),
    ("node_encoder.4.weight", (L,)), ("node_encoder.4.bias", (L,)),
    ("edge_encoder.0.weight", (L, 1)), ("edge_encoder.0.bias", (L,)),
    ("edge_encoder.2.weight", (L, L)), ("edge_encoder.2.bias", (L,)),
    ("edge_encoder.4.weight", (L,)), ("edge_encoder.4.bias", (L,)),
    ("processor.edge_net.0.weight", (L, 3 * L)), ("processor.edge_net.0.bias", (L,)),
    ("processor.edge_net.2.weight", (L, L)), ("processor.edge_net.2.bias", (L,)),
    ("processor.edge_net.4.weight", (L,)), ("processor.edge_net.4.bias", (L,)),
    ("processor.node_net.0.weight", (L, 2 * L)), ("processor.node_net.0.bias", (L,)),
    ("processor.node_net.2.weight", (L, L)), ("processor.node_net.2.bias", (L,)),
    ("processor.node_net.4.weight", (L,)), ("processor.node_net.4.bias", (L,)),
    ("node_decoder.0.weight", (L, L)), ("node_decoder.0.bias", (L,)),
    ("node_decoder.2.weight", (3, L)), ("node_decoder.2.bias", (3,)),
]
PARAM_NAMES = [n for n, _ in PARAM_SHAPES]


def _p(t):
    return None if t is None else t.data_ptr()


# Kernel variants of the engine: attribute -> (A/B environment variable, shipped default).  The
# defaults are the product path, the only one the full-size parity tests (tests/test_gpu_fullsize.py)
# and the bench time; the alternatives are kept for same-box A/B timing (tools/ab_env.sh) and are
# checked against the defaults by the GPU op / model tests.  Tests select them through the engine
# attributes; the environment is read only under PDG_AB=1, and a non-default value set in the
# environment without it is an error (a stray variable must not swap kernels silently).
VARIANTS = {
    # edge backward with the W2 / Wc weight gradients fused (pdg_edge_bwd_w2 / pdg_edge_gout_wc); False:
    # pdg_edge_bwd + deferred pdg_wgrad_segments passes
    "fused_edge_wgrad": ("PDG_FUSED_EDGE_WGRAD", True),
    # P/Q gather backward before the Wc pass (gz1m / gz1e re-read while still in the Infinity Cache:
    # pq_scatter_bwd 63.6 -> 59.7 us and edge_gout_wc 145 -> 140 us per call, same box)
    "pq_first": ("PDG_PQ_FIRST", True),
    # fused edge backward: gz1e not stored; the P/Q gather backward forms it per row as gC - gz1m (one fp32
    # rounding of |gC|) from the gC rows the Wc pass reads anyway: one E-row array written fewer per step
    "gz1e_from_gc": ("PDG_GZ1E_FROM_GC", True),
    # edge forward in the block-cooperative layout (pdg_edge_fwd_coop; 240 -> 230 us per call at config 2)
    # instead of pdg_edge_fwd
    "coop_fwd": ("PDG_EDGE_FWD_COOP", True),
    # inference (no backward): the edge forward of at least INFER_PIPE_MIN_EDGES edges in 16-row rounds with one
    # barrier per round (pdg_edge_fwd_infer; bitwise the same rows): 494 -> 446 us per 614k-edge call
    "fwd_infer_pipe": ("PDG_EDGE_FWD_INFER", True),
    # the backward's input gradient of x (gP, gQ -> gx) in bf16x6 (pdg_gemm_sum2_coop) instead of the fp32-MFMA
    # pdg_gemm_sum2_rw
    "gsum2_coop": ("PDG_GSUM2_COOP", True),
    # node_net backward likewise (pdg_node_bwd_coop, three W^T products in bf16x6), and the cooperative
    # node-encoder / decoder backward
    "nbwd_coop": ("PDG_NODE_BWD_COOP", True),
    # pdg_wgrad_pairs blocks per CU (2 per CU ran as two sequential block waves at 166 VGPRs: 9.07-9.12 vs
    # 9.14-9.23 ms per config-2 step, same box)
    "pair_blocks_per_cu": ("PDG_PAIR_BLOCKS_PER_CU", 1),
    # the node encoder in the cooperative layout with an unbiased bf16x6 W2 product (pdg_node_enc_fwd) instead of
    # the LDS-weight fp32-MFMA pdg_encoder_fwd
    "node_enc_coop": ("PDG_NODE_ENC_COOP", True),
    # the decoder likewise (pdg_decoder_fwd_coop) instead of the LDS-weight pdg_decoder_fwd[_fin]
    "decoder_coop": ("PDG_DECODER_COOP", True),
    # pdg_edge_enc_fwd blocks per CU (104 VGPRs, 41 KB LDS per 8-wave block)
    "enc_blocks_per_cu": ("PDG_ENC_BLOCKS_PER_CU", 2),
}


# pdg_edge_fwd_infer from this many edges on (alone, 256 blocks: +1.5 us against pdg_edge_fwd_coop at 2.5k - 11k
# edges, equal at 27k, -3 us at 59k, -10 % from 150k edges on; tools/diag/efwd_sweep.py)
INFER_PIPE_MIN_EDGES = 32768


def _parse_variant(name: str, raw: str):
    env, default = VARIANTS[name]
    if isinstance(default, bool):
        if raw not in ("0", "1"):
            raise ValueError(f"{env}={raw!r}: expected 0 or 1")
        return raw == "1"
    try:
        v = int(raw)
    except ValueError:
        raise ValueError(f"{env}={raw!r}: expected an integer") from None
    if v < 1 or v > 4:
        raise ValueError(f"{env}={raw!r}: expected 1..4")
    return v


def kernel_variants(overrides: dict | None = None) -> dict:
    """The variant settings an engine starts with: the shipped defaults, the environment's A/B
    selection under PDG_AB=1 (refused without it unless every value equals the default), then
    ``overrides``."""
    out = {k: d for k, (_, d) in VARIANTS.items()}
    ab = os.environ.get("PDG_AB") == "1"
    for name, (env, default) in VARIANTS.items():
        raw = os.environ.get(env)
        if raw is None:
            continue
        val = _parse_variant(name, raw)
        if val != default and not ab:
            raise RuntimeError(f"{env}={raw} selects a non-default kernel variant of the HIP path; these are "
                               "for A/B timing only (set PDG_AB=1 to allow them), unset it to run the shipped "
                               "kernels")
        out[name] = val
    for k, v in (overrides or {}).items():
        if k not in VARIANTS:
            raise KeyError(f"unknown kernel variant {k!r} (known: {sorted(VARIANTS)})")
        out[k] = v
    return out


class _StatBuf:
    """A device array of pdg_ln_stat (or pdg_ln_bwd) structs."""

    def __init__(self, n: int, nbytes: int, device, zero: bool = True) -> None:
        # zero=False: every entry is written (pdg_ln_finalize / the producers' fused finalize) before
        # it is read, so no fill launch
        alloc = torch.zeros if zero else torch.empty
        self.buf = alloc(max(n, 1) * nbytes, dtype=torch.uint8, device=device)
        self.nbytes = nbytes

    def __getitem__(self, i: int) -> int:
        return self.buf.data_ptr() + i * self.nbytes


@dataclass
class FwdCtx:
    plan: GraphPlan
    steps: int
    scale_output: bool
    x_in: torch.Tensor = None
    e_in: torch.Tensor = None
    a1_ne: torch.Tensor = None
    a2_ne: torch.Tensor = None
    a1_ee: torch.Tensor = None
    a2_ee: torch.Tensor = None
    per_step: list = field(default_factory=list)
    x_S: torch.Tensor = None
    a1d: torch.Tensor = None
    stats: _StatBuf = None


class EPDEngine:
    """Stateless executor; parameters are passed per call as a name->tensor dict."""

    def __init__(self, device: torch.device, variants: dict | None = None) -> None:
        self.device = torch.device(device)
        var = kernel_variants(variants)
        self.max_blocks = lib.pdg_max_blocks()
        f64 = dict(dtype=torch.float64, device=self.device)
        self._part_a = torch.empty(self.max_blocks * 2, **f64)
        self._part_b = torch.empty(self.max_blocks * 2, **f64)
        self._part_col = torch.empty(self.max_blocks * 256, **f64)
        # LayerNorm backward (no finalize launches, pdg_ln_colsum in include/pdivgnn.h): per-block
        # column accumulators of the 4 LayerNorm parameter groups (node_net, edge_net, node and edge
        # encoder), rows <= the largest producer grid (2 x CUs), zeroed once per backward
        self._acc_rows = min(2 * torch.cuda.get_device_properties(self.device).multi_processor_count,
                             self.max_blocks)
        self._ln_acc = torch.zeros(4, self._acc_rows * 256, **f64)
        self._sync_pairs = torch.zeros(8, 2, **f64)
        self._part_narrow = torch.empty(self.max_blocks * (L * 6 + L + 6), **f64)
        # block partials of the two narrow gradients formed inside the encoder / decoder backward, held until
        # the backward's epilogue (apart from _part_narrow, the scratch of pdg_wgrad_narrow)
        self._part_narrow_d = torch.empty(self.max_blocks * (L * 3 + L + 3), **f64)
        self._part_narrow_ne = torch.empty(self.max_blocks * (L * 6 + L + 6), **f64)
        self._nparts = ctypes.c_int(0)
        # one weight-gradient slab per block of pdg_wgrad_segments: three blocks per CU
        self._nslabs = lib.pdg_wgrad_slabs_per_cu() * torch.cuda.get_device_properties(self.device).multi_processor_count
        self._nslabs_p = min(var["pair_blocks_per_cu"] *
                             torch.cuda.get_device_properties(self.device).multi_processor_count, lib.pdg_max_blocks())
        self._pair = torch.zeros(2, **f64)
        self.sync = None
        # kernel variants (VARIANTS above; tests and A/B tools flip these attributes)
        self.fused_edge_wgrad = var["fused_edge_wgrad"]
        self.pq_first = var["pq_first"]
        self.gz1e_from_gc = var["gz1e_from_gc"]
        self.coop_fwd = var["coop_fwd"]
        self.fwd_infer_pipe = var["fwd_infer_pipe"]
        self.node_enc_coop = var["node_enc_coop"]
        self.decoder_coop = var["decoder_coop"]
        # the P / Q layout the library's node pre-pass writes and its cooperative edge forward reads
        self.pq_blocked = bool(lib.pdg_pq_layout())
        self._nslabs_e = min(torch.cuda.get_device_properties(self.device).multi_processor_count,
                             lib.pdg_max_blocks())
        self.gsum2_coop = var["gsum2_coop"]
        self.nbwd_coop = var["nbwd_coop"]
        self._enc_blocks = min(var["enc_blocks_per_cu"] *
                               torch.cuda.get_device_properties(self.device).multi_processor_count, lib.pdg_max_blocks())
        # optional live kernel timing: name -> list of (start, end) hiptimer.Event pairs
        self.timed: dict | None = None
        # optional backward probe (tools/grad_err_stages.py): step t -> copies of d loss / d x_t,
        # d loss / d e_t (edges in plan order) and d loss / d aggr_t
        self.probe: dict | None = None

    def variants(self) -> dict:
        """The kernel variants in effect (recorded in the bench line): every VARIANTS entry, so a new
        variant cannot be left out of the record."""
        cus = torch.cuda.get_device_properties(self.device).multi_processor_count
        derived = {"pair_blocks_per_cu": self._nslabs_p // cus, "enc_blocks_per_cu": self._enc_blocks // cus}
        return {k: derived[k] if k in derived else getattr(self, k) for k in VARIANTS}

    def _t(self, name: str, fn, *args):
        """Launch fn(*args); when timing is enabled for `name`, bracket it with HIP events
        on the current stream (the stream every launch of this engine uses)."""
        if self.timed is None or name not in self.timed:
            return fn(*args)
        a, b = hiptimer.Event(), hiptimer.Event()   # no system-scope fence per record (pdg/hiptimer.py)
        a.record()
        r = fn(*args)
        b.record()
        self.timed[name].append((a, b))
        return r

    # ------------------------------------------------------------------ helpers
    def _empty(self, *shape):
        return torch.empty(*shape, dtype=torch.float32, device=self.device)

    def _finalize(self, part, count: int, out_ptr: int, s, edges: bool = False) -> None:
        if self.sync is None:
            lib.pdg_ln_finalize(part.data_ptr(), self._nparts.value, float(count), out_ptr, s)
            return
        # exact DP LayerNorm: statistics of the whole minibatch over all ranks
        group, n_glob, e_glob = self.sync
        lib.pdg_ln_partials_sum(part.data_ptr(), self._nparts.value, self._pair.data_ptr(), s)
        self._t("sync_collective", lambda: torch.distributed.all_reduce(self._pair, group=group))
        lib.pdg_ln_finalize(self._pair.data_ptr(), 1, float((e_glob if edges else n_glob) * L), out_ptr, s)

    def set_sync(self, group, n_nodes_global: int = 0, n_edges_global: int = 0) -> None:
        """Enable (group given) or disable (None) the exact data-parallel LayerNorm: every
        graph-LayerNorm of forward and backward uses the statistics of the global minibatch
        of n_nodes_global / n_edges_global rows, as one device running all of it would."""
        self.sync = None if group is None else (group, int(n_nodes_global), int(n_edges_global))

    # ------------------------------------------------------------------ forward
    def forward(self, P: dict, stats8: torch.Tensor, plan: GraphPlan, pos, mean_stress, nodes_types,
                edge_attr, steps: int, scale_input: bool, scale_output: bool, need_grad: bool):
        s = stream_handle(self.device)
        N, E = plan.n_nodes, plan.n_edges
        if N == 0:
            raise ValueError("empty graph")
        # E == 0 (an edgeless batch): as in the reference, every message aggregate is zero
        # (scatter of no rows), the edge branch produces empty tensors and the edge parameters get
        # zero gradients; the edge kernels are skipped
        if E == 0 and self.sync is not None:
            raise ValueError("exact (sync) data parallelism needs edges on every rank's shard")
        np_ = ctypes.byref(self._nparts)
        ctx = FwdCtx(plan=plan, steps=steps, scale_output=scale_output)
        # without edges the edge LayerNorms' entries are never finalized (zeros keep them finite)
        ctx.stats = _StatBuf(2 + 3 * steps, LN_STAT_BYTES, self.device, zero=E == 0)
        st = ctx.stats
        x_in = self._empty(N, 6)
        e_in = self._empty(E)
        lib.pdg_format_inputs(N, E, _p(pos), _p(mean_stress), _p(nodes_types), _p(edge_attr), _p(plan.perm),
                              _p(stats8), int(scale_input), _p(x_in), _p(e_in), s)
        # encoders (models.py:308-309)
        a1_ne, a2_ne = self._empty(N, L), self._empty(N, L)
        if self.node_enc_coop:
            nb = self._nslabs_e   # one 8-wave block per CU (168 VGPRs)
            self._t("node_enc_fwd", lib.pdg_node_enc_fwd, N, _p(x_in), _p(P["node_encoder.0.weight"]),
                    _p(P["node_encoder.0.bias"]), _p(P["node_encoder.2.weight"]), _p(P["node_encoder.2.bias"]),
                    _p(a1_ne), _p(a2_ne), _p(self._part_b), nb, s)
            self._nparts.value = nb
        else:
            lib.pdg_encoder_fwd(N, 6, _p(x_in), _p(P["node_encoder.0.weight"]), _p(P["node_encoder.0.bias"]),
                                _p(P["node_encoder.2.weight"]), _p(P["node_encoder.2.bias"]), _p(a1_ne), _p(a2_ne),
                                _p(self._part_b), np_, s)
        # the node encoder's LayerNorm statistics are reduced inside step 0's node_pq (pdg_node_pq_rw_fin, as
        # every later step's; one launch fewer), its partials in _part_b until then (the edge encoder and the
        # first edge forward write _part_a / _part_b only after that node_pq)
        pend_n, pend_buf = None, self._part_b
        if self.sync is None:
            pend_n = self._nparts.value
        else:
            self._finalize(self._part_b, N * L, st[0], s)
        # the edge encoder's layer-1 output is stored only for the unfused backward (pdg_mlp2_bwd);
        # pdg_edge_enc_bwd recomputes it from the scalar input
        a1_ee = self._empty(E, L) if (need_grad and not self.fused_edge_wgrad) else None
        a2_ee = self._empty(E, L)
        if E and a1_ee is None:   # bf16x6 W2 product, register-stationary (pdg_edge_enc_fwd)
            nb = self._enc_blocks
            self._t("edge_enc_fwd", lib.pdg_edge_enc_fwd, E, _p(e_in), _p(P["edge_encoder.0.weight"]),
                    _p(P["edge_encoder.0.bias"]), _p(P["edge_encoder.2.weight"]), _p(P["edge_encoder.2.bias"]),
                    _p(a2_ee), _p(self._part_a), nb, s)
            self._nparts.value = nb
            self._finalize(self._part_a, E * L, st[1], s, True)
        elif E:
            lib.pdg_encoder_fwd(E, 1, _p(e_in), _p(P["edge_encoder.0.weight"]), _p(P["edge_encoder.0.bias"]),
                                _p(P["edge_encoder.2.weight"]), _p(P["edge_encoder.2.bias"]), _p(a1_ee), _p(a2_ee),
                                _p(self._part_a), np_, s)
            self._finalize(self._part_a, E * L, st[1], s, True)
        if need_grad:
            ctx.x_in, ctx.e_in, ctx.a1_ne, ctx.a2_ne, ctx.a1_ee, ctx.a2_ee = x_in, e_in, a1_ne, a2_ne, a1_ee, a2_ee

        W1, b1 = P["processor.edge_net.0.weight"], P["processor.edge_net.0.bias"]
        W2, b2 = P["processor.edge_net.2.weight"], P["processor.edge_net.2.bias"]
        ge, be = P["processor.edge_net.4.weight"], P["processor.edge_net.4.bias"]
        Wn1, bn1 = P["processor.node_net.0.weight"], P["processor.node_net.0.bias"]
        Wn2, bn2 = P["processor.node_net.2.weight"], P["processor.node_net.2.bias"]
        gn, bnn = P["processor.node_net.4.weight"], P["processor.node_net.4.bias"]

        a2n_prev, stn_prev, gn_prev, bn_prev = a2_ne, st[0], P["node_encoder.4.weight"], P["node_encoder.4.bias"]
        a2e_prev, ste_prev, ge_prev, be_prev = a2_ee, st[1], P["edge_encoder.4.weight"], P["edge_encoder.4.bias"]
        x_prev = e_prev = None
        if self.pq_blocked:   # one N x 256 array, Q's blocks 16 floats after P's (pdg_pq_layout)
            PQm = self._empty(N, 2 * L)
            Pm, Qm = PQm, PQm.view(-1)[16:]
        else:
            Pm, Qm = self._empty(N, L), self._empty(N, L)
        # pend_n: deferred node LayerNorm statistics (nparts of the partials in pend_buf)
        for t in range(steps):
            i_m, i_e, i_n = 2 + 3 * t, 3 + 3 * t, 4 + 3 * t
            x_t = self._empty(N, L)
            if pend_n is not None:    # the previous step's node statistics, reduced inside node_pq
                self._t("node_pq", lib.pdg_node_pq_rw_fin, N, _p(a2n_prev), pend_buf.data_ptr(), pend_n,
                        float(N * L), stn_prev, _p(gn_prev), _p(bn_prev), _p(x_prev), _p(x_t), _p(W1), _p(Pm),
                        _p(Qm), s)
                pend_n = None
            else:
                self._t("node_pq", lib.pdg_node_pq_rw, N, _p(a2n_prev), stn_prev, _p(gn_prev), _p(bn_prev),
                        _p(x_prev), _p(x_t), _p(W1), _p(Pm), _p(Qm), s)
            # the last step's edge update has no consumer (models.py:316 decodes nodes only)
            eu = t < steps - 1
            e_t = self._empty(E, L)
            a2m = self._empty(E, L)
            a1m = self._empty(E, L) if need_grad else None   # layer-1 outputs: backward only
            a2e = self._empty(E, L) if eu else None
            a1e = self._empty(E, L) if (eu and need_grad) else None
            if E and self.coop_fwd and not need_grad and self.fwd_infer_pipe and E >= INFER_PIPE_MIN_EDGES:
                self._t("edge_fwd" if eu else "edge_fwd_last", lib.pdg_edge_fwd_infer, E, _p(a2e_prev), ste_prev,
                        _p(ge_prev), _p(be_prev), _p(e_prev), _p(e_t), _p(plan.src), _p(plan.dst), _p(Pm), _p(Qm),
                        _p(W1), _p(b1), _p(W2), _p(b2), _p(a2m), _p(a2e), _p(self._part_a), _p(self._part_b), int(eu),
                        self._nslabs_e, s)
                self._nparts.value = self._nslabs_e
            elif E and self.coop_fwd:
                self._t("edge_fwd" if eu else "edge_fwd_last", lib.pdg_edge_fwd_coop, E, _p(a2e_prev), ste_prev,
                        _p(ge_prev), _p(be_prev), _p(e_prev), _p(e_t), _p(plan.src), _p(plan.dst), _p(Pm), _p(Qm),
                        _p(W1), _p(b1), _p(W2), _p(b2), _p(a1m), _p(a2m), _p(a1e), _p(a2e), _p(self._part_a),
                        _p(self._part_b), int(eu), self._nslabs_e, s)
                self._nparts.value = self._nslabs_e
            elif E:
                Pu, Qu = Pm, Qm
                if self.pq_blocked:   # pdg_edge_fwd (the A/B / reference kernel) reads two N x 128 arrays
                    v = PQm.view(N, 8, 2, 16)
                    Pu, Qu = v[:, :, 0].reshape(N, L).contiguous(), v[:, :, 1].reshape(N, L).contiguous()
                self._t("edge_fwd" if eu else "edge_fwd_last", lib.pdg_edge_fwd, E, _p(a2e_prev), ste_prev, _p(ge_prev), _p(be_prev), _p(e_prev),
                        _p(e_t), _p(plan.src), _p(plan.dst), _p(Pu), _p(Qu), _p(W1), _p(b1), _p(W2), _p(b2),
                        _p(a1m), _p(a2m), _p(a1e), _p(a2e), _p(self._part_a), _p(self._part_b), int(eu), np_, s)
            fin_in_segsum = bool(E) and self.sync is None   # reduced inside pdg_segment_sum_fin
            if E and not fin_in_segsum:
                if eu and self.sync is None:    # both edge LayerNorms in one launch
                    lib.pdg_ln_finalize2(self._part_a.data_ptr(), self._part_b.data_ptr(), self._nparts.value,
                                         float(E * L), st[i_m], st[i_e], s)
                else:
                    self._finalize(self._part_a, E * L, st[i_m], s, True)
                    if eu:
                        self._finalize(self._part_b, E * L, st[i_e], s, True)
            # aggregation (models.py:215-217) and node_net (:240-243)
            a1n = self._empty(N, L) if need_grad else None
            a2n = self._empty(N, L)
            if E:
                aggr = self._empty(N, L)
                xs = self._empty(N, L) if need_grad else None
                if fin_in_segsum:   # + both edge LayerNorms' statistics from the edge forward's partials
                    self._t("segment_sum", lib.pdg_segment_sum_fin, N, _p(plan.rowptr_dst), _p(a2m),
                            _p(self._part_a), _p(self._part_b) if eu else None, self._nparts.value, float(E * L),
                            st[i_m], st[i_e] if eu else None, _p(ge), _p(be), _p(aggr), _p(xs), s)
                else:
                    self._t("segment_sum", lib.pdg_segment_sum, N, _p(plan.rowptr_dst), _p(a2m), st[i_m], _p(ge),
                            _p(be), _p(aggr), _p(xs), s)
            else:
                aggr = torch.zeros(N, L, dtype=torch.float32, device=self.device)
                xs = torch.zeros(N, L, dtype=torch.float32, device=self.device) if need_grad else None
            self._t("node_net", lib.pdg_node_net, N, _p(aggr), _p(x_t), _p(Wn1), _p(bn1), _p(Wn2), _p(bn2), _p(a1n),
                    _p(a2n), _p(self._part_a), np_, s)
            if self.sync is None:
                # finalised by the next step's node_pq, or by the decoder after the last step
                pend_n, pend_buf = self._nparts.value, self._part_a
            else:
                self._finalize(self._part_a, N * L, st[i_n], s)
            if need_grad:
                ctx.per_step.append(dict(x=x_t, e=e_t, a1m=a1m, a2m=a2m, a1e=a1e, a2e=a2e, aggr=aggr, xs=xs,
                                         a1n=a1n, a2n=a2n, i_m=i_m, i_e=i_e, i_n=i_n, eu=eu))
            a2n_prev, stn_prev, gn_prev, bn_prev = a2n, st[i_n], gn, bnn
            a2e_prev, ste_prev, ge_prev, be_prev = a2e, st[i_e], ge, be
            x_prev, e_prev = x_t, e_t
        # decoder (models.py:316-321)
        x_S, a1d, y = self._empty(N, L), self._empty(N, L), self._empty(N, 3)
        if x_prev is None:
            raise ValueError("message_passing_steps must be >= 1")
        if self.decoder_coop:   # (pend_n: the last node LayerNorm's statistics reduced inside the decoder)
            self._t("decoder_fwd", lib.pdg_decoder_fwd_coop, N, _p(a2n_prev), None if pend_n is not None else stn_prev,
                    pend_buf.data_ptr() if pend_n is not None else None, pend_n or 0, float(N * L),
                    stn_prev if pend_n is not None else None, _p(gn_prev), _p(bn_prev), _p(x_prev), _p(x_S),
                    _p(P["node_decoder.0.weight"]), _p(P["node_decoder.0.bias"]), _p(a1d),
                    _p(P["node_decoder.2.weight"]), _p(P["node_decoder.2.bias"]), _p(stats8), int(scale_output),
                    _p(y), self._nslabs_e, s)
        elif pend_n is not None:   # the last node LayerNorm's statistics reduced inside the decoder
            lib.pdg_decoder_fwd_fin(N, _p(a2n_prev), pend_buf.data_ptr(), pend_n, float(N * L), stn_prev,
                                    _p(gn_prev), _p(bn_prev), _p(x_prev), _p(x_S), _p(P["node_decoder.0.weight"]),
                                    _p(P["node_decoder.0.bias"]), _p(a1d), _p(P["node_decoder.2.weight"]),
                                    _p(P["node_decoder.2.bias"]), _p(stats8), int(scale_output), _p(y), s)
        else:
            lib.pdg_decoder_fwd(N, _p(a2n_prev), stn_prev, _p(gn_prev), _p(bn_prev), _p(x_prev), _p(x_S),
                                _p(P["node_decoder.0.weight"]), _p(P["node_decoder.0.bias"]), _p(a1d),
                                _p(P["node_decoder.2.weight"]), _p(P["node_decoder.2.bias"]), _p(stats8),
                                int(scale_output), _p(y), s)
        if need_grad:
            ctx.x_S, ctx.a1d = x_S, a1d
        return y, ctx

    # ------------------------------------------------------------------ backward
    def transposed(self, P: dict) -> dict:
        """W^T copies of every weight block the backward GEMMs read."""
        s = stream_handle(self.device)
        out = {}
        jobs = []

        def tr(name, key, col0, ld):
            out[key] = T = self._empty(L, L)
            jobs.append((P[name].data_ptr() + 4 * col0, ld, T.data_ptr()))

        tr("node_decoder.0.weight", "Wd1T", 0, L)
        tr("processor.edge_net.2.weight", "W2T", 0, L)
        tr("processor.edge_net.0.weight", "WaT", 0, 3 * L)
        tr("processor.edge_net.0.weight", "WbT", L, 3 * L)
        tr("processor.edge_net.0.weight", "WcT", 2 * L, 3 * L)
        tr("processor.node_net.2.weight", "Wn2T", 0, L)
        tr("processor.node_net.0.weight", "Wn1aT", 0, 2 * L)
        tr("processor.node_net.0.weight", "Wn1bT", L, 2 * L)
        tr("node_encoder.2.weight", "Wne2T", 0, L)
        tr("edge_encoder.2.weight", "Wee2T", 0, L)
        n = len(jobs)
        lib.pdg_transpose128_batch(n, (ctypes.c_void_p * n)(*[j[0] for j in jobs]), (ctypes.c_int * n)(*[j[1] for j in jobs]),
                                   (ctypes.c_void_p * n)(*[j[2] for j in jobs]), s)
        return out

    def backward(self, P: dict, ctx: FwdCtx, gy: torch.Tensor, G: dict) -> None:
        """Accumulate d(loss)/d(param) into G[name] (fp32, same shapes as P).

        The input-gradient chain runs step by step (reverse order); the weight
        gradients of the shared 128x128 blocks are deferred: every step's row
        segments (G, X pairs, kept resident in HBM) are reduced at the end in
        one segmented MFMA pass per weight (pdg_wgrad_segments)."""
        s = stream_handle(self.device)
        plan = ctx.plan
        N, E = plan.n_nodes, plan.n_edges
        np_ = ctypes.byref(self._nparts)
        T = self.transposed(P)
        st = ctx.stats
        segs: dict[str, list] = {k: [] for k in ("W2", "Wc", "Wa", "Wb", "Wn2", "Wn1a", "Wn1b", "d1", "ne2", "ee2")}
        fused = self.fused_edge_wgrad
        # LayerNorm backward scalars without finalize launches: every column-sum producer adds its
        # per-block rows into the group accumulator and writes per-block (S1, S2) pairs; the consumer
        # kernel reduces the pairs (include/pdivgnn.h, pdg_ln_colsum)
        if fused:
            # the three fused weight-gradient slab sets (W2, Wc, the edge encoder's W2) are written by the
            # first call of the backward (slab_init) and need no fill; the LayerNorm column-sum
            # accumulators are zeroed (one fill launch)
            nse = self._nslabs_e
            # (an edgeless batch runs no edge kernel: zeros, so the edge weights get zero gradients)
            sl = (torch.empty if E else torch.zeros)(3, nse, L * L + L, dtype=torch.float32, device=self.device)
            slabs_w2, slabs_wc, slabs_ee = sl[0], sl[1], sl[2]
            acc = torch.zeros(self._ln_acc.shape, dtype=torch.float64, device=self.device)
        else:
            acc = self._ln_acc
            acc.zero_()
        reds = []   # deferred slab reductions (in the one pdg_bwd_epilogue launch at the end)
        epi_narrow = []   # narrow weight-gradient finalizes for pdg_bwd_epilogue
        epi_enc = None    # the edge encoder's first-layer sums for pdg_bwd_epilogue
        ACC_N, ACC_E, ACC_NE, ACC_EE = (acc[i] for i in range(4))
        S = ctx.steps
        pairs = torch.empty(3 * S + 2, self.max_blocks * 2, dtype=torch.float64, device=self.device)
        PN, PM, PE = (lambda t: pairs[t]), (lambda t: pairs[S + t]), (lambda t: pairs[2 * S + t])
        P_NENC, P_EENC = pairs[3 * S], pairs[3 * S + 1]
        g_node, g_edge = P["processor.node_net.4.weight"], P["processor.edge_net.4.weight"]
        sync_slot = [0]

        def src(pp, n):
            """(pairs pointer, count) for a consumer; sync DP mode reduces them first and
            all-reduces the (S1, S2) pair over the ranks (global-minibatch LayerNorm)."""
            if self.sync is None:
                return _p(pp), n
            out = self._sync_pairs[sync_slot[0] % 8]
            sync_slot[0] += 1
            lib.pdg_ln_partials_sum(_p(pp), n, _p(out), s)
            self._t("sync_collective", lambda: torch.distributed.all_reduce(out, group=self.sync[0]))
            return _p(out), 1

        def edge_ln_pairs(pp, gy_rows, a2, st_ptr, accb, g):
            """Pairs of the LayerNorm that produced an edge state e: fused mode has them from
            pdg_edge_gout_wc (written while producing gy_rows = d loss / d e)."""
            if not fused:
                lib.pdg_ln_colsum(E, _p(gy_rows), None, _p(a2), st_ptr, _p(accb), np_, _p(g), _p(pp), 1, s)
                return pp, self._nparts.value
            return pp, nse

        gy = gy.contiguous()
        if ctx.scale_output:
            gy = gy * P["_std_local_stress"]
        # decoder
        gz1d, gx = self._empty(N, L), self._empty(N, L)
        dl = ctx.per_step[S - 1]
        if self.nbwd_coop:   # + the column sums of the last node LayerNorm (upstream gradient: gx)
            # + node_decoder.2's weight / bias gradient from the same a1d / gy rows (block partials)
            self._t("decoder_bwd", lib.pdg_decoder_bwd_coop, N, _p(gy), _p(ctx.a1d), _p(P["node_decoder.2.weight"]),
                    _p(T["Wd1T"]), _p(gz1d), _p(gx), _p(dl["a2n"]), st[dl["i_n"]], _p(ACC_N), _p(g_node),
                    _p(PN(S - 1)), 1, _p(self._part_narrow_d), self._nslabs_e, s)
            self._nparts.value = self._nslabs_e
            epi_narrow.append((self._part_narrow_d, self._nslabs_e, 3, 1, G["node_decoder.2.weight"], None,
                               G["node_decoder.2.bias"]))
        else:
            lib.pdg_decoder_bwd(N, _p(gy), _p(ctx.a1d), _p(P["node_decoder.2.weight"]), _p(T["Wd1T"]), _p(gz1d),
                                _p(gx), s)
            lib.pdg_wgrad_narrow(N, _p(ctx.a1d), _p(gy), 3, 1, _p(self._part_narrow), _p(G["node_decoder.2.weight"]),
                                 None, _p(G["node_decoder.2.bias"]), s)
        segs["d1"].append((gz1d, ctx.x_S, N))

        ge_next = None              # d loss / d e_S: the last edge update has no consumer
        gaggr, gx_part, gx_t = (self._empty(N, L) for _ in range(3))
        e_sum = fused and self.gz1e_from_gc   # gz1e never stored: pdg_pq_scatter_bwd takes gC - gz1m
        gz1m = self._empty(E, L)
        gz1e = None if e_sum else self._empty(E, L)
        ge_bufs = [self._empty(E, L), self._empty(E, L)]
        gC_fused = self._empty(E, L) if fused else None
        gx_next = gx
        # node LayerNorm of the last step (upstream gradient: the decoder's); for the earlier steps
        # the previous iteration's pdg_gemm_sum2_rw produces these partials
        if not self.nbwd_coop:
            lib.pdg_ln_colsum(N, _p(gx_next), None, _p(dl["a2n"]), st[dl["i_n"]], _p(ACC_N), np_, _p(g_node),
                              _p(PN(S - 1)), 1, s)
        n_node = self._nparts.value
        n_edge = 0
        for t in reversed(range(S)):
            d = ctx.per_step[t]
            eu = d["eu"]
            assert E == 0 or eu == (ge_next is not None)
            gz2n, gz1n, gP, gQ = (self._empty(N, L) for _ in range(4))
            gC = gC_fused if fused else self._empty(E, L)   # fused: consumed within the step
            if fused and not eu:
                gC = gz1m   # message branch only: gC = gz1m, written once (pdg_edge_bwd_w2)
            gz2m = None if fused else self._empty(E, L)
            gz2e = self._empty(E, L) if (eu and not fused) else None
            ge_out = ge_bufs[t % 2]
            # node_net backward (n_t = LN_n(a2n_t), gy = gx_next; x_{t+1} = n_t + x_t)
            pn, nn = src(PN(t), n_node)
            if self.nbwd_coop:
                self._t("node_bwd", lib.pdg_node_bwd_coop, N, _p(gx_next), _p(d["a2n"]), _p(d["a1n"]),
                        st[d["i_n"]], None, _p(g_node), _p(T["Wn2T"]), _p(T["Wn1aT"]), _p(T["Wn1bT"]), _p(gz2n),
                        _p(gz1n), _p(gaggr), _p(gx_part), pn, nn, self._nslabs_e, s)
            else:
                self._t("node_bwd", lib.pdg_node_bwd, N, _p(gx_next), _p(d["a2n"]), _p(d["a1n"]), st[d["i_n"]],
                        None, _p(g_node), _p(T["Wn2T"]), _p(T["Wn1aT"]), _p(T["Wn1bT"]), _p(gz2n), _p(gz1n),
                        _p(gaggr), _p(gx_part), pn, nn, s)
            if E == 0:             # no edge: P and Q feed nothing (models.py:215-222 on empty tensors)
                gP.zero_()
                gQ.zero_()
            else:
                # message LayerNorm: gy = gaggr[dst], summed per node with the forward's sum of xhat
                lib.pdg_ln_colsum_nodes(N, _p(gaggr), _p(plan.rowptr_dst), _p(d["xs"]), _p(ACC_E), np_, _p(g_edge),
                                        _p(PM(t)), 1, s)
                pm, nm = src(PM(t), self._nparts.value)
                pe, ne = None, 0
                if eu:   # edge-update LayerNorm: gy = ge_next (per edge)
                    pp, n_e = edge_ln_pairs(PE(t), ge_next, d["a2e"], st[d["i_e"]], ACC_E, g_edge)
                    pe, ne = src(pp, n_e if not fused else n_edge)
                if fused:
                    self._t("edge_bwd" if eu else "edge_bwd_last", lib.pdg_edge_bwd_w2, E, _p(plan.dst), _p(gaggr),
                            _p(ge_next), _p(d["a2m"]), _p(d["a1m"]), _p(d["a2e"]), _p(d["a1e"]), st[d["i_m"]],
                            st[d["i_e"]] if eu else None, None, None, _p(g_edge), _p(T["W2T"]), _p(gz1m),
                            _p(gz1e if eu else None), _p(gC), _p(slabs_w2), nse, pm, nm, pe, ne, int(t == S - 1), s)
                    # the edge-update rows of the P/Q gather backward: gz1e, or gC (= gz1m + gz1e) with e_is_sum
                    ge_rows, e_is_sum = (gC, 1) if (e_sum and eu) else (gz1e if eu else None, 0)
                    # + the column sums / pairs of the LayerNorm that produced e_t (LN_e of step t-1, or the
                    # edge encoder's)
                    if t > 0:
                        a2ln, st_ln, accb, gl, pp = (ctx.per_step[t - 1]["a2e"], st[ctx.per_step[t - 1]["i_e"]], ACC_E,
                                                     g_edge, PE(t - 1))
                    else:
                        a2ln, st_ln, accb, gl, pp = ctx.a2_ee, st[1], ACC_EE, P["edge_encoder.4.weight"], P_EENC
                    tail = (_p(d["e"]), _p(ge_next), _p(T["WcT"]), _p(ge_out), _p(slabs_wc), nse, _p(a2ln), st_ln,
                            _p(accb), _p(gl), _p(pp), 1, int(t == S - 1), s)
                    gout_fn, gout_args = lib.pdg_edge_gout_wc, (E, _p(gC)) + tail
                    if not self.pq_first:
                        self._t("edge_gout", gout_fn, *gout_args)
                    n_edge = nse
                else:
                    self._t("edge_bwd" if eu else "edge_bwd_last", lib.pdg_edge_bwd, E, _p(plan.dst), _p(gaggr),
                            _p(ge_next), _p(d["a2m"]), _p(d["a1m"]), _p(d["a2e"]), _p(d["a1e"]), st[d["i_m"]],
                            st[d["i_e"]] if eu else None, None, None, _p(g_edge), _p(T["W2T"]), _p(T["WcT"]),
                            _p(gz2m), _p(gz1m), _p(gz2e), _p(gz1e if eu else None), _p(gC), _p(ge_out), pm, nm, pe, ne, s)
                    ge_rows, e_is_sum = gz1e if eu else None, 0
                self._t("pq_scatter_bwd", lib.pdg_pq_scatter_bwd, N, _p(plan.rowptr_dst), _p(plan.rowptr_src),
                        _p(plan.perm_src), _p(gz1m), _p(ge_rows), e_is_sum, _p(gP), _p(gQ), s)
                if fused and self.pq_first:   # gz1m / gz1e read while still in the Infinity Cache
                    self._t("edge_gout", gout_fn, *gout_args)
            # gx_t, with the column sums / pairs of the LayerNorm whose output it is the gradient of:
            # the node LayerNorm of step t-1, or the node encoder's
            if t > 0:
                a2n_prev, st_prev, accb, gl, pp = (ctx.per_step[t - 1]["a2n"], st[ctx.per_step[t - 1]["i_n"]], ACC_N,
                                                   g_node, PN(t - 1))
            else:
                a2n_prev, st_prev, accb, gl, pp = ctx.a2_ne, st[0], ACC_NE, P["node_encoder.4.weight"], P_NENC
            if self.gsum2_coop:
                self._t("gemm_sum2", lib.pdg_gemm_sum2_coop, N, _p(gP), _p(gQ), _p(T["WaT"]), _p(T["WbT"]),
                        _p(gx_part), _p(gx_t), _p(a2n_prev), st_prev, _p(accb), _p(gl), _p(pp), 1, self._nslabs_e, s)
                self._nparts.value = self._nslabs_e
            else:
                self._t("gemm_sum2", lib.pdg_gemm_sum2_rw, N, _p(gP), _p(gQ), _p(T["WaT"]), _p(T["WbT"]),
                        _p(gx_part), _p(gx_t), _p(a2n_prev), st_prev, _p(accb), np_, _p(gl), _p(pp), 1, s)
            n_node = self._nparts.value
            if not fused and E:
                segs["W2"].append((gz2m, d["a1m"], E))
                if eu:
                    segs["W2"].append((gz2e, d["a1e"], E))
                segs["Wc"].append((gC, d["e"], E))
            segs["Wa"].append((gP, d["x"], N))
            segs["Wb"].append((gQ, d["x"], N))
            segs["Wn2"].append((gz2n, d["a1n"], N))
            segs["Wn1a"].append((gz1n, d["aggr"], N))
            segs["Wn1b"].append((gz1n, d["x"], N))
            if self.probe is not None:
                self.probe[t] = dict(gx=gx_t.clone(), ge=ge_out.clone() if E else None, gaggr=gaggr.clone())
            gx_next, gx_t = gx_t, gx_next
            ge_next = ge_out
        # encoders
        gz2 = self._empty(N, L)
        gz1 = None if self.nbwd_coop else self._empty(N, L)
        pn, nn = src(P_NENC, n_node)
        if self.nbwd_coop:   # the node encoder's backward, bf16x6 (pdg_mlp2_bwd_coop), + its first layer's
            # weight / bias gradient from gz1 and the encoder input (block partials; gz1 is not stored)
            self._t("node_enc_bwd", lib.pdg_mlp2_bwd_coop, N, _p(gx_next), _p(ctx.a2_ne), _p(ctx.a1_ne), st[0], None,
                    _p(P["node_encoder.4.weight"]), _p(T["Wne2T"]), _p(gz2), None, pn, nn, _p(ctx.x_in),
                    _p(self._part_narrow_ne), self._nslabs_e, s)
            epi_narrow.append((self._part_narrow_ne, self._nslabs_e, 6, 0, G["node_encoder.0.weight"],
                               G["node_encoder.0.bias"], None))
        else:
            lib.pdg_mlp2_bwd(N, _p(gx_next), None, _p(ctx.a2_ne), _p(ctx.a1_ne), st[0], None,
                             _p(P["node_encoder.4.weight"]), _p(T["Wne2T"]), _p(gz2), _p(gz1), pn, nn, s)
            lib.pdg_wgrad_narrow(N, _p(gz1), _p(ctx.x_in), 6, 0, _p(self._part_narrow),
                                 _p(G["node_encoder.0.weight"]), _p(G["node_encoder.0.bias"]), None, s)
        segs["ne2"].append((gz2, ctx.a1_ne, N))
        if E:
            pp, n_e = edge_ln_pairs(P_EENC, ge_next, ctx.a2_ee, st[1], ACC_EE, P["edge_encoder.4.weight"])
            pe, ne = src(pp, n_e if not fused else n_edge)
            if fused:   # one pass: weight gradients in slabs (zeroed above), the 1 -> 128 layer's as per-block sums
                nsum = torch.empty(nse, 2 * L, dtype=torch.float64, device=self.device)
                self._t("edge_enc_bwd", lib.pdg_edge_enc_bwd, E, _p(ge_next), _p(ctx.a2_ee), _p(ctx.e_in),
                        _p(P["edge_encoder.0.weight"]), _p(P["edge_encoder.0.bias"]), st[1], None, pe, ne,
                        _p(P["edge_encoder.4.weight"]), _p(T["Wee2T"]), _p(slabs_ee), _p(nsum), nse, 1, s)
                reds.append((slabs_ee, nse, G["edge_encoder.2.weight"], L, 0, G["edge_encoder.2.bias"]))
                epi_enc = (nsum, nse, G["edge_encoder.0.weight"], G["edge_encoder.0.bias"])
            else:
                gz2e_, gz1e_ = self._empty(E, L), self._empty(E, L)
                lib.pdg_mlp2_bwd(E, _p(ge_next), None, _p(ctx.a2_ee), _p(ctx.a1_ee), st[1], None,
                                 _p(P["edge_encoder.4.weight"]), _p(T["Wee2T"]), _p(gz2e_), _p(gz1e_), pe, ne, s)
                segs["ee2"].append((gz2e_, ctx.a1_ee, E))
                lib.pdg_wgrad_narrow(E, _p(gz1e_), _p(ctx.e_in), 1, 0, _p(self._part_narrow),
                                     _p(G["edge_encoder.0.weight"]), _p(G["edge_encoder.0.bias"]), None, s)
        # deferred weight gradients: one segmented pass + slab reduction per shared weight block
        red = [
            ("W2", "processor.edge_net.2.weight", L, 0, "processor.edge_net.2.bias"),
            ("Wc", "processor.edge_net.0.weight", 3 * L, 2 * L, "processor.edge_net.0.bias"),
            ("Wa", "processor.edge_net.0.weight", 3 * L, 0, None),
            ("Wb", "processor.edge_net.0.weight", 3 * L, L, None),
            ("Wn2", "processor.node_net.2.weight", L, 0, "processor.node_net.2.bias"),
            ("Wn1a", "processor.node_net.0.weight", 2 * L, 0, "processor.node_net.0.bias"),
            ("Wn1b", "processor.node_net.0.weight", 2 * L, L, None),
            ("d1", "node_decoder.0.weight", L, 0, "node_decoder.0.bias"),
            ("ne2", "node_encoder.2.weight", L, 0, "node_encoder.2.bias"),
            ("ee2", "edge_encoder.2.weight", L, 0, "edge_encoder.2.bias"),
        ]
        ns = self._nslabs
        slab_sets = self.__dict__.setdefault("_slab_sets", {})

        def slab_set(key):
            """The slab set of one deferred weight (the reductions run batched at the end), allocated
            the first time that weight has a segment pass: with the fused edge backward and the pair
            passes only node_net.2, the decoder and the node encoder need one."""
            if key not in slab_sets:
                slab_sets[key] = torch.empty(ns, L * L + L, dtype=torch.float32, device=self.device)
            return slab_sets[key]
        # the weight pairs that share an operand, one pass each (pdg_wgrad_pairs): Wa / Wb against x
        # (gP, gQ), node_net.0's halves from gz1n (against aggr, x)
        nsp = self._nslabs_p
        if getattr(self, "_slabs_p", None) is None or self._slabs_p.device != self.device:
            self._slabs_p = torch.empty(2, 2, nsp, L * L + L, dtype=torch.float32, device=self.device)
        pairs_w = [
            (1, [(g, q, x, n) for (g, x, n), (q, _, _) in zip(segs.pop("Wa"), segs.pop("Wb"))],
             ("processor.edge_net.0.weight", 3 * L, 0, None), ("processor.edge_net.0.weight", 3 * L, L, None)),
            (0, [(g, a, x, n) for (g, a, n), (_, x, _) in zip(segs.pop("Wn1a"), segs.pop("Wn1b"))],
             ("processor.node_net.0.weight", 2 * L, 0, "processor.node_net.0.bias"),
             ("processor.node_net.0.weight", 2 * L, L, None)),
        ]
        def reduce_now_or_later(slabs, n, wname, ld, col0, bname, later):
            job = (slabs, n, G[wname], ld, col0, G[bname] if bname else None)
            if later:
                reds.append(job)
            else:   # a slab set reused by the next chunk: reduce before it is overwritten
                lib.pdg_wgrad_reduce(_p(slabs), n, _p(job[2]), ld, col0, _p(job[5]), s)

        for gi, (shx, sl, (w0n, ld0, c00, b0n), (w1n, ld1, c01, b1n)) in enumerate(pairs_w):
            sp0, sp1 = self._slabs_p[gi]
            for c0 in range(0, len(sl), 32):
                chunk = sl[c0:c0 + 32]
                n = len(chunk)
                arr = [(ctypes.c_void_p * n)(*[t[k].data_ptr() for t in chunk]) for k in range(3)]
                rw = (ctypes.c_int * n)(*[t[3] for t in chunk])
                self._t("wgrad_pair", lib.pdg_wgrad_pairs, n, arr[0], arr[1], arr[2], rw, shx, _p(sp0), _p(sp1), nsp,
                        s)
                later = len(sl) <= 32
                reduce_now_or_later(sp0, nsp, w0n, ld0, c00, b0n, later)
                reduce_now_or_later(sp1, nsp, w1n, ld1, c01, b1n, later)
        red_k = [r for r in red if r[0] in segs]
        # weights of at most 32 segments: up to three passes per launch (pdg_wgrad_segments_batch)
        small = [r for r in red_k if 0 < len(segs[r[0]]) <= 32]
        for c0 in range(0, len(small), 3):
            grp = small[c0:c0 + 3]
            segl = [segs[r[0]] for r in grp]
            flat = [t for sl in segl for t in sl]
            n = len(flat)
            self._t("wgrad_batch", lib.pdg_wgrad_segments_batch, len(grp),
                    (ctypes.c_int * len(grp))(*[len(sl) for sl in segl]),
                    (ctypes.c_void_p * n)(*[g.data_ptr() for g, _, _ in flat]),
                    (ctypes.c_void_p * n)(*[x.data_ptr() for _, x, _ in flat]),
                    (ctypes.c_int * n)(*[r for _, _, r in flat]),
                    (ctypes.c_void_p * len(grp))(*[_p(slab_set(k[0])) for k in grp]),
                    ns, s)
            for key, wname, ld, col0, bname in grp:
                reduce_now_or_later(slab_set(key), ns, wname, ld, col0, bname, True)
        for key, wname, ld, col0, bname in red_k:
            sl = segs[key]
            if len(sl) <= 32:
                continue
            slabs_k = slab_set(key)
            for c0 in range(0, len(sl), 32):
                chunk = sl[c0:c0 + 32]
                n = len(chunk)
                gp = (ctypes.c_void_p * n)(*[g.data_ptr() for g, _, _ in chunk])
                xp = (ctypes.c_void_p * n)(*[x.data_ptr() for _, x, _ in chunk])
                rw = (ctypes.c_int * n)(*[r for _, _, r in chunk])
                self._t("wgrad_" + key, lib.pdg_wgrad_segments, n, gp, xp, rw, _p(slabs_k), ns, s)
                reduce_now_or_later(slabs_k, ns, wname, ld, col0, bname, len(sl) <= 32)
        if fused:   # the slabs of the fused edge backward, accumulated over all steps
            reds.append((slabs_w2, nse, G["processor.edge_net.2.weight"], L, 0, G["processor.edge_net.2.bias"]))
            reds.append((slabs_wc, nse, G["processor.edge_net.0.weight"], 3 * L, 2 * L,
                         G["processor.edge_net.0.bias"]))
        # every end-of-backward reduction in one launch (pdg_bwd_epilogue): the deferred slab reductions,
        # the LayerNorm weight / bias gradients of the four accumulator groups, the narrow weight gradients
        # and the edge encoder's first layer (more than 16 slab sets: the rest in pdg_wgrad_reduce_batch)
        VP, IA = ctypes.c_void_p, ctypes.c_int
        for c0 in range(16, len(reds), 16):
            jb = reds[c0:c0 + 16]
            n = len(jb)
            lib.pdg_wgrad_reduce_batch(n, (VP * n)(*[_p(j[0]) for j in jb]), (IA * n)(*[j[1] for j in jb]),
                                       (VP * n)(*[_p(j[2]) for j in jb]), (IA * n)(*[j[3] for j in jb]),
                                       (IA * n)(*[j[4] for j in jb]), (VP * n)(*[_p(j[5]) for j in jb]), s)
        jb = reds[:16]
        n = len(jb)
        names = ("processor.node_net.4", "processor.edge_net.4", "node_encoder.4", "edge_encoder.4")
        m = len(epi_narrow)
        lib.pdg_bwd_epilogue(n, (VP * n)(*[_p(j[0]) for j in jb]), (IA * n)(*[j[1] for j in jb]),
                             (VP * n)(*[_p(j[2]) for j in jb]), (IA * n)(*[j[3] for j in jb]),
                             (IA * n)(*[j[4] for j in jb]), (VP * n)(*[_p(j[5]) for j in jb]),
                             4, (VP * 4)(*[_p(acc[i]) for i in range(4)]), (IA * 4)(*([self._acc_rows] * 4)),
                             (VP * 4)(*[_p(G[k + ".weight"]) for k in names]),
                             (VP * 4)(*[_p(G[k + ".bias"]) for k in names]),
                             m, (VP * m)(*[_p(j[0]) for j in epi_narrow]), (IA * m)(*[j[1] for j in epi_narrow]),
                             (IA * m)(*[j[2] for j in epi_narrow]), (IA * m)(*[j[3] for j in epi_narrow]),
                             (VP * m)(*[_p(j[4]) for j in epi_narrow]), (VP * m)(*[_p(j[5]) for j in epi_narrow]),
                             (VP * m)(*[_p(j[6]) for j in epi_narrow]),
                             _p(epi_enc[0]) if epi_enc else None, epi_enc[1] if epi_enc else 0,
                             _p(epi_enc[2]) if epi_enc else None, _p(epi_enc[3]) if epi_enc else None, s)
