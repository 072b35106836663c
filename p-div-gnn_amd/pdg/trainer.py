"""Native training step: the hot loop of scripts/gnn_train.py:154-207 on the HIP path.

Per step (one minibatch already resident in HBM):
  forward  model.forward(batch, scale_output=False, scale_input=True)      (gnn_train.py:159-161)
  target   standardize(local_stress, mean/std_local_stress)                (:162-167)
  loss     sum_g NMSE_g / B  [+ lambda * sum_g div_g / B]                  (:168-197)
  backward                                                                 (:205)
  DP       one all-reduce (sum) of the flat fp32 gradient bucket over RCCL (graph-batch data
           parallelism across GPUs; new in this build).  Every rank divides its
           graphs' losses by the GLOBAL minibatch's graph count, so each graph weighs 1/B in the
           summed gradient whatever rank it landed on and however unequal the shards are (the
           reference's 1/B, gnn_train.py:193/196).  The bucket also carries the zero-stress flag
           and the two loss partials, so the reported losses are the global minibatch's with no
           further collective.  dp_mode="replica" (default) normalises each graph-LayerNorm over
           the rank's own shard; dp_mode="sync" reproduces one device running the whole global
           minibatch: every graph-LayerNorm all-reduces its (sum, sumsq) pair in the forward and
           its (S1, S2) pair in the backward (2 x 47 sixteen-byte collectives more per step).
  update   Adam(lr, betas=(0.9, 0.999), eps=1e-8) on the flat parameter buffer (:118, :206),
           stepped as GradScaler.step does it (:204-207): a step whose gradient holds an inf/NaN
           leaves parameters, moments and Adam's step count unchanged.  The step count lives
           on the device (no per-step host sync); state_dict()/load_state_dict() speak
           torch.optim.Adam's format so checkpoints round-trip with the reference's
           save_model_checkpoint / load_optimizer_checkpoint (models.py:44-95).

Parameters and gradients live in one flat buffer each (the model's Parameters
are views into it), so the all-reduce is a single 669 KB collective and Adam a
single kernel.  GradScaler (gnn_train.py:111) is an fp32 power-of-two rescale,
numerically the identity except that it skips the update when a gradient is
non-finite; the same skip is applied here.

capture=True records forward, loss and backward of a batch once in a HIP graph
(torch.cuda.CUDAGraph = hipGraph on ROCm) and replays it on later steps with the
same batch object: ~250 kernel launches per step become one graph launch.  The
all-reduce, the non-finite check and Adam stay eager.  Replays run the same kernels on the same buffers,
so the results are bit-identical to eager steps (tests/test_gpu_trainer_graph.py).
"""
from __future__ import annotations

import torch

from . import hiptimer
from .engine import PARAM_NAMES, PARAM_SHAPES, EPDEngine
from .lib import lib, stream_handle
from .plan import plan_for


class Trainer:
    def __init__(self, model, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 divergence: bool = False, divergence_penalty: float = 1.0, process_group=None,
                 dp_mode: str = "replica", capture: bool = False) -> None:
        if dp_mode not in ("replica", "sync"):
            raise ValueError("dp_mode must be 'replica' or 'sync'")
        dev = next(model.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("Trainer needs the model on a HIP device")
        self.model = model
        self.device = dev
        self.engine: EPDEngine = model._engine_for(dev)
        self.lr, self.betas, self.eps = lr, betas, eps
        self.divergence = divergence
        self.penalty = float(divergence_penalty)
        self.pg = process_group
        self.sync = dp_mode == "sync" and process_group is not None
        sizes = [int(torch.Size(s).numel()) for _, s in PARAM_SHAPES]
        total = sum(sizes)
        self.flat_p = torch.empty(total, dtype=torch.float32, device=dev)
        # the all-reduced bucket: every parameter gradient, then (pdg_loss_reduce's four scalars) one slot
        # holding 1.0 when this rank's batch has a nonzero mean stress (the zero-mean-stress guard of
        # models.py:294-299, below) and this rank's shares of the global minibatch's NMSE, divergence and
        # total loss
        self._bucket = torch.zeros(total + 4, dtype=torch.float32, device=dev)
        self.flat_g = self._bucket[:total]
        self.exp_avg = torch.zeros(total, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(total, dtype=torch.float32, device=dev)
        self.P, self.G = {}, {}
        off = 0
        with torch.no_grad():
            for (name, shape), n in zip(PARAM_SHAPES, sizes):
                p = model.get_parameter(name)
                view = self.flat_p[off:off + n].view(shape)
                view.copy_(p.detach())
                p.data = view                       # the model now shares the flat storage
                self.P[name] = view
                self.G[name] = self.flat_g[off:off + n].view(shape)
                off += n
        self._gt_cache: dict = {}
        # the step's skip flag (non-finite gradient or all-zero mean stress), double-buffered by call
        # parity like Adam's step count (pdg_nonfinite2 clears the other slot: no memset per step)
        self._flags = torch.zeros(2, dtype=torch.int32, device=dev)
        # Adam's step count on the device, double-buffered by call parity (pdg_adam), and the
        # host's bound on it (optimizer calls since the count was last set)
        self._count = torch.zeros(2, dtype=torch.int32, device=dev)
        self._calls = 0
        self._count_bound = 0
        self._table = None
        self._table_key = None
        self._nz_cache: dict = {}
        self._consts: dict = {}
        # captured forward+backward per batch object (dp_mode="sync" reads counts on the host: eager)
        self.capture = capture and not self.sync
        self._graph = None            # (id(batch), torch.cuda.CUDAGraph, static outputs)
        # optional live timing of the data-parallel collectives: name -> list of (start, end) event
        # pairs on the current stream ("allreduce": the gradient bucket; "sync_collective": the
        # global row counts of dp_mode="sync")
        self.timed: dict | None = None

    def _mark(self, name: str):
        """Start an event-timed region on the current stream; returns its end() (a no-op when
        timing is off)."""
        if self.timed is None:
            return lambda: None
        a = hiptimer.Event()
        a.record()

        def end():
            b = hiptimer.Event()
            b.record()
            self.timed.setdefault(name, []).append((a, b))
        return end

    def _gt(self, batch) -> torch.Tensor:
        key = id(batch)
        if key not in self._gt_cache:
            m = self.model
            self._gt_cache = {key: ((batch.local_stress - m.mean_local_stress) / m.std_local_stress).float().contiguous()}
        return self._gt_cache[key]

    def _const(self, v: float) -> torch.Tensor:
        """A (1,) fp32 device tensor holding v, kept for the trainer's lifetime (one fill launch fewer per
        step: the loss normalisers only change with the batch's graph count or the penalty, so the
        cache holds a few entries per distinct minibatch size).  Never evicted: a captured HIP graph
        reads these tensors by address."""
        t = self._consts.get(v)
        if t is None:
            t = self._consts[v] = torch.full((1,), v, dtype=torch.float32, device=self.device)
        return t

    def _nonzero_flag(self, batch) -> torch.Tensor:
        """1.0 when any mean stress of `batch` is nonzero, else 0.0 (a device scalar): the guard of
        models.py:294-299 without its host sync.  Cached per batch object while mean_stress is
        unchanged (bench / training re-use resident batches)."""
        ms = batch.mean_stress
        c = self._nz_cache
        # identity, not id(): the entry holds the batch and its mean_stress tensor, so neither can be
        # freed and its id reused by another tensor while the entry lives
        if not (c and c["batch"] is batch and c["ms"] is ms and c["ver"] == ms._version):
            flag = torch.zeros(1, dtype=torch.int32, device=self.device)
            msf = ms.float().contiguous()
            lib.pdg_any_nonzero(msf.data_ptr(), msf.numel(), flag.data_ptr(), stream_handle(self.device))
            self._nz_cache = {"batch": batch, "ms": ms, "ver": ms._version, "v": flag.float()}
        return self._nz_cache["v"]

    def _global_graphs(self, B: int) -> int:
        """Graphs in the global minibatch when the caller did not say (one small all-reduce and a
        host read; the harness and the bench pass it)."""
        t = torch.tensor([B], dtype=torch.float64, device=self.device)
        torch.distributed.all_reduce(t, group=self.pg)
        return int(t.item())

    def step(self, batch, n_global_graphs: int | None = None, solo: bool = False) -> dict:
        """One optimisation step; returns device scalars (no host sync, except one read of the
        global row counts in dp_mode="sync", or of the global graph count when a process group is
        set and `n_global_graphs` is not given).

        `n_global_graphs`: graphs in the global minibatch this rank's `batch` is a shard of (the
        loss normaliser B of gnn_train.py:193/196); defaults to the batch's own count on one device.
        `batch=None` under a process group: this rank got no graph of the minibatch; it contributes
        zero gradient and zero loss to the collective and takes the same Adam step as every rank.

        `solo=True` (dp_mode="sync", a minibatch that cannot give every rank a shard with edges, e.g. the
        last minibatch of an epoch holding fewer graphs than ranks): ONE rank passes the whole minibatch
        and every other rank passes None, all with solo=True.  No LayerNorm statistic is exchanged; the
        whole-minibatch rank normalises its losses by its own graph count and the others contribute zeros,
        so the summed bucket is exactly one device's step on the minibatch (gnn_local_stress/train.py)."""
        m = self.model
        s = stream_handle(self.device)
        f32 = dict(dtype=torch.float32, device=self.device)
        if solo and self.pg is None:
            raise ValueError("solo=True needs a process group")
        if batch is None:
            if self.pg is None or (self.sync and not solo):
                raise ValueError("batch=None (an empty shard) needs a process group, and in dp_mode='sync' "
                                 "solo=True with the whole minibatch on one rank")
            if n_global_graphs is None and not solo:
                n_global_graphs = self._global_graphs(0)
            self.flat_g.zero_()
            return self._update({"B": 0}, f32, s, None)
        plan = plan_for(batch)
        stats8 = m.stats_tensor(self.device)
        B, N = plan.n_graphs, plan.n_nodes
        Bn = B                                      # loss normaliser (gnn_train.py:193/196)
        if solo:
            if n_global_graphs is not None and int(n_global_graphs) != B:
                raise ValueError(f"solo=True: this rank must hold the whole minibatch ({n_global_graphs} graphs), "
                                 f"it holds {B}")
        elif self.pg is not None and not self.sync:
            Bn = int(n_global_graphs) if n_global_graphs is not None else self._global_graphs(B)
            if Bn < B:
                raise ValueError(f"n_global_graphs={Bn} is smaller than this rank's {B} graphs")
        if self.sync and not solo:
            cnt = torch.tensor([N, plan.n_edges, B], dtype=torch.float64, device=self.device)
            end = self._mark("sync_collective")
            torch.distributed.all_reduce(cnt, group=self.pg)
            end()
            n_g, e_g, Bn = (int(v) for v in cnt.tolist())
            if n_global_graphs is not None and int(n_global_graphs) != Bn:
                raise ValueError(f"n_global_graphs={n_global_graphs} but the ranks hold {Bn} graphs")
            self.engine.set_sync(self.pg, n_g, e_g)
        try:
            if self.capture:
                out = self._replay(batch, plan, stats8, B, N, Bn, f32)
            else:
                out = self._fwd_bwd(batch, plan, stats8, B, N, Bn, f32, s)
            return self._update(out, f32, s, self._nonzero_flag(batch))
        finally:
            self.engine.set_sync(None)

    def _replay(self, batch, plan, stats8, B, N, Bn, f32) -> dict:
        """Forward + loss + backward through a HIP graph captured for this batch object.

        Every device buffer the graph reads must outlive it at a fixed address: the batch and
        its plan are held by the record, the target by the record's copy of the _gt cache entry,
        and the 8 dataset statistics (a fresh tensor per step) are copied into the captured one."""
        # keyed by (batch object, loss normaliser): 1/Bn is a captured constant, so a step on the same batch
        # with another n_global_graphs must record a new graph, not replay the old normaliser
        if self._graph is None or self._graph[0] is not batch or self._graph[6] != Bn:
            self._graph = None
            stats_c = stats8.clone()
            side = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):      # warm the allocator on the capture stream's pool
                self._fwd_bwd(batch, plan, stats_c, B, N, Bn, f32, stream_handle(self.device))
            torch.cuda.current_stream(self.device).wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                static = self._fwd_bwd(batch, plan, stats_c, B, N, Bn, f32, stream_handle(self.device))
            self._graph = (batch, g, static, stats_c, plan, self._gt(batch), Bn)
        _, g, static, stats_c, _, _, _ = self._graph
        stats_c.copy_(stats8)
        g.replay()
        return dict(static)

    def _fwd_bwd(self, batch, plan, stats8, B, N, Bn, f32, s) -> dict:
        m = self.model
        y, ctx = self.engine.forward(self.P, stats8, plan, batch.pos, batch.mean_stress,
                                     batch.nodes_types.reshape(-1).contiguous(), batch.edge_attr.reshape(-1),
                                     m.message_passing_steps, True, False, True)
        gt = self._gt(batch)
        loss_g, den = torch.empty(B, **f32), torch.empty(B, 3, **f32)
        scale = self._const(1.0 / Bn)
        gy = torch.empty(N, 3, **f32)
        # per-graph NMSE and its gradient in one launch (pdg_nmse_fwd_bwd, bitwise pdg_nmse_fwd + pdg_nmse_bwd)
        lib.pdg_nmse_fwd_bwd(B, plan.ptr.data_ptr(), gt.data_ptr(), y.data_ptr(), loss_g.data_ptr(), den.data_ptr(),
                             scale.data_ptr(), 0, gy.data_ptr(), s)
        # per-graph losses; _update reduces them (pdg_loss_reduce: sum / B_global [x penalty])
        out = {"B": B, "Bn": Bn, "loss_g": loss_g}
        if self.divergence:
            types = batch.surfaces_nodes_for_div if batch.surfaces_nodes_for_div is not None else batch.nodes_types
            types = types.reshape(-1).to(torch.int64).contiguous()
            div = torch.empty(N, 2, **f32)
            loss_d = torch.empty(B, **f32)
            lib.pdg_div_fwd(B, plan.ptr.data_ptr(), plan.a_rowptr.data_ptr(), plan.a_col.data_ptr(),
                            plan.a_val.data_ptr(), types.data_ptr(), y.data_ptr(), 0, div.data_ptr(),
                            loss_d.data_ptr(), s)
            sd = self._const(self.penalty / Bn)
            lib.pdg_div_bwd(B, plan.ptr.data_ptr(), N, plan.at_rowptr.data_ptr(), plan.at_row.data_ptr(),
                            plan.at_comp.data_ptr(), plan.at_val.data_ptr(), div.data_ptr(), sd.data_ptr(), 0, 1,
                            gy.data_ptr(), s)
            out["loss_d"] = loss_d
        self.flat_g.zero_()
        self.engine.backward(self.P, ctx, gy, self.G)
        del ctx
        return out

    def _update(self, fb, f32, s, nz) -> dict:
        """Loss scalars, the data-parallel all-reduce, the skip test and Adam.  `fb`: _fwd_bwd's per-graph
        losses (or {"B": 0} for an empty shard); `nz`: this rank's nonzero-mean-stress flag (a device
        float, None for an empty shard)."""
        # zero-mean-stress guard (models.py:294-299): the reference's forward returns zeros without a
        # graph there, so its backward() raises and no update happens.  Here the step is skipped like a
        # non-finite one (parameters, moments and Adam's count unchanged; out["skipped"] = 1), decided
        # on the device.  Under data parallelism the flag rides in the gradient bucket, so the step is
        # skipped on every rank exactly when the GLOBAL minibatch is all zero, as one device would.
        # pdg_loss_reduce writes [flag, nmse / B_global, penalty * div / B_global, total] (one launch for
        # what were torch's sum / scale / add kernels): into the bucket's tail under data parallelism (every
        # rank's shares are already / B_global, so the summed bucket holds the global minibatch's losses)
        tail = self._bucket[-4:] if self.pg is not None else torch.empty(4, **f32)
        if fb["B"] > 0:
            ld = fb.get("loss_d")
            lib.pdg_loss_reduce(fb["B"], fb["loss_g"].data_ptr(), ld.data_ptr() if ld is not None else None,
                                1.0 / fb["Bn"], self.penalty / fb["Bn"], nz.data_ptr(), tail.data_ptr(), s)
        else:
            tail.zero_()
        if self.pg is not None:
            end = self._mark("allreduce")
            torch.distributed.all_reduce(self._bucket, group=self.pg)
            end()
        parity = self._calls & 1
        self._ensure_table(self._count_bound + 1)
        # skip = non-finite gradient OR the (global) minibatch's stress flag == 0, one launch
        lib.pdg_nonfinite2(self.flat_g.data_ptr(), self.flat_g.numel(), tail.data_ptr(), self._flags.data_ptr(),
                           parity, s)
        skip = self._flags[parity:parity + 1]
        lib.pdg_adam(self.flat_p.numel(), self.flat_p.data_ptr(), self.flat_g.data_ptr(), self.exp_avg.data_ptr(),
                     self.exp_avg_sq.data_ptr(), self._table.data_ptr(), self._table.shape[0],
                     float(1.0 - self.betas[0]), self.betas[1], float(1.0 - self.betas[1]), self.eps,
                     skip.data_ptr(), self._count.data_ptr(), parity, s)
        self._calls += 1
        self._count_bound += 1
        vals = tail[1:].clone() if self.pg is not None else tail[1:]   # (the bucket is rewritten next step)
        out = {"nmse": vals[0], "total": vals[2], "skipped": skip}      # skipped: valid until the next step
        if self.divergence:
            out["div"] = vals[1]
        return out


    # ------------------------------------------------------------------ optimizer state
    def _ensure_table(self, need: int) -> None:
        """Bias-correction table of torch.optim.Adam (_single_tensor_adam, capturable=False): entry
        t-1 = (lr / (1 - beta1**t), (1 - beta2**t) ** 0.5) in Python double, stored as float32 (the
        precision the elementwise ops apply them in).  Grown by doubling, never per step; rebuilt when
        lr or betas are reassigned (e.g. a learning-rate schedule writing trainer.lr)."""
        key = (float(self.lr), tuple(float(b) for b in self.betas))
        if self._table is not None and self._table.shape[0] >= need and self._table_key == key:
            return
        self._table_key = key
        n = max(64, 2 * need)
        b1, b2 = self.betas
        rows = []
        for t in range(1, n + 1):
            step = float(t)
            rows.append((self.lr / (1 - b1 ** step), (1 - b2 ** step) ** 0.5))
        self._table = torch.tensor(rows, dtype=torch.float32).to(self.device)

    @property
    def step_count(self) -> int:
        """Adam steps taken (skipped steps excluded); reads the device counter (one sync)."""
        return int(self._count[self._calls & 1])

    def _param_views(self) -> list:
        """(name, offset, numel, shape) of every parameter in model.parameters() order (the index
        order of torch.optim.Adam's state_dict)."""
        offs, off = {}, 0
        for name, shape in PARAM_SHAPES:
            n = int(torch.Size(shape).numel())
            offs[name] = (off, n, shape)
            off += n
        return [(name, *offs[name]) for name, _ in self.model.named_parameters()]

    def state_dict(self) -> dict:
        """torch.optim.Adam(model.parameters()).state_dict() equivalent (what the reference saves
        as optimizer_state_dict, models.py:50-62)."""
        sd = torch.optim.Adam(self.model.parameters(), lr=self.lr, betas=self.betas, eps=self.eps).state_dict()
        steps = self.step_count
        if steps > 0:
            for i, (_, o, n, shape) in enumerate(self._param_views()):
                sd["state"][i] = {"step": torch.tensor(float(steps)),
                                  "exp_avg": self.exp_avg[o:o + n].view(shape).clone(),
                                  "exp_avg_sq": self.exp_avg_sq[o:o + n].view(shape).clone()}
        return sd

    def load_state_dict(self, sd: dict) -> None:
        """Resume from a torch.optim.Adam state_dict (load_optimizer_checkpoint, models.py:89-95)."""
        groups = sd["param_groups"]
        if len(groups) != 1:
            raise ValueError("expected one Adam param group")
        g = groups[0]
        if g.get("amsgrad") or g.get("weight_decay", 0) or g.get("maximize"):
            raise ValueError("only plain Adam (amsgrad=False, weight_decay=0, maximize=False) is supported")
        self.lr, self.betas, self.eps = float(g["lr"]), tuple(float(b) for b in g["betas"]), float(g["eps"])
        self._table = None
        views = self._param_views()
        if len(g["params"]) != len(views):
            raise ValueError("parameter count mismatch")
        steps = set()
        with torch.no_grad():
            self.exp_avg.zero_()
            self.exp_avg_sq.zero_()
            for pid, (_, o, n, _) in zip(g["params"], views):
                st = sd["state"].get(pid)
                if not st:
                    steps.add(0)
                    continue
                self.exp_avg[o:o + n].copy_(st["exp_avg"].reshape(-1))
                self.exp_avg_sq[o:o + n].copy_(st["exp_avg_sq"].reshape(-1))
                steps.add(int(float(st["step"])))
        if len(steps) != 1:
            raise ValueError(f"parameters at different Adam steps: {sorted(steps)}")
        c = steps.pop()
        self._count.fill_(c)
        self._count_bound = c


def param_names() -> list:
    return list(PARAM_NAMES)
