#!/usr/bin/env python3
"""P-DivGNN training throughput on MI355X: mesh-nodes/sec (fwd+bwd), 1..8 GPUs.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One process per GPU.  Launched without a torch.distributed launcher (no WORLD_SIZE in the
environment), ``--gpus N`` > 1 spawns the N ranks itself (torch.multiprocessing "spawn",
before anything touches the GPU); under torchrun the launcher's ranks are used and must
number ``--gpus``.  Ranks talk over RCCL (torch.distributed backend "nccl").

A step is one full training step of the reference's hot loop (scripts/gnn_train.py:154-207)
on one minibatch resident in HBM: forward of EncodeProcessDecode (10 message-passing steps,
latent 128), per-graph NMSE (+ lambda * divergence), backward, RCCL all-reduce of the flat
gradient bucket (N > 1), the non-finite check and the Adam update — all on the HIP kernels of
libpdivgnn_hip.so.

Main line (the driver's metric): BASELINE.json configs[1] = 8 synthetic periodic triangulated
71x71 meshes (5,041 nodes, 29,968 edges each) PER GPU (weak scaling, graph-level DP).
value = nodes processed by all ranks / max-over-ranks wall time of the K timed steps.

Sub-results in the same JSON line ("sub_results"; skipped with --no-extras), each timed the
same way (barrier + synchronize on both sides, max over ranks):
  config3  P-DivGNN with the divergence loss, 32 x 5,041-node meshes per GPU (weak)
  config4  hyperelastic-style hole plates, FIXED global batch of 64 graphs sharded over the
           ranks by pdg.dist.shard_graphs (64/32/16/8 per GPU at N = 1/2/4/8: strong scaling)
  config5  inference, one 100,489-node mesh per GPU, 15 MP layers (N independent replicas)

Also reported: the roofline of the dominant kernel (HIP events around its launches inside the
timed region) and the reference algorithm's CPU path (the op-for-op oracle restatement) timed
on this host's cores (rank 0, N = 1 only).  --plumbing runs the launch / rendezvous / timing /
reporting flow with a gradient-bucket all-reduce as the only work (CPU tests with gloo); its
line says so and carries no throughput claim.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT), str(ROOT / "p-div-gnn_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# rocprofv3 --pmc of this bench (tools/final_pass.sh writes profiles/rNN_pmc_traffic.json with the tree it
# measured under "_meta"); the bench takes traffic only from a file of ITS OWN tree (pmc_file())
PMC_GLOB = "profiles/r*_pmc_traffic.json"      # config 2 (the main line); config c: r*_pmc_traffic_c{c}.json


def _cfg_glob(glob: str, config: int) -> str:
    """The profiles/ glob of `config`'s counter files: the main line's (config 2) as named, the
    sub-results' with a _c{config} suffix (tools/final_pass.sh TAG measure_cfg C)."""
    return glob if config == 2 else glob.replace(".json", f"_c{config}.json")
TREE_GLOBS = ("p-div-gnn_amd/pdg/libpdivgnn_hip.so", "p-div-gnn_amd/csrc/*.hip", "p-div-gnn_amd/csrc/*.hpp", "include/*.h", "p-div-gnn_amd/pdg/*.py",
              "p-div-gnn_amd/gnn_local_stress/*.py", "bench.py")
# the edge forward's training kernel, its inference kernel (calls of >= 32k edges without a backward) and the
# LDS-weight reference
PMC_NAMES = {"edge_fwd": ("void edge_fwd_coop_kernel<true, true", "void edge_fwd_infer_kernel<true, true",
                          "void edge_fwd_kernel<true, true>"),
             "edge_bwd": "void edge_bwd_kernel<true>",
             "segment_sum": ("segment_sum_kernel",), "node_net": ("node_net_x6_kernel", "node_net_pair_kernel", "node_net_kernel"),
             # the edge-update steps' instantiation (gz1e formed as gC - gz1m); the last step's is <false>
             "pq_scatter_bwd": ("void pq_scatter_bwd_kernel<true>", "pq_scatter_bwd_kernel"),
             "wgrad_W2": "wgrad_x6_kernel",
             # the edge-update instantiations
             "edge_bwd_w2": "void edge_bwd_w2_kernel<true>",
             "edge_gout": ("void edge_gout_wc_kernel<true, true>", "void edge_gout_wc_kernel<true>"),
             "node_bwd": "node_bwd_coop_kernel", "node_pq": "void node_pq_x6_kernel<true>",
             "gemm_sum2": ("void gemm_sum2_coop_kernel<true, true>", "void gemm_sum2_coop_kernel<true>"), "wgrad_pairs": "void wgrad_x6_pair2_kernel"}
PEAK_FP32_MFMA = 157.3e12   # MI355X dense fp32 MFMA, /opt/skills/guides/MI355X_MICROARCH.md
PEAK_BF16_MFMA = 16 * PEAK_FP32_MFMA   # dense bf16 MFMA (2.5 PF; the fp32 rate is 1/16 of it, same guide)
X6 = 6                      # bf16x6: six bf16 products per fp32-accurate product
PEAK_HBM = 8.0e12           # MI355X HBM3E spec bandwidth (same guide; 6.3 TB/s measured copy)
L = 128
N_PARAMS = 167_299

CONFIGS = {
    2: dict(workload="P-GNN linear-elastic, 8 x 5,041-node periodic meshes per GPU, fwd+bwd (BASELINE configs[1])",
            graphs=8, n=71, hole=(0.0, 0.0), divergence=False, steps=10),
    3: dict(workload="P-DivGNN with divergence loss (lambda=10), 32 x 5,041-node periodic meshes per GPU "
                     "(BASELINE configs[2])",
            graphs=32, n=71, hole=(0.0, 0.0), divergence=True, steps=10),
    4: dict(workload="P-DivGNN hyperelastic-style hole plates (strain range +-0.15), fixed global batch of 64 "
                     "~4.8k-node periodic meshes sharded over the ranks (BASELINE configs[3])",
            graphs=64, n=71, hole=(0.08, 0.12), divergence=True, steps=10, strain=(-0.15, 0.15), global_batch=True),
    5: dict(workload="inference, one synthetic 100,489-node periodic mesh per GPU, 15 MP layers (BASELINE configs[4])",
            graphs=1, n=317, hole=(0.0, 0.0), divergence=False, steps=15, inference=True),
}


# ---------------------------------------------------------------------------------- workload
def shard_indices(cfg, rank: int, world: int) -> list[int]:
    """Graph indices this rank builds: the whole per-GPU batch (weak scaling), or its share of
    the fixed global batch (strong scaling), balanced by node count (pdg.dist.shard_graphs)."""
    from pdg import meshgen
    from pdg.dist import shard_graphs
    if not cfg.get("global_batch"):
        return list(range(cfg["graphs"]))
    specs = meshgen.dataset_specs(cfg["graphs"], cfg["hole"], seed=69)
    counts = [meshgen.hole_plate_node_count(cfg["n"], r) for r, _ in specs]
    return shard_graphs(counts, world)[rank]


def build_batch(cfg, seed, device, indices=None):
    from pdg import graph, meshgen
    samples = meshgen.make_dataset(cfg["graphs"], n=cfg["n"], hole_radius=cfg["hole"], seed=seed,
                                   strain_range=cfg.get("strain"), indices=indices)
    datas = [graph.sample_to_data(s) for s in samples]
    return graph.Batch.from_data_list(datas).to(device), samples


def dataset_stats(b):
    return {"mean_pos": b.pos.mean(), "std_pos": b.pos.std(), "mean_mean_stress": b.mean_stress.mean(),
            "std_mean_stress": b.mean_stress.std(), "mean_local_stress": b.local_stress.mean(),
            "std_local_stress": b.local_stress.std(), "mean_edge_weight": b.edge_attr.mean(),
            "std_edge_weight": b.edge_attr.std()}


def tree_hash() -> str:
    """sha256 (16 hex) over the sources of the timed path (kernels, C ABI, engine, bench): the same
    value in the bench line and in the profiles/ files measured from the same tree, on any box (the
    GPU box's snapshot has no .git)."""
    import hashlib
    h = hashlib.sha256()
    for pat in TREE_GLOBS:
        for f in sorted(ROOT.glob(pat)):
            h.update(f.relative_to(ROOT).as_posix().encode())
            h.update(f.read_bytes())
    return h.hexdigest()[:16]


# ---------------------------------------------------------------------------------- CPU baseline
def _cpu_model_name() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads() -> tuple[int, dict]:
    """Threads for the CPU baseline: the CPUs this process may really use.  The affinity mask of a
    GPU box lists every core of the host (256), but the container's CPU quota (cgroup cpu.max) and
    the OMP_NUM_THREADS the box exports (16) grant far fewer; torch at 256 threads on 16 CPUs would
    time oversubscription.  Returns (threads, the three figures and which one bounds)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    omp = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    cands = {"sched_getaffinity": aff, "cgroup_cpu_max": quota, "OMP_NUM_THREADS": omp}
    n = min(v for v in cands.values() if v)
    bound = [k for k, v in cands.items() if v == n][0]
    return n, {**cands, "bound_by": bound}


def _oracle_step_fn(cfg, samples):
    """One step of the reference algorithm (oracle/epd_oracle.py, the op-for-op restatement of
    models.py + gnn_train.py losses, validated against the reference's own outputs in
    tests/golden) on a batch of `samples`, fp32, torch CPU."""
    from oracle import epd_oracle as O
    from pdg import graph
    datas = [graph.sample_to_data(s) for s in samples]
    b = graph.Batch.from_data_list(datas)
    st = {k: v.float() for k, v in dataset_stats(b).items()}
    P = {k: v.requires_grad_(True) for k, v in O.init_params().items()}
    args = (b.pos, b.mean_stress, b.nodes_types, b.edge_index, b.edge_attr)
    gt = (b.local_stress - st["mean_local_stress"]) / st["std_local_stress"]
    ops = [d.op_div_matrix for d in datas]

    def step():
        if cfg.get("inference"):
            with torch.no_grad():
                O.epd_forward(P, st, *args, cfg["steps"], scale_output=True)
            return
        pred = O.epd_forward(P, st, *args, cfg["steps"], scale_output=False)
        total, _, _ = O.batch_loss(pred, gt, b.ptr, ops, b.nodes_types, cfg["divergence"], 10.0)
        for p in P.values():
            p.grad = None
        total.backward()
    return step, b.num_nodes


def _median_rate(step, nodes, reps):
    step()                                       # warm-up
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    return nodes / statistics.median(ts), ts


def cpu_baseline(cfg, samples, full_graphs: int, reps: int = 5, one_thread: bool = True):
    """The reference algorithm on this host's CPU cores: median of
    `reps` steps after one warm-up, at the threads this process may use (cpu_threads) and, with
    `one_thread`, at 1 thread on one graph.  `samples` is a bounded sample of the config's batch
    (10-30 s of CPU work; the whole config-2 batch takes ~19 s per step on 16 host threads): every
    op of the path is linear in the number of graphs (per-graph losses, row-wise MLPs, segment
    sums, graph-global LayerNorm statistics), so nodes/s on the sample stands for the batch of
    `full_graphs` graphs; the sample is named in the record."""
    threads, tinfo = cpu_threads()
    prev = torch.get_num_threads()
    what = "inference forwards" if cfg.get("inference") else \
        f"training steps (fwd+NMSE{'+div' if cfg['divergence'] else ''}+bwd)"
    rec = {"unit": "nodes/s", "cores": threads, "kind": "port", "threads_info": tinfo}
    try:
        torch.set_num_threads(threads)
        step, nodes = _oracle_step_fn(cfg, samples)
        rate, ts = _median_rate(step, nodes, reps)
        rec.update(value=round(rate, 1), step_s=[round(t, 3) for t in ts],
                   sample=f"median of {reps} {what} (after 1 warm-up) on {len(samples)} of the config's "
                          f"{full_graphs} graph(s) ({nodes} nodes), {cfg['steps']} MP steps, fp32, torch CPU "
                          f"at {threads} threads, oracle/epd_oracle.py"
                          + ("" if len(samples) == full_graphs else
                             "; nodes/s extrapolates linearly to the full batch (every op is linear in the "
                             "number of graphs)"),
                   extrapolated=len(samples) != full_graphs)
        if one_thread:
            torch.set_num_threads(1)
            step1, nodes1 = _oracle_step_fn(cfg, samples[:1])
            rate1, _ = _median_rate(step1, nodes1, reps)
            rec.update(value_1thread=round(rate1, 1),
                       sample_1thread=f"median of {reps} (after 1 warm-up), 1 graph, {nodes1} nodes, 1 thread")
    finally:
        torch.set_num_threads(prev)
    rec.update(host_cpu_count=os.cpu_count(), cpu_model=_cpu_model_name())
    return rec


# ---------------------------------------------------------------------------------- roofline
def kernel_work(infer: bool, N: int, E: int, S: int, nslab_bytes: int, fused: bool, e_sum: bool = True) -> dict:
    """Algorithmic work per launch (DESIGN.md "Kernels"): executed MFMA flops with the peak of their
    instruction type, and the bytes the kernel must read/write (inputs once, outputs once, int32
    indices).  An fp32-accurate 128x128 product per row costs 2*L*L fp32 flops on the fp32 MFMA,
    or 6x that in bf16 (bf16x6)."""
    g = 2 * L * L
    out = {
        # W_c product + 2 W2 products (all bf16x6 since round 5) per edge; reads a2e_prev, e_prev, 4
        # gathered P/Q rows, src, dst; writes e_t, a2m, a2e and, when training, a1m, a1e
        "edge_fwd": ([(E * 3 * g * X6, PEAK_BF16_MFMA)],
                     E * ((9 if infer else 11) * 4 * L + 8)),
        # fused (pdg_edge_bwd_w2): 2 W2^T products + 2 weight-gradient products per edge (bf16x6);
        # reads gaggr[dst], ge_next, a2m, a1m, a2e, a1e, dst; writes gz1m, gC (+ gz1e unless e_sum: the
        # P/Q gather backward forms it from gC - gz1m); one slab read+write per block.  unfused
        # (pdg_edge_bwd): W2^T x2 (bf16x6) + Wc^T (fp32); writes gz2m, gz1m, gz2e, gz1e, gC, ge_out
        "edge_bwd": (([(E * 4 * g * X6, PEAK_BF16_MFMA)], E * ((8 if e_sum else 9) * 4 * L + 4) + 2 * nslab_bytes)
                     if fused
                     else ([(E * 2 * g * X6, PEAK_BF16_MFMA), (E * g, PEAK_FP32_MFMA)], E * (12 * 4 * L + 4))),
        # fused Wc path (pdg_edge_gout_wc): Wc^T product + weight-gradient product (bf16x6); reads gC,
        # e, ge_next and the LayerNorm input of e (column sums), writes ge_out; one slab read+write
        "edge_gout": ([(E * 2 * g * X6, PEAK_BF16_MFMA)], E * 5 * 4 * L + 2 * nslab_bytes),
        # all steps' W2 segments: 2E rows per step of (G, X) 512-byte rows, one 64 KB slab per block
        "wgrad_W2": ([(S * 2 * E * g * X6, PEAK_BF16_MFMA)], S * 2 * E * 2 * 4 * L + 512 * (L * L + L) * 4),
        # dst-segment sum of LN(a2m): reads a2m (E rows) and rowptr, writes aggr (+ x-hat sums)
        "segment_sum": ([], 4 * L * E + 4 * (N + 1) + (1 if infer else 2) * 4 * L * N),
        # node_net, 2 fp32-accurate GEMMs (K = 256, 128) per node as bf16x6 products (node_net_x6_kernel;
        # the fp32-MFMA kernels are A/B build variants): reads aggr, x; writes a2n (+ a1n)
        "node_net": ([(N * 2 * L * (2 * L + L) * X6, PEAK_BF16_MFMA)],
                     2 * 4 * L * N + (1 if infer else 2) * 4 * L * N),
        "pq_scatter_bwd": ([], 2 * 4 * L * E + 4 * E + 8 * (N + 1) + 2 * 4 * L * N),
    }
    return out


def compulsory_bytes(work: dict, N: int, E: int) -> dict:
    """Per-launch bytes with every GATHERED row priced once per node instead of once per edge (the
    compulsory traffic when each node's row is fetched from HBM once and every later use is a cache
    hit): the edge forward's 4 P / Q gathers (4 N rows instead of 4 E; 2 with no edge update) and the
    fused edge backward's gaggr[dst] (N instead of E).  kernel_work's figure prices a gather per edge
    (SURVEY §8d); `frac_compulsory` in the roofline is this figure's rate, the lower of the two."""
    row = 4 * L
    out = {k: nb for k, (_, nb) in work.items()}
    if "edge_fwd" in out:   # the timed "edge_fwd" launches are the steps with an edge update: 4 gathers
        out["edge_fwd"] = work["edge_fwd"][1] - 4 * E * row + 4 * N * row
    if "edge_bwd" in out:
        out["edge_bwd"] = work["edge_bwd"][1] - E * row + N * row
    return out


def pmc_file(tree: str | None = None, config: int = 2):
    """(path, None) of the newest profiles/rNN_pmc_traffic[_cC].json of `config` measured on this tree
    (its "_meta" "tree" equals tree_hash()), or (None, reason).  PMC bytes of another tree would price a
    kernel's launches with the bytes of different code, so they are never used."""
    tree = tree or tree_hash()
    files = sorted(ROOT.glob(_cfg_glob(PMC_GLOB, config)), reverse=True)
    if not files:
        return None, f"no {_cfg_glob(PMC_GLOB, config)}"
    seen = []
    for f in files:
        try:
            t = json.loads(f.read_text()).get("_meta", {}).get("tree")
        except (OSError, ValueError):
            continue
        if t == tree:
            return f, None
        seen.append(f"{f.name}: {t}")
    return None, f"no PMC file of tree {tree} ({'; '.join(seen)})"


def pmc_tree() -> str | None:
    """Tree hash of the PMC file the bench uses (None when no file matches this tree)."""
    f, _ = pmc_file()
    return json.loads(f.read_text())["_meta"]["tree"] if f else None


def load_pmc(fused: bool, path=None) -> dict:
    """Per-launch PMC bytes by kernel from `path` (a pmc_file() result; {} when None)."""
    pmc = {}
    if path is not None and Path(path).exists():
        data = json.loads(Path(path).read_text())
        data.pop("_meta", None)
        for k, prefix in PMC_NAMES.items():
            if fused and k == "edge_bwd":
                prefix = PMC_NAMES["edge_bwd_w2"]
            hit = [v for name, v in data.items() if name.startswith(prefix if isinstance(prefix, tuple) else (prefix,))]
            if hit:
                pmc[k] = round(hit[0]["total"])
    return pmc


SQ_GLOB = "profiles/r*_sq.json"   # tools/sq_pass.sh (SQ_VALU_MFMA_BUSY_CYCLES per dispatch, tools/sq_summary.py)


def sq_file(tree: str | None = None, config: int = 2):
    """(path, None) of the newest profiles/rNN_sq[_cC].json of `config` measured on this tree, or
    (None, reason)."""
    tree = tree or tree_hash()
    files = sorted(ROOT.glob(_cfg_glob(SQ_GLOB, config)), reverse=True)
    if not files:
        return None, f"no {_cfg_glob(SQ_GLOB, config)}"
    for f in files:
        try:
            if json.loads(f.read_text()).get("_meta", {}).get("tree") == tree:
                return f, None
        except (OSError, ValueError):
            continue
    return None, f"no SQ counter file of tree {tree}"


def load_sq(path) -> dict:
    """Counter MFMA busy fraction (at the nominal 2.4 GHz) per bench kernel key, from an sq_file()."""
    out = {}
    if path is None:
        return out
    rows = json.loads(Path(path).read_text()).get("kernels", [])
    for k, prefix in PMC_NAMES.items():
        pre = prefix if isinstance(prefix, tuple) else (prefix,)
        hit = [r for r in rows if r["kernel"].startswith(pre) and r.get("mfma_busy_at_2.4GHz") is not None]
        if hit:
            out[k] = round(hit[0]["mfma_busy_at_2.4GHz"], 4)
    return out


def reads_only_bytes(k: str, E: int, calls: int = 2) -> int | None:
    """SURVEY §8(d)'s literal figure for a kernel that fuses the gather into the GEMM: its reads only,
    12L bytes per edge per edge_net evaluation (x_i, x_j, e rows) + the int32 src / dst once; the timed
    edge forward launches evaluate edge_net twice (message + edge update).  None for other kernels."""
    if k != "edge_fwd":
        return None
    return calls * 12 * L * E + 8 * E


def roofline(k, work, kt, ktot, step_s, pmc, nlaunch=None, pmc_source=None, comp=None, reads_only=None):
    """Roofline of kernel `k`.  The headline `frac` is the COMPULSORY-byte fraction:
    every streamed row once and every gathered row once per node (compulsory_bytes) over the event-timed
    launch average, against 8 TB/s; `frac_pmc` is the same rate with the rocprofv3 PMC bytes of the same
    tree.  `frac_gather_priced` prices every gathered row per edge (kernel_work: gathers served from L2 /
    the Infinity Cache counted at HBM cost, so it reads high) and `frac_reads_only` is §8(d)'s reads-only
    formula (reads_only_bytes); both are reported beside it, neither is the headline."""
    nlaunch = nlaunch or {}
    terms, nbytes = work[k]
    cbytes = (comp or {}).get(k, nbytes)
    t = kt[k]
    flops = sum(f for f, _ in terms)
    t_peak = sum(f / pk for f, pk in terms)     # matrix-core time at peak rate
    f_mfma = t_peak / t
    f_hbm = cbytes / t / PEAK_HBM
    bound = "mfma" if f_mfma >= f_hbm else "hbm"
    if bound == "mfma":   # executed flops / time against the flop-weighted peak of the mix
        ach, peak, unit = flops / t / 1e12, flops / t_peak / 1e12, "TFLOP/s"
    else:
        ach, peak, unit = cbytes / t / 1e9, PEAK_HBM / 1e9, "GB/s"
    traffic = pmc.get(k)
    return {"kernel": k, "bound": bound, "achieved": round(ach, 2), "peak": round(peak, 1), "unit": unit,
            "frac": round(f_hbm if bound == "hbm" else ach / peak, 4), "traffic": traffic,
            # real DRAM rate: the PMC bytes of a launch (profiles/, same tree when traffic_tree matches)
            # over this run's event-timed launch average, against 8 TB/s
            "frac_pmc": round(traffic / t / PEAK_HBM, 4) if traffic else None,
            "pmc_over_compulsory": round(traffic / cbytes, 4) if traffic else None,
            "bytes_per_launch": cbytes, "bytes_compulsory_per_launch": cbytes,
            "frac_compulsory": round(f_hbm, 4),
            "bytes_gather_priced_per_launch": nbytes, "frac_gather_priced": round(nbytes / t / PEAK_HBM, 4),
            "bytes_reads_only_per_launch": reads_only,
            "frac_reads_only": round(reads_only / t / PEAK_HBM, 4) if reads_only else None,
            "traffic_source": (f"profiles/{Path(pmc_source).name}: 2*FETCH_SIZE+WRITE_SIZE per dispatch"
                               if k in pmc and pmc_source else None),
            "flops_per_launch": flops, "frac_mfma": round(f_mfma, 4),
            "frac_hbm": round(f_hbm, 4), "avg_launch_ms": round(t * 1e3, 4), "launches_timed": nlaunch.get(k),
            "share_of_step": round(ktot[k] / step_s, 4)}


# ---------------------------------------------------------------------------------- timing
TIMED_KERNELS = ["edge_fwd", "edge_bwd", "edge_gout", "wgrad_W2", "segment_sum", "node_net", "node_bwd", "edge_enc_fwd", "edge_enc_bwd",
                 "node_pq", "gemm_sum2", "pq_scatter_bwd", "sync_collective"]


def _allgather_ints(vals, world, device):
    t = torch.tensor(vals, dtype=torch.int64, device=device)
    if world == 1:
        return [vals]
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def _allgather_floats(vals, world, device):
    if world == 1:
        return [list(vals)]
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.tolist() for o in out]


def _max_over_ranks(x: float, world: int, device) -> float:
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t)


def per_rank_fields(world: int, device, pg, counts, step_ms: float, allreduce_ms: float, sync_ms: float) -> dict:
    """Every rank's share and the split of its step (gathered to all ranks): nodes / edges / graphs,
    the world size its process group reports, its own ms per step, the RCCL gradient all-reduce and
    the sync-LN collectives per step (event-timed on the compute stream, so they include waiting for
    the slowest rank), the rest as compute, and the node balance max/mean over ranks."""
    ints = _allgather_ints(list(counts) + [dist.get_world_size() if pg is not None else 1], world, device)
    fl = _allgather_floats([step_ms, allreduce_ms, sync_ms], world, device)
    nodes = [r[0] for r in ints]
    return {"nodes": nodes, "edges": [r[1] for r in ints], "graphs": [r[2] for r in ints],
            "world_size_rccl": [r[3] for r in ints],
            "step_ms": [round(r[0], 3) for r in fl], "allreduce_ms": [round(r[1], 4) for r in fl],
            "sync_ln_collectives_ms": [round(r[2], 4) for r in fl],
            "compute_ms": [round(r[0] - r[1] - r[2], 3) for r in fl],
            "node_balance": round(max(nodes) / (sum(nodes) / world), 4) if sum(nodes) else None}


def time_config(cid: int, args, rank: int, world: int, pg, device) -> tuple[dict, list]:
    """Build this rank's batch of config `cid`, run W warm-up and K timed steps, return the
    record (value over all ranks, ms/step, rooflines) and this rank's samples."""
    from gnn_local_stress.models import EncodeProcessDecode
    from pdg.plan import plan_for
    from pdg.trainer import Trainer

    cfg = CONFIGS[cid]
    idx = shard_indices(cfg, rank, world)
    seed = 69 if cfg.get("global_batch") else 69 + rank
    batch, samples = build_batch(cfg, seed=seed, device=device, indices=idx)
    stats = dataset_stats(batch)
    if pg is not None:  # dataset statistics are global constants of the training set
        v = torch.stack([stats[k].float() for k in stats])
        dist.all_reduce(v)
        stats = {k: v[i] / world for i, k in enumerate(stats)}
    torch.manual_seed(69)
    model = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=cfg["steps"], latent_size=L,
                                input_nodes_features_size=6, output_nodes_features_size=3, **stats).to(device)
    trainer = Trainer(model, lr=1e-3, divergence=cfg["divergence"], divergence_penalty=10.0, process_group=pg,
                      dp_mode=args.dp_mode, capture=args.graph)
    plan = plan_for(batch)
    N, E = plan.n_nodes, plan.n_edges
    infer = cfg.get("inference", False)
    if infer:
        def run_step():
            with torch.no_grad():
                return {"total": model(batch, scale_output=True).local_stress.abs().mean()}
    else:
        # the global minibatch's graph count (every rank's losses are / B_global, pdg/trainer.py)
        n_global = cfg["graphs"] if cfg.get("global_batch") else cfg["graphs"] * world

        def run_step():
            return trainer.step(batch, n_global_graphs=n_global if pg is not None else None)
    for _ in range(args.warmup):
        run_step()
    torch.cuda.synchronize()
    eng = trainer.engine
    # HIP events bracket the timed kernels' launches in the last `ev_steps` steps of the timed
    # region (each event pair costs a few us of queue time; sampling keeps the region clean)
    ev_steps = min(args.steps, 3)
    graph_steps = 0 if (infer or not trainer.capture) else args.steps - ev_steps
    if pg is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i == args.steps - ev_steps:
            # the event-timed steps launch eagerly (events cannot bracket launches inside a graph
            # replay); the other timed steps replay the graph captured during warmup
            trainer.capture = False
            eng.timed = {k: [] for k in TIMED_KERNELS}
            trainer.timed = {}
        out = run_step()
    torch.cuda.synchronize()
    el_local = time.perf_counter() - t0     # this rank's time (the max below adds the barrier skew)
    if pg is not None:
        dist.barrier()
    el = _max_over_ranks(time.perf_counter() - t0, world, device)
    ev = {k: v for k, v in eng.timed.items() if v}
    coll = {k: sum(a.elapsed_time(b) for a, b in v) / ev_steps for k, v in (trainer.timed or {}).items()}
    eng.timed = None
    trainer.timed = None
    # per-rank split of a step: collectives (event-timed on the compute stream: the RCCL gradient
    # all-reduce including its wait for the slowest rank, and the sync-LN collectives) and the rest
    sync_ms = coll.get("sync_collective", 0.0) + (sum(a.elapsed_time(b) for a, b in ev["sync_collective"]) / ev_steps
                                                   if "sync_collective" in ev else 0.0)
    ar_ms = coll.get("allreduce", 0.0)
    step_ms_local = el_local / args.steps * 1e3
    loss = float(out["total"])
    per_rank_rec = per_rank_fields(world, device, pg, [N, E, len(idx)], step_ms_local, ar_ms, sync_ms)
    total_nodes = sum(per_rank_rec["nodes"])

    ev.pop("sync_collective", None)
    kt = {k: sum(a.elapsed_time(b) for a, b in v) / len(v) * 1e-3 for k, v in ev.items()}
    nlaunch = {k: len(v) for k, v in ev.items()}
    ktot = {k: sum(a.elapsed_time(b) for a, b in v) * 1e-3 for k, v in ev.items()}
    fused = eng.fused_edge_wgrad
    nslab_bytes = getattr(eng, "_nslabs_e", 256) * (L * L + L) * 4
    work = kernel_work(infer, N, E, cfg["steps"], nslab_bytes, fused, fused and getattr(eng, "gz1e_from_gc", False))
    comp = compulsory_bytes(work, N, E)
    pmc_path, pmc_reason = pmc_file(config=cid)
    pmc = load_pmc(fused, pmc_path)
    sq_path, sq_reason = sq_file(config=cid)
    sq = load_sq(sq_path)
    step_s = el * ev_steps / args.steps
    dominant = max([k for k in ("edge_fwd", "edge_bwd", "edge_gout", "wgrad_W2") if k in ktot], key=lambda k: ktot[k])
    strong = bool(cfg.get("global_batch"))
    rec = {
        "metric": ("mesh-nodes/sec (inference) on periodic FEM graphs" if infer
                   else "mesh-nodes/sec (fwd+bwd) on periodic FEM graphs"),
        "value": round(total_nodes * args.steps / el, 1),
        "unit": "nodes/s",
        "n_gpus": world,
        "ms_per_step": round(el / args.steps * 1e3, 3),
        "scaling": "strong" if strong else "weak",
        "config": {"workload": cfg["workload"], "graphs_per_gpu": None if strong else cfg["graphs"],
                   "nodes_per_gpu": N, "edges_per_gpu": E,
                   "global_batch": cfg["graphs"] if strong else cfg["graphs"] * world,
                   "message_passing_steps": cfg["steps"], "latent": L, "divergence": cfg["divergence"],
                   "parallelism": f"graph-DP x{world}" + ("" if args.dp_mode == "replica" else " (sync-LN)"),
                   "final_loss": round(loss, 6), "hip_graph_steps": graph_steps,
                   "per_rank": per_rank_rec},
        "kernel_variants": eng.variants(),
        "roofline": roofline(dominant, work, kt, ktot, step_s, pmc, nlaunch, pmc_path, comp,
                             reads_only_bytes(dominant, E)),
        "roofline_gather_scatter": [roofline(k, work, kt, ktot, step_s, pmc, nlaunch, pmc_path, comp)
                                    for k in ("segment_sum", "pq_scatter_bwd") if k in kt],
        "roofline_node_net": (roofline("node_net", work, kt, ktot, step_s, pmc, nlaunch, pmc_path, comp)
                              if "node_net" in kt else None),
        "traffic_null_reason": pmc_reason,
        # MFMA busy from rocprofv3 SQ counters of this tree (tools/sq_pass.sh), beside each roofline's
        # flop-derived frac_mfma: {bench kernel key: SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x 2.4 GHz x duration)}
        "mfma_busy_counters": sq or None,
        "mfma_busy_source": (f"profiles/{Path(sq_path).name}" if sq_path else sq_reason),
        "kernel_ms": {k: round(v * 1e3, 4) for k, v in kt.items()},
    }
    del trainer, model, batch, plan
    torch.cuda.empty_cache()
    return rec, samples


# the reference's only published timings (docs/benchmark_hyperelast.svg, made by
# scripts/benchmark_gnn_fem.py:81-100,485-587): batch-1 forward, 10 MP steps, latent 128, one periodic
# hole plate per size, the mean of 5 strain samples after one warm-up, on an unnamed CUDA GPU.
# (reference nodes, decoded fwd ms, decoded fwd + mesh->graph ms, our grid n, hole radius / plate side):
# pdg.meshgen.hole_plate(n, r) gives a triangulated 100 x 100 periodic plate with a central hole of the
# reference's radius (30, i.e. 0.29-0.31 here) and within 2 nodes of each reference node count; the
# reference's gmsh mesh refines towards the hole instead (same graph format, similar E/N).
PUBLISHED_SWEEP = [(458, 11.6, 15.4, 25, 0.3005), (1918, 34.5, 39.2, 51, 0.297), (4624, 74.6, 84.7, 79, 0.292),
                   (9957, 161.1, 175.3, 119, 0.3105), (15259, 242.1, 261.3, 147, 0.308),
                   (20411, 320.5, 345.7, 168, 0.2985), (25556, 402.8, 436.5, 186, 0.29)]


def published_mesh(n: int, r: float):
    """One sweep mesh as the reference's benchmark holds it on the host before the timed region: points
    (N, 3) float32 with z = 0 (pyvista), triangles (F, 3) int64, node labels (compute_node_labels)."""
    import numpy as np
    from pdg import meshgen
    m = meshgen.hole_plate(n=n, hole_radius=r, seed=69, strain_range=(-0.15, 0.15))
    pts = np.concatenate([m.pos, np.zeros((m.num_nodes, 1), np.float32)], 1)
    return m, pts, m.faces.astype(np.int64), m.node_types.astype(np.int64)


def published_model(device, sample):
    from gnn_local_stress.models import EncodeProcessDecode
    torch.manual_seed(69)
    st = {"mean_pos": float(sample.pos.mean()), "std_pos": float(sample.pos.std(ddof=1)),
          "mean_mean_stress": 0.0, "std_mean_stress": 0.1, "mean_local_stress": float(sample.local_stress.mean()),
          "std_local_stress": float(sample.local_stress.std(ddof=1)), "mean_edge_weight": float(sample.edge_attr.mean()),
          "std_edge_weight": float(sample.edge_attr.std(ddof=1))}
    st = {k: torch.tensor(v) for k, v in st.items()}
    m = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=10, latent_size=L,
                            input_nodes_features_size=6, output_nodes_features_size=3, **st).to(device)
    return m.eval()


def published_sweep(device, reps: int = 5) -> dict:
    """The reference's published workload (benchmark_gnn_fem.py:485-587) on this GPU: per mesh size, the
    mean (as the reference reports) and median of `reps` strain samples after one warm-up of
      fwd         the reference's blue series (:87-100, use_preprocessing=False): the device graph is built
                  before the clock starts; timed = model.forward(graph) (zero-stress guard with its host
                  synchronisation, the graph's CSR plan, format / encode / 10 steps / decode)
      fwd_prepro  the orange series (use_preprocessing=True): timed = host mesh -> HBM (points, triangles,
                  labels), FaceToEdge + lengths + periodic pairs + coalesce on the device (pdg_mesh_graph),
                  the graph's fields, model.forward
      fwd_replay  the same forward replayed from a HIP graph captured once per mesh (pdg/serve.py: the
                  graph is fixed, only the imposed mean strain changes, as in the reference's loop :560-567)
    with the GPU time of one replay (HIP events on the stream; launches back to back, so it is the
    kernel sum plus the intra-graph gaps) and the library calls per forward.  Each row also checks the
    three series' outputs are bitwise equal."""
    import numpy as np
    from pdg import devgraph, hiptimer
    from pdg.lib import lib
    from pdg.serve import CapturedForward
    rng = np.random.default_rng(69)
    rows = []
    sync = torch.cuda.synchronize
    for ref_n, ref_fwd, ref_pre, n, r in PUBLISHED_SWEEP:
        sample, pts_h, faces_h, lab_h = published_mesh(n, r)
        model = published_model(device, sample)
        strains = rng.uniform(-0.15, 0.15, size=(reps + 1, 3)).astype(np.float32)
        pts_d, faces_d, lab_d = (torch.from_numpy(a).to(device) for a in (pts_h, faces_h, lab_h))

        def fwd_only(ms):
            g = devgraph.convert_mesh_to_graph(pts_d, faces_d, ms, lab_d)
            sync()
            t0 = time.perf_counter()
            with torch.no_grad():
                y = model(g).local_stress
            sync()
            return time.perf_counter() - t0, y, g

        def fwd_prepro(ms):
            sync()
            t0 = time.perf_counter()
            p, f, lab = (torch.from_numpy(a).to(device) for a in (pts_h, faces_h, lab_h))
            g = devgraph.convert_mesh_to_graph(p, f, ms, lab)
            with torch.no_grad():
                y = model(g).local_stress
            sync()
            return time.perf_counter() - t0, y

        _, _, g0 = fwd_only(strains[0])             # warm-up (the reference's dummy launch, :536-538)
        fwd_prepro(strains[0])
        cap = CapturedForward(model, g0)
        cap(strains[0])
        t_f, t_p, t_r, gpu = [], [], [], []
        same = True
        for ms in strains[1:]:
            c0 = lib.calls
            t, y_f, _ = fwd_only(ms)
            calls = lib.calls - c0
            t_f.append(t)
            t, y_p = fwd_prepro(ms)
            t_p.append(t)
            a, b = hiptimer.Event(), hiptimer.Event()
            sync()
            t0 = time.perf_counter()
            a.record()
            y_r = cap(ms)
            b.record()
            sync()
            t_r.append(time.perf_counter() - t0)
            gpu.append(a.elapsed_time(b) * 1e-3)
            same = same and torch.equal(y_f, y_p) and torch.equal(y_f, y_r)

        def ms_(v):
            return {"mean_ms": round(statistics.mean(v) * 1e3, 4), "median_ms": round(statistics.median(v) * 1e3, 4)}
        N, E = sample.num_nodes, sample.num_edges
        rows.append({"nodes": N, "edges": E, "grid_n": n, "hole_radius": r, "reference_nodes": ref_n,
                     "fwd": ms_(t_f), "fwd_prepro": ms_(t_p), "fwd_replay": ms_(t_r),
                     "replay_gpu_ms": round(statistics.median(gpu) * 1e3, 4),
                     "library_calls_per_fwd": calls, "graph_launches_per_replay": cap.launches,
                     "nodes_per_s_fwd": round(N / statistics.mean(t_f), 1),
                     "nodes_per_s_replay": round(N / statistics.mean(t_r), 1),
                     "reference_fwd_ms": ref_fwd, "reference_fwd_prepro_ms": ref_pre,
                     "speedup_vs_reference_fwd": round(ref_fwd / (statistics.mean(t_f) * 1e3), 2),
                     "speedup_vs_reference_fwd_prepro": round(ref_pre / (statistics.mean(t_p) * 1e3), 2),
                     "outputs_bitwise_equal": bool(same)})
        del cap, model
        torch.cuda.empty_cache()
    return {"workload": "the reference's published sweep (scripts/benchmark_gnn_fem.py:81-100,485-587): batch-1 "
                        "forward, 10 MP steps, latent 128, one periodic 100 x 100 hole plate (hole radius ~30) per size, "
                        f"mean of {reps} imposed mean strains in +-0.15 after one warm-up, fp32",
            "reference_source": "BASELINE.md §1 (decoded from docs/benchmark_hyperelast.svg; unnamed CUDA GPU, "
                                "not a same-node comparison)",
            "rows": rows}


def time_plumbing(args, rank: int, world: int, pg, device) -> dict:
    """--plumbing: the multi-rank flow of time_config with one all-reduce of a gradient-sized
    bucket as the only work (no HIP kernels; CPU tests with gloo)."""
    bucket = torch.zeros(N_PARAMS, dtype=torch.float32, device=device)
    for _ in range(args.warmup):
        dist.all_reduce(bucket) if pg is not None else None
    if pg is not None:
        dist.barrier()
    t0 = time.perf_counter()
    ar = 0.0
    for _ in range(args.steps):
        if pg is not None:
            t1 = time.perf_counter()
            dist.all_reduce(bucket)
            ar += time.perf_counter() - t1
    el_local = time.perf_counter() - t0
    if pg is not None:
        dist.barrier()
    el = _max_over_ranks(time.perf_counter() - t0, world, device)
    per_rank = _allgather_ints([rank, dist.get_world_size() if pg is not None else 1], world, device)
    split = per_rank_fields(world, device, pg, [0, 0, 0], el_local / args.steps * 1e3, ar / args.steps * 1e3, 0.0)
    return {"metric": "plumbing only (no HIP kernels): launch, rendezvous, timing and reporting of bench.py",
            "value": None, "unit": "nodes/s", "n_gpus": world, "ms_per_step": round(el / args.steps * 1e3, 3),
            "scaling": "weak", "plumbing": True,
            "config": {"workload": "gradient-bucket all-reduce only", "parallelism": f"graph-DP x{world}",
                       "per_rank": {"rank": [r[0] for r in per_rank], "world_seen": [r[1] for r in per_rank],
                                    **split}}}


# ---------------------------------------------------------------------------------- launch
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _spawned_rank(i: int, n: int) -> None:
    os.environ.update(RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(n))
    main()


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--dp-mode", default="replica", choices=["replica", "sync"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="main line only (no config 3/4/5 sub-results)")
    ap.add_argument("--extra-steps", type=int, default=10, help="timed steps of each sub-result")
    ap.add_argument("--graph", action="store_true",
                    help="replay forward+backward from a HIP graph captured in warmup (measured no faster: DESIGN §6)")
    ap.add_argument("--no-sweep", action="store_true", help="skip the published-workload sweep (sub_results)")
    ap.add_argument("--sweep-only", action="store_true", help="only the published-workload sweep (one JSON line)")
    ap.add_argument("--plumbing", action="store_true",
                    help="launch/rendezvous/report flow only, no HIP kernels (CPU tests)")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: spawn one rank per GPU before anything initialises the GPU here
        import torch.multiprocessing as mp
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        mp.start_processes(_spawned_rank, args=(args.gpus,), nprocs=args.gpus, start_method="spawn", join=True)
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} ranks")
    # one process per GPU; PDG_DIST_BACKEND=gloo with more ranks than GPUs only rehearses the
    # multi-rank flow (ranks share devices round-robin)
    backend = os.environ.get("PDG_DIST_BACKEND", "gloo" if args.plumbing else "nccl")
    if args.plumbing:
        device = torch.device("cpu")
    else:
        dev_index = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(dev_index)
        device = torch.device("cuda", dev_index)
    pg = None
    # PDG_FORCE_PG=1: a process group (and the Trainer's all-reduce) even at one rank, to rehearse the
    # RCCL data path on a one-GPU box
    if world > 1 or os.environ.get("PDG_FORCE_PG") == "1":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
        pg = dist.group.WORLD
        assert dist.get_world_size() == world

    if args.sweep_only:
        if rank == 0:
            print(json.dumps({"published_sweep": published_sweep(device), "tree": tree_hash()}), flush=True)
        return
    if args.plumbing:
        res = time_plumbing(args, rank, world, pg, device)
        subs = {}
    else:
        res, samples = time_config(args.config, args, rank, world, pg, device)
        subs = {}
        if args.config == 2 and not args.no_extras:
            sub_args = argparse.Namespace(**{**vars(args), "steps": args.extra_steps})
            for cid in (3, 4, 5):
                r, s = time_config(cid, sub_args, rank, world, pg, device)
                subs[f"config{cid}"] = (r, s)
    if rank == 0:
        line = {"metric": res["metric"], "value": res["value"], "unit": res["unit"], "n_gpus": res["n_gpus"],
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": res["ms_per_step"],
                "higher_is_better": True, "scaling": res["scaling"], "vs_baseline": None, "dtype": "f32",
                "data": "synthetic periodic triangulated meshes (pdg.meshgen, seed 69+rank), random-init weights (seed 69)",
                "world_size_rccl": dist.get_world_size() if pg is not None else 1,
                "backend": backend if pg is not None else None}
        line.update({k: v for k, v in res.items() if k not in line})
        cpu_ok = world == 1 and not args.no_cpu_baseline and not args.plumbing
        line["tree"] = tree_hash()
        line["pmc_tree"] = pmc_tree()
        line["traffic_tree_match"] = line["pmc_tree"] == line["tree"]
        cfg0 = CONFIGS[args.config]
        # bounded samples (10-30 s of CPU work each): 2 graphs of a training batch, the config-5 mesh itself
        line["cpu_baseline"] = (cpu_baseline(cfg0, samples[:2], full_graphs=cfg0["graphs"]) if cpu_ok else None)
        if subs:
            line["sub_results"] = {}
            for name, (r, s) in subs.items():
                cfg = CONFIGS[int(name[-1])]
                if cpu_ok:
                    r["cpu_baseline"] = cpu_baseline(cfg, s[:2], full_graphs=cfg["graphs"], one_thread=False)
                r["steps"], r["warmup"] = args.extra_steps, args.warmup
                line["sub_results"][name] = r
        if cpu_ok and args.config == 2 and not args.no_extras and not args.no_sweep:
            line.setdefault("sub_results", {})["published_sweep"] = published_sweep(device)
        print(json.dumps(line), flush=True)
    if pg is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
