"""bench.py's multi-rank launch paths on the CPU (gloo), without HIP kernels (--plumbing):

* `bench.py --gpus 2` with no launcher spawns the two ranks itself;
* under torch.distributed.run (the driver's SCALE command) the launcher's ranks are used;
* a rank count that disagrees with --gpus is refused.

Each run must print one JSON line from rank 0 reporting 2 GPUs, the world size the process
group saw on every rank, and per-rank records."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(PDG_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    return env


def _line(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def _check(d):
    assert d["n_gpus"] == 2 and d["world_size_rccl"] == 2 and d["plumbing"] is True
    assert d["config"]["per_rank"]["rank"] == [0, 1]
    assert d["config"]["per_rank"]["world_seen"] == [2, 2]
    pr = d["config"]["per_rank"]
    # the per-rank split of a step the driver's 8-GPU run reports
    for k in ("step_ms", "allreduce_ms", "sync_ln_collectives_ms", "compute_ms", "world_size_rccl", "nodes"):
        assert len(pr[k]) == 2, k
    assert pr["world_size_rccl"] == [2, 2]
    assert all(a > 0 for a in pr["allreduce_ms"])
    assert all(abs(s - a - c) < 1e-2 for s, a, c in zip(pr["step_ms"], pr["allreduce_ms"], pr["compute_ms"]))
    assert d["value"] is None and d["ms_per_step"] > 0


def test_bench_spawns_ranks_itself():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--plumbing", "--steps", "3",
                        "--warmup", "1"], capture_output=True, text=True, env=_env(), timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    _check(_line(r.stdout))


def test_bench_under_torchrun():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(ROOT / "bench.py"),
                        "--gpus", "2", "--plumbing", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, env=_env(), timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    _check(_line(r.stdout))


def test_bench_refuses_rank_mismatch():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--plumbing"],
                       capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)
    assert r.returncode != 0 and "--gpus 2" in (r.stderr + r.stdout)
