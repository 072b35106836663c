"""The cached oracle results at the BASELINE sizes (tests/golden/fullsize_c*.npz, made by
tests/golden/make_fullsize.py) belong to the workloads bench.py builds today: each fixture's hash of
the batch arrays, divergence operators, initial parameters and statistics equals the hash of the
workload built now (a stale fixture is caught here, on the CPU, before the GPU suite would fall back to
the slow live oracle), and it holds the fp32 oracle's distance for every parameter."""
import sys
from pathlib import Path

import numpy as np
import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))


@pytest.mark.parametrize("config", [2, 3, 4, 5])
def test_fullsize_fixture_matches_the_bench_workload(config):
    from make_fullsize import workload, workload_hash
    from pdg.engine import PARAM_NAMES
    path = Path(__file__).resolve().parent / "golden" / f"fullsize_c{config}.npz"
    z = np.load(path, allow_pickle=False)
    cfg, batch, stats, params = workload(config)
    assert str(z["hash"]) == workload_hash(batch, params, stats)
    assert z["pred64"].shape == (batch.num_nodes, 3)
    assert {k[5:]: float(z[k]) for k in z.files if k.startswith("stat.")} == stats
    if not cfg.get("inference"):
        assert {k[7:] for k in z.files if k.startswith("grad64.")} == set(PARAM_NAMES)
        assert all(0.0 < float(z[f"grad32_vs_f64.{n}"]) < 1e-3 for n in PARAM_NAMES)
