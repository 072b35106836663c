"""The CPU oracle (oracle/epd_oracle.py) reproduces the reference's own outputs,
losses and gradients stored in tests/golden (made by tests/golden/make_golden.py)."""
import numpy as np
import pytest
import torch

from golden_io import CASES, load
from oracle import epd_oracle as O


def _rel(a, b):
    a = torch.as_tensor(a).double()
    b = torch.as_tensor(b).double()
    return float((a - b).norm() / max(b.norm(), 1e-30))


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference_outputs_and_grads(case):
    torch.set_num_threads(1)
    g = load(case)
    p = {k: v.clone().requires_grad_(True) for k, v in g["params"].items()}
    args = (torch.from_numpy(g["pos"]), torch.from_numpy(g["mean_stress"]),
            torch.from_numpy(g["nodes_types"]), torch.from_numpy(g["edge_index"]),
            torch.from_numpy(g["edge_attr"]))
    steps = int(g["steps"])
    with torch.no_grad():
        lat = []
        out = O.epd_forward(p, g["stats"], *args, steps, scale_output=True, latents=lat)
    assert _rel(out, g["out_scaled"]) < 1e-6
    for t in range(steps):
        if f"latent_x_{t}" in g:
            assert _rel(lat[t + 1][0], g[f"latent_x_{t}"]) < 1e-6
            assert _rel(lat[t + 1][1], g[f"latent_e_{t}"]) < 1e-6
    pred = O.epd_forward(p, g["stats"], *args, steps, scale_output=False)
    assert _rel(pred.detach(), g["pred"]) < 1e-6
    gt = (torch.from_numpy(g["local_stress"]) - g["stats"]["mean_local_stress"]) / g["stats"]["std_local_stress"]
    assert _rel(gt, g["gt_std"]) == 0.0
    total, nmse, div = O.batch_loss(pred, gt, g["ptr"], g["op_divs"], torch.from_numpy(g["nodes_types"]),
                                    divergence=bool(g["divergence"]), divergence_penalty=float(g["penalty"]))
    assert abs(float(total) - float(g["loss_total"])) <= 1e-6 * abs(float(g["loss_total"]))
    assert abs(float(nmse) - float(g["loss_nmse"])) <= 1e-6 * abs(float(g["loss_nmse"]))
    total.backward()
    for k, ref in g["grads"].items():
        assert _rel(p[k].grad, ref) < 1e-5, k


def test_oracle_init_matches_reference_init():
    g = load("tiny_periodic")
    p = O.init_params(seed=69)
    assert set(p) == set(g["params"])
    for k, v in g["params"].items():
        assert torch.equal(p[k], v), k


def test_divergence_bad_strategy_raises():
    with pytest.raises(AttributeError):
        O.compute_divergence(torch.zeros(3, 3), torch.zeros(3, 6).to_sparse(), torch.zeros(3, 1), "cube")
