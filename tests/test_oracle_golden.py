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
    # Gradients: the reference's fp32 gradients carry their own rounding error (through S graph-global
    # LayerNorms and the divergence term; up to 6e-3 of the exact value on edge_encoder.0.weight), and an
    # fp32 rerun agrees with them bit for bit only on the CPU that made them (the CPU kernels' summation
    # order depends on the vector ISA: on one host the fp32 oracle lands 4e-5 from batch3_div's).  So the
    # fp32 oracle must be within max(1e-5, 2 x the reference's own error), the error measured against the
    # oracle in fp64 — the rule tests/test_gpu_fullsize.py applies to the HIP path.
    e64 = _grads_vs_golden_f64(g, args, steps)
    for k, ref in g["grads"].items():
        assert _rel(p[k].grad, ref) < max(1e-5, 2.0 * e64[k]), (k, _rel(p[k].grad, ref), e64[k])


def _grads_vs_golden_f64(g, args, steps):
    """Relative error of the reference's fp32 gradients against the oracle run in fp64."""
    d = torch.float64
    p = {k: v.clone().to(d).requires_grad_(True) for k, v in g["params"].items()}
    st = {k: (v.to(d) if torch.is_tensor(v) else v) for k, v in g["stats"].items()}
    a = tuple(t.to(d) if t.is_floating_point() else t for t in args)
    pred = O.epd_forward(p, st, *a, steps, scale_output=False)
    gt = (torch.from_numpy(g["local_stress"]).to(d) - st["mean_local_stress"]) / st["std_local_stress"]
    ops = [m.to(d) for m in g["op_divs"]] if g["op_divs"] is not None else None
    total, _, _ = O.batch_loss(pred, gt, g["ptr"], ops, torch.from_numpy(g["nodes_types"]),
                               divergence=bool(g["divergence"]), divergence_penalty=float(g["penalty"]))
    total.backward()
    return {k: _rel(ref, p[k].grad) for k, ref in g["grads"].items()}


def test_oracle_init_matches_reference_init():
    g = load("tiny_periodic")
    p = O.init_params(seed=69)
    assert set(p) == set(g["params"])
    for k, v in g["params"].items():
        assert torch.equal(p[k], v), k


def test_divergence_bad_strategy_raises():
    with pytest.raises(AttributeError):
        O.compute_divergence(torch.zeros(3, 3), torch.zeros(3, 6).to_sparse(), torch.zeros(3, 1), "cube")


def _golden_grads(g, dtype, region=None):
    p = {k: v.clone().to(dtype).requires_grad_(True) for k, v in g["params"].items()}
    st = {k: v.to(dtype) for k, v in g["stats"].items()}
    args = (torch.from_numpy(g["pos"]).to(dtype), torch.from_numpy(g["mean_stress"]).to(dtype),
            torch.from_numpy(g["nodes_types"]), torch.from_numpy(g["edge_index"]),
            torch.from_numpy(g["edge_attr"]).to(dtype))
    pred = O.epd_forward(p, st, *args, int(g["steps"]), scale_output=False, region=region)
    gt = (torch.from_numpy(g["local_stress"]).to(dtype) - st["mean_local_stress"]) / st["std_local_stress"]
    total, _, _ = O.batch_loss(pred, gt, g["ptr"], [m.to(dtype) for m in g["op_divs"]],
                               torch.from_numpy(g["nodes_types"]), divergence=bool(g["divergence"]),
                               divergence_penalty=float(g["penalty"]))
    total.backward()
    return {k: v.grad for k, v in p.items()}


def test_relu_region_is_the_reference_math_inside_its_own_masks():
    """ReluRegion (the analysis hook of the golden GPU gate): with the evaluation's own masks it is
    the reference's math (gradients equal to 1e-14); keep records every relu's pre-activation."""
    g = load("tiny_periodic")
    r = O.ReluRegion(keep=True)
    g0 = _golden_grads(g, torch.float64, r)
    steps = int(g["steps"])
    assert {"enc_n.1", "enc_n.2", "enc_e.1", "enc_e.2", "dec.1"} <= set(r.keep)
    assert all(f"s{t}.{b}.{i}" in r.keep for t in range(steps) for b in "men" for i in (1, 2))
    g1 = _golden_grads(g, torch.float64, O.ReluRegion(masks={k: v > 0 for k, v in r.keep.items()}))
    for k in g0:
        assert _rel(g1[k], g0[k]) < 1e-14, k


def test_fp32_gradient_error_on_the_10_step_case_is_relu_flips():
    """The mechanism behind the golden gate: on batch2_div_s10 the fp32 oracle's
    gradients sit up to ~1e-4 from fp64 because a few relu pre-activations within rounding of zero
    flip; evaluated in its own relu region, fp64 is within 1e-6 of the fp32 gradients on every
    tensor, and every flipped pre-activation is below 1e-5 of its layer's rms."""
    torch.set_num_threads(4)
    g = load("batch2_div_s10")
    r64, r32 = O.ReluRegion(keep=True), O.ReluRegion(keep=True)
    g64 = _golden_grads(g, torch.float64, r64)
    g32 = _golden_grads(g, torch.float32, r32)
    m32 = {k: v > 0 for k, v in r32.keep.items()}
    g64m = _golden_grads(g, torch.float64, O.ReluRegion(masks=m32))
    flips = [(k, int((m32[k] != (r64.keep[k] > 0)).sum())) for k in m32]
    flips = [f for f in flips if f[1]]
    for k, _ in flips:
        h = r64.keep[k]
        assert float(h[m32[k] != (h > 0)].abs().max()) < 1e-5 * float(h.pow(2).mean().sqrt()), k
    in_region = max(_rel(g32[k], g64m[k]) for k in g64)
    assert in_region < 1e-6, in_region
    if flips:   # (how far the flips alone move the gradient is host-dependent; recorded, not bounded)
        print("flips", flips, "in-region", in_region, "unmasked", max(_rel(g32[k], g64[k]) for k in g64))
