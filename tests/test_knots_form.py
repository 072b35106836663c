"""The piecewise-linear ("knot table") form of the edge encoder that pdg_edge_enc_fwd_knots evaluates
(DESIGN §4, A/B variant), restated in numpy and checked against the direct form of models.py:264-275
(a1 = relu(w0 e + b0), a2 = relu(W2 a1 + b2)): the interval relu mask equals the direct fp32 mask on every
edge, and the knot form's a2 is within fp32 rounding of fp64 -- on random weights with zero first-layer
weights and repeated knots, and on the reference checkpoint's edge encoder with the batch3_div golden edges.
Host-side restatement of the kernel's table (edge_knots_kernel); the kernel itself is tested on the GPU
(tests/test_gpu_ops.py::test_edge_enc_fwd_knots_edge_cases)."""
import numpy as np
import pytest
import torch

from golden_io import GOLDEN, load


def knot_table(w0, b0, W2, b2):
    tau = np.where(w0 != 0, -b0 / np.where(w0 != 0, w0, 1), np.float32(3.4028235e38)).astype(np.float32)
    order = np.lexsort((np.arange(tau.size), tau))   # ties by feature index, as the kernel's ranks
    rank = np.empty(tau.size, int)
    rank[order] = np.arange(tau.size)
    W = W2.astype(np.float64)
    U = np.zeros((tau.size + 1, W.shape[0]))
    V = np.zeros_like(U)
    for i in range(tau.size + 1):
        act = np.where(w0 > 0, rank < i, np.where(w0 < 0, rank >= i, b0 > 0))
        U[i] = W[:, act] @ w0[act].astype(np.float64)
        V[i] = b2.astype(np.float64) + W[:, act] @ b0[act].astype(np.float64)
    return tau[order], rank, U.astype(np.float32), V.astype(np.float32)


def check(e, w0, b0, W2, b2):
    knots, rank, U, V = knot_table(w0, b0, W2, b2)
    pos = np.searchsorted(knots, e, side="left")     # knots strictly below e
    act = np.where(w0 > 0, rank[None, :] < pos[:, None], np.where(w0 < 0, rank[None, :] >= pos[:, None], b0 > 0))
    direct = (e[:, None] * w0).astype(np.float32) + b0 > 0
    assert (act == direct).all()
    a2 = np.maximum((e[:, None].astype(np.float64) * U[pos] + V[pos]).astype(np.float32), 0)   # one fma
    ref = np.maximum(np.maximum(e[:, None].astype(np.float64) * w0 + b0, 0) @ W2.T.astype(np.float64) + b2, 0)
    err = np.linalg.norm(a2 - ref) / np.linalg.norm(ref)
    assert err < 2e-7, err


def test_knot_form_random_weights():
    rng = np.random.default_rng(3)
    w0 = rng.normal(size=128).astype(np.float32)
    b0 = rng.normal(size=128).astype(np.float32)
    w0[:6] = 0
    b0[:3] = np.abs(b0[:3])
    w0[40], b0[40] = w0[41], b0[41]                 # a repeated knot
    W2 = (rng.normal(size=(128, 128)) / 11).astype(np.float32)
    b2 = rng.normal(size=128).astype(np.float32)
    e = np.concatenate([rng.normal(scale=3, size=4000), [0.0, -0.0]]).astype(np.float32)
    check(e, w0, b0, W2, b2)


def test_knot_form_reference_checkpoint():
    sd = torch.load(GOLDEN / "ref_checkpoint.pth", weights_only=True, map_location="cpu")
    sd = sd.get("model_state_dict", sd)
    if "edge_encoder.0.weight" not in sd:
        pytest.skip("checkpoint layout without the edge encoder")
    e = np.asarray(load("batch3_div")["edge_attr"], dtype=np.float32).reshape(-1)
    check(e, sd["edge_encoder.0.weight"].numpy()[:, 0].astype(np.float32),
          sd["edge_encoder.0.bias"].numpy().astype(np.float32), sd["edge_encoder.2.weight"].numpy().astype(np.float32),
          sd["edge_encoder.2.bias"].numpy().astype(np.float32))
