"""The torch.library boundary: torch.ops.pdivgnn.epd_forward / epd_backward and
batch_loss / batch_loss_backward, called directly, through autograd, and under opcheck.

* the op called with the batch tensors gives the model's output bit for bit (the model runs
  through the same op) and its registered backward gives the model's gradients bit for bit;
* the activations behind a handle are released after the backward and when the graph is
  dropped without one (no leak across training steps);
* torch.library.opcheck: schema, fake (meta) implementation and autograd registration.
"""
import gc

import pytest
import torch

from gpu_common import dataset_stats, make_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _setup(steps=3, n=13, graphs=2):
    from gnn_local_stress.models import EncodeProcessDecode
    from pdg import meshgen
    samples = meshgen.make_dataset(graphs, n=n, hole_radius=(0.15, 0.25), seed=11)
    batch = make_batch(samples)
    stats = {k: torch.as_tensor(float(v)) for k, v in dataset_stats(batch).items()}
    torch.manual_seed(69)
    m = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=steps, latent_size=128,
                            input_nodes_features_size=6, output_nodes_features_size=3, **stats).to("cuda")
    return m, batch


def _op_args(m, b, need_grad):
    from pdg.engine import PARAM_NAMES
    params = [m.get_parameter(n) for n in PARAM_NAMES]
    return (params, m.stats_tensor(b.pos.device), b.pos, b.mean_stress, b.nodes_types, b.edge_attr, b.edge_index,
            b.num_nodes, m.message_passing_steps, True, True, need_grad, 0)


def test_epd_forward_op_equals_model_and_backward_releases_handles():
    from pdg import ops
    from pdg.engine import PARAM_NAMES
    m, b = _setup()
    with torch.no_grad():
        ref = m(b).local_stress
        y, h = torch.ops.pdivgnn.epd_forward(*_op_args(m, b, False))
    assert torch.equal(y, ref) and int(h[0]) == 0
    # autograd through the op (model path) vs the op called directly
    n0 = len(ops._ctx)
    out = m(b).local_stress
    (out * out).sum().backward()
    g_model = {n: m.get_parameter(n).grad.clone() for n in PARAM_NAMES}
    m.zero_grad()
    y, h = torch.ops.pdivgnn.epd_forward(*_op_args(m, b, True))
    assert len(ops._ctx) == n0 + 1
    (y * y).sum().backward()
    assert len(ops._ctx) == n0            # popped by the backward
    for n in PARAM_NAMES:
        assert torch.equal(m.get_parameter(n).grad, g_model[n]), n
    # a forward whose graph is dropped without a backward releases its activations
    y, h = torch.ops.pdivgnn.epd_forward(*_op_args(m, b, True))
    assert len(ops._ctx) == n0 + 1
    del y, h
    gc.collect()
    assert len(ops._ctx) == n0


def test_batch_loss_op_matches_and_opcheck():
    from gnn_local_stress import losses
    from pdg.plan import plan_for
    m, b = _setup(steps=2)
    with torch.no_grad():
        pred = m(b, scale_output=False).local_stress
    pred = pred.clone().requires_grad_(True)
    gt = (b.local_stress - m.mean_local_stress) / m.std_local_stress
    total, nmse, div = losses.batch_loss(pred, b, gt, divergence=True, divergence_penalty=10.0)
    total.backward()
    p = plan_for(b)
    args = (pred.detach(), gt, p.ptr, b.nodes_types, p.a_rowptr, p.a_col, p.a_val, p.at_rowptr, p.at_row,
            p.at_comp, p.at_val, True, True, 10.0, False)
    t2, n2, d2, _, _ = torch.ops.pdivgnn.batch_loss(*args)
    assert torch.equal(t2, total.detach()) and torch.equal(n2, nmse) and torch.equal(d2, div)
    assert float(pred.grad.abs().sum()) > 0
    args_g = (pred.detach().clone().requires_grad_(True),) + args[1:]
    torch.library.opcheck(torch.ops.pdivgnn.batch_loss.default, args_g,
                          test_utils=("test_schema", "test_faketensor", "test_autograd_registration"))


def test_epd_forward_opcheck_schema_and_fake():
    m, b = _setup(steps=2, n=9, graphs=1)
    with torch.no_grad():
        args = _op_args(m, b, False)
    args = ([p.detach() for p in args[0]],) + args[1:]
    torch.library.opcheck(torch.ops.pdivgnn.epd_forward.default, args,
                          test_utils=("test_schema", "test_faketensor"))


def test_ops_refuse_cpu_tensors():
    m, b = _setup(steps=1, n=7, graphs=1)
    args = list(_op_args(m, b, False))
    args[2] = args[2].cpu()
    with pytest.raises(RuntimeError, match="HIP device"):
        torch.ops.pdivgnn.epd_forward(*args)


def test_batch_loss_separate_outputs_carry_gradients():
    """nmse and div are differentiable outputs (total = nmse + div): d(a*nmse + b*div)/d(pred)
    = a*d(nmse) + b*d(div), each part checked against the fp64 oracle's gradient."""
    from gnn_local_stress import losses
    from oracle import epd_oracle as O
    m, b = _setup(steps=2)
    with torch.no_grad():
        pred0 = m(b, scale_output=False).local_stress
    gt = ((b.local_stress - m.mean_local_stress) / m.std_local_stress).float().contiguous()
    ops64 = [d.op_div_matrix.double() for d in b._data_list]

    def oracle_grad(wn, wd):
        p = pred0.detach().cpu().double().requires_grad_(True)
        _, n, d = O.batch_loss(p, gt.cpu().double(), b.ptr, ops64, b.nodes_types.cpu(), True, 10.0)
        (wn * n + wd * d).backward()
        return p.grad

    for wn, wd in ((1.0, 0.0), (0.0, 1.0), (2.0, -0.5)):
        pred = pred0.clone().requires_grad_(True)
        _, nmse, div = losses.batch_loss(pred, b, gt, divergence=True, divergence_penalty=10.0)
        (wn * nmse + wd * div).backward()
        ref = oracle_grad(wn, wd)
        err = float((pred.grad.double().cpu() - ref).norm() / ref.norm())
        assert err < 1e-5, (wn, wd, err)


def test_model_engines_are_freed_with_the_model():
    """A model's executor (and its device scratch) is unregistered when the model is collected."""
    from pdg import ops
    n0 = len(ops._engines)
    for _ in range(3):
        m, b = _setup(steps=1, n=9, graphs=1)
        out = m(b).local_stress
        out.sum().backward()
        assert len(ops._engines) == n0 + 1
        del m, out
        gc.collect()
        assert len(ops._engines) == n0
