"""Optimizer-step parity: the HIP Adam + non-finite skip of pdg.trainer.Trainer
against the reference's own update, torch.optim.Adam(lr=1e-3) stepped through
GradScaler (scripts/gnn_train.py:111,118,204-207), applied on the CPU to the SAME gradients
the HIP backward produced.

* Five steps: exp_avg and exp_avg_sq are BIT-IDENTICAL (pdg_adam rounds every operation the
  way torch's CPU kernels do: fma in lerp_ and addcmul_, (s*m)/d in addcdiv_); parameters agree
  to a few ulps: torch's vectorised CPU sqrt (SLEEF, 0.5001 ulp) differs from the correctly
  rounded sqrt of the GPU (and of CUDA, where the reference trains) in ~0.7 % of elements by
  one ulp of the denominator.
* An injected NaN gradient: GradScaler skips optimizer.step(), so parameters, moments and
  Adam's step count stay put and the next step's bias correction is that of the step after
  the last real one (the advisor's round-1 finding).
* A batch whose mean stress is all zero (the guard of gnn_local_stress/models.py:294-299, where
  the reference's forward returns zeros without a graph and no update can follow) skips the
  step the same way: nothing moves, ``skipped`` is 1.
* Assigning ``trainer.lr`` between steps takes effect at the next step, as assigning the
  param group's lr does for torch.optim.Adam.
* state_dict() speaks torch.optim.Adam's format: a Trainer resumed from it, and a torch Adam
  resumed from it, continue identically.
"""
import pytest
import torch

from gpu_common import dataset_stats, dev
from pdg import graph, meshgen

pytestmark = pytest.mark.gpu

RTOL_P, ATOL_P = 5e-7, 1e-9       # a few fp32 ulps of the parameters (sqrt rounding, above)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _setup(divergence=True):
    from gnn_local_stress.models import EncodeProcessDecode
    from pdg.trainer import Trainer
    samples = meshgen.make_dataset(3, n=11, hole_radius=(0.1, 0.2), seed=5)
    batch = graph.Batch.from_data_list([graph.sample_to_data(s) for s in samples]).to(dev())
    stats = {k: torch.tensor(float(v)) for k, v in dataset_stats(batch).items()}
    torch.manual_seed(69)
    model = EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=2, latent_size=128,
                                input_nodes_features_size=6, output_nodes_features_size=3, **stats).to(dev())
    tr = Trainer(model, lr=1e-3, divergence=divergence, divergence_penalty=10.0)
    return tr, batch


class _RefAdam:
    """The reference update on CPU copies of the parameters: Adam + GradScaler (init scale 2^16)."""

    def __init__(self, tr, state=None):
        self.names = [n for n, _ in tr.model.named_parameters()]
        self.params = [torch.nn.Parameter(tr.model.get_parameter(n).detach().cpu().clone()) for n in self.names]
        self.opt = torch.optim.Adam(self.params, lr=1e-3, foreach=False)
        if state is not None:
            self.opt.load_state_dict(state)
        self.scaler = torch.amp.GradScaler("cpu", init_scale=2.0 ** 16)
        self.scaler.scale(torch.ones(()))      # lazy init, as scaler.scale(loss) does in the loop

    def step(self, tr):
        scale = self.scaler.get_scale()
        for n, p in zip(self.names, self.params):
            p.grad = tr.G[n].detach().cpu().clone() * scale   # what backward of scale*loss yields
        self.scaler.step(self.opt)
        self.scaler.update()

    def check(self, tr):
        for n, p in zip(self.names, self.params):
            torch.testing.assert_close(tr.model.get_parameter(n).detach().cpu(), p.detach(), rtol=RTOL_P,
                                       atol=ATOL_P, msg=lambda m: f"{n}: {m}")
        views = {v[0]: v for v in tr._param_views()}
        for i, (n, p) in enumerate(zip(self.names, self.params)):
            st = self.opt.state.get(p)
            _, o, k, shape = views[n]
            m = tr.exp_avg[o:o + k].view(shape).cpu()
            v = tr.exp_avg_sq[o:o + k].view(shape).cpu()
            if not st:
                assert not m.any() and not v.any()
                continue
            assert torch.equal(m, st["exp_avg"]), n
            assert torch.equal(v, st["exp_avg_sq"]), n

    def steps_taken(self):
        st = self.opt.state.get(self.params[0])
        return int(float(st["step"])) if st else 0


def _step(tr, batch, poison=False):
    """Trainer.step with an optional NaN injected between backward and the update."""
    from pdg.lib import stream_handle
    from pdg.plan import plan_for
    if not poison:
        return tr.step(batch)
    plan = plan_for(batch)
    f32 = dict(dtype=torch.float32, device=tr.device)
    out = tr._fwd_bwd(batch, plan, tr.model.stats_tensor(tr.device), plan.n_graphs, plan.n_nodes, plan.n_graphs,
                      f32, stream_handle(tr.device))
    tr.flat_g[1234] = float("nan")
    return tr._update(out, f32, stream_handle(tr.device), tr._nonzero_flag(batch))


def test_adam_matches_torch_over_steps():
    tr, batch = _setup()
    ref = _RefAdam(tr)
    p0 = tr.flat_p.clone()
    for _ in range(5):
        _step(tr, batch)
        torch.cuda.synchronize()
        ref.step(tr)
        ref.check(tr)
    assert tr.step_count == ref.steps_taken() == 5
    assert not torch.equal(p0, tr.flat_p)


def test_nonfinite_gradient_skips_step_and_count():
    tr, batch = _setup()
    ref = _RefAdam(tr)
    for poison in (False, False, True, False, True, True, False):
        before = (tr.flat_p.clone(), tr.exp_avg.clone(), tr.exp_avg_sq.clone(), tr.step_count)
        out = _step(tr, batch, poison)
        torch.cuda.synchronize()
        assert int(out["skipped"]) == int(poison)
        ref.step(tr)
        if poison:   # GradScaler skipped optimizer.step(): nothing moved
            assert torch.equal(before[0], tr.flat_p) and torch.equal(before[1], tr.exp_avg)
            assert torch.equal(before[2], tr.exp_avg_sq) and before[3] == tr.step_count
        ref.check(tr)
        assert tr.step_count == ref.steps_taken()
    assert tr.step_count == 4


def test_state_dict_round_trip_with_torch_adam():
    from pdg.trainer import Trainer
    tr, batch = _setup(divergence=False)
    for _ in range(3):
        tr.step(batch)
    sd = tr.state_dict()
    assert set(sd["state"]) == set(range(len(list(tr.model.parameters()))))
    assert all(float(s["step"]) == 3.0 for s in sd["state"].values())
    # a torch Adam loads it (format check) and a fresh Trainer resumes from it
    ref = _RefAdam(tr, state=sd)
    tr2 = Trainer(tr.model, lr=5.0, divergence=False)   # lr comes from the state dict
    tr2.load_state_dict(sd)
    assert tr2.lr == 1e-3 and tr2.step_count == 3
    for _ in range(2):
        tr2.step(batch)
        torch.cuda.synchronize()
        ref.step(tr2)
        ref.check(tr2)
    assert tr2.step_count == 5


def test_zero_mean_stress_batch_skips_update():
    tr, batch = _setup(divergence=True)
    tr.step(batch)
    torch.cuda.synchronize()
    import copy
    zero = copy.copy(batch)                   # same graph, its own attribute dict
    zero.mean_stress = torch.zeros_like(batch.mean_stress)
    before = (tr.flat_p.clone(), tr.exp_avg.clone(), tr.exp_avg_sq.clone(), tr.step_count)
    out = tr.step(zero)
    torch.cuda.synchronize()
    assert int(out["skipped"]) == 1
    assert torch.equal(before[0], tr.flat_p) and torch.equal(before[1], tr.exp_avg)
    assert torch.equal(before[2], tr.exp_avg_sq) and tr.step_count == before[3]
    # the guard is per batch content: the original batch steps again, and an in-place zeroing of a
    # batch already seen is noticed (the flag cache keys on the tensor's version counter)
    out = tr.step(batch)
    torch.cuda.synchronize()
    assert int(out["skipped"]) == 0 and tr.step_count == before[3] + 1
    batch.mean_stress.zero_()
    out = tr.step(batch)
    torch.cuda.synchronize()
    assert int(out["skipped"]) == 1 and tr.step_count == before[3] + 1


def test_lr_assignment_takes_effect():
    tr, batch = _setup(divergence=False)
    ref = _RefAdam(tr)
    for lr in (1e-3, 1e-3, 3e-4, 3e-4, 2e-3):
        tr.lr = lr
        for g in ref.opt.param_groups:
            g["lr"] = lr
        _step(tr, batch)
        torch.cuda.synchronize()
        ref.step(tr)
        ref.check(tr)
