"""Resume from a checkpoint written by the reference: the fixture
tests/golden/ref_checkpoint.pth holds the reference model + torch.optim.Adam state after one
training step of gnn_train.py:154-207 on the batch3_div golden batch (3 MP steps, divergence
lambda=10).  Loaded with the drop-in load_model_checkpoint (weights_only=True):

* the HIP forward reproduces the reference's post-step output (1e-5 relative);
* a Trainer resumed from the checkpoint's optimizer state takes the reference's second step:
  the loss it reports equals the reference's step-2 loss (1e-5) and the parameters after it
  equal the reference's (relative L2 per tensor; Adam's m/sqrt(v) amplifies fp32 gradient
  noise only where a gradient component is itself at noise level)."""
import numpy as np
import pytest
import torch

from golden_io import GOLDEN
from gpu_common import dev, golden_batch, rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _loaded_model():
    from gnn_local_stress import models
    m = models.EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=3, latent_size=128,
                                   input_nodes_features_size=6, output_nodes_features_size=3)
    epoch = models.load_model_checkpoint(m, (GOLDEN / "ref_checkpoint.pth").as_posix())
    return m.to(dev()), epoch


def test_forward_from_reference_checkpoint():
    case = np.load(GOLDEN / "ref_checkpoint_case.npz", allow_pickle=False)
    _, batch = golden_batch("batch3_div")
    m, epoch = _loaded_model()
    assert epoch == 1
    with torch.no_grad():
        out = m(batch, scale_output=True).local_stress
    assert rel(out, case["out_scaled_after_step1"]) < 1e-5


def test_resume_training_from_reference_checkpoint():
    from gnn_local_stress import models
    from pdg.trainer import Trainer
    case = np.load(GOLDEN / "ref_checkpoint_case.npz", allow_pickle=False)
    _, batch = golden_batch("batch3_div")
    m, _ = _loaded_model()
    tr = Trainer(m, lr=0.5, divergence=True, divergence_penalty=10.0)      # lr is taken from the checkpoint
    models.load_model_checkpoint(m, (GOLDEN / "ref_checkpoint.pth").as_posix(), optimizer=tr)
    assert tr.lr == 1e-3 and tr.step_count == 1
    out = tr.step(batch)
    torch.cuda.synchronize()
    assert abs(float(out["total"]) - float(case["loss_step2"])) <= 1e-5 * abs(float(case["loss_step2"]))
    assert tr.step_count == 2
    worst = max(rel(p, case[f"param_after_step2.{n}"]) for n, p in m.state_dict().items())
    assert worst < 1e-5, worst
