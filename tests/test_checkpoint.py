"""A checkpoint written by the REFERENCE's own save_model_checkpoint (models.py:44-63; the
fixture tests/golden/ref_checkpoint.pth is made by tests/golden/make_golden.py after one
reference training step) loads through the drop-in models.load_model_checkpoint with
weights_only=True: parameters, the 8 statistics, the epoch and the Adam state.  The GPU half
(tests/test_gpu_checkpoint.py) runs the loaded model and resumes training from it."""
import numpy as np
import torch

from golden_io import GOLDEN


def test_reference_checkpoint_loads_weights_only():
    from gnn_local_stress import models
    raw = torch.load(GOLDEN / "ref_checkpoint.pth", map_location="cpu", weights_only=True)
    assert set(raw) >= {"model_state_dict", "optimizer_state_dict", "epoch", "mean_pos", "std_pos",
                        "mean_mean_stress", "std_mean_stress", "mean_local_stress", "std_local_stress",
                        "mean_edge_weight", "std_edge_weight"}
    m = models.EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=3, latent_size=128,
                                   input_nodes_features_size=6, output_nodes_features_size=3)
    epoch = models.load_model_checkpoint(m, (GOLDEN / "ref_checkpoint.pth").as_posix())
    assert epoch == 1
    sd = m.state_dict()
    assert set(sd) == set(raw["model_state_dict"])
    for k, v in raw["model_state_dict"].items():
        assert torch.equal(sd[k], v), k
    for k in ("mean_pos", "std_local_stress", "std_edge_weight"):
        assert torch.equal(torch.as_tensor(getattr(m, k)), raw[k])
    assert m.stats_tensor("cpu").shape == (8,)
    # the optimizer state is torch.optim.Adam's: one step taken, moments for every parameter
    opt = raw["optimizer_state_dict"]
    assert len(opt["state"]) == len(list(m.parameters()))
    assert all(float(s["step"]) == 1.0 for s in opt["state"].values())
    case = np.load(GOLDEN / "ref_checkpoint_case.npz", allow_pickle=False)
    assert float(case["loss_step2"]) < float(case["loss_step1"])
