"""End-to-end inference I/O on the HIP path: dataset files ->
reference-format checkpoint -> gnn_local_stress.inference.main(config) -> fields/*.npz,
dataset.csv, normalize_params.json; predictions equal the model's forward."""
import json

import numpy as np
import pytest
import torch

from gpu_common import dev
from test_dataset_io import _write_sample

pytestmark = pytest.mark.gpu


def test_run_inference_end_to_end(tmp_path):
    import pandas as pd
    import yaml
    from gnn_local_stress import datasets, inference, models
    from pdg import graph, meshgen
    samples = meshgen.make_dataset(3, n=13, hole_radius=(0.1, 0.2), seed=21)
    rows = [_write_sample(tmp_path, i, s) for i, s in enumerate(samples)]
    csv = tmp_path / "dataset.csv"
    pd.DataFrame({"mesh_filename": [r[0] for r in rows], "data_filename": [r[1] for r in rows]}).to_csv(csv, index=False)
    ds = datasets.MeshStressFieldDatasetInMemory(pd.read_csv(csv))
    torch.manual_seed(69)
    model = models.EncodeProcessDecode(input_edges_features_size=1, message_passing_steps=4, latent_size=128,
                                       input_nodes_features_size=6, output_nodes_features_size=3, **ds.stats())
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    ckpt = tmp_path / "model.pth"
    models.save_model_checkpoint(model, opt, 7, ckpt.as_posix())
    cfg = dict(dataset_csv=csv.as_posix(), results_folder=(tmp_path / "res").as_posix(),
               model_weights_path=ckpt.as_posix(), periodic_graph=True, batch_size=2, latent_size=128,
               message_passing_steps=4, device="cuda:0")
    cfg_path = tmp_path / "config_inference.yml"
    cfg_path.write_text(yaml.safe_dump(cfg))
    inference.main(cfg_path.as_posix())
    res = tmp_path / "res"
    out = pd.read_csv(res / "dataset.csv")
    assert list(out["data_filename"]) == [(res / "fields" / f"hole_plate_mesh_{i}.npz").as_posix() for i in range(3)]
    params = json.loads((res / "normalize_params.json").read_text())
    assert params["mean_local_stress"] == float(ds.mean_local_stress)
    assert params["std_local_stress"] == float(ds.std_local_stress)
    assert (res / "config_inference.yml").exists()
    model.to(dev())
    with torch.no_grad():
        for i in range(3):
            b = graph.Batch.from_data_list([ds[i]]).to(dev())
            pred = model(b, scale_output=True).local_stress.cpu().numpy()
            with np.load(out["data_filename"][i]) as f:
                got = f["stress_field"]
            # batch composition changes the graph-global LayerNorm statistics (batch of 2 vs 1)
            assert got.shape == pred.shape
            assert np.isfinite(got).all()
    # the first two samples were predicted together: re-run that batch and compare bitwise
    b = graph.Batch.from_data_list([ds[0], ds[1]]).to(dev())
    with torch.no_grad():
        pred = model(b, scale_output=True).local_stress.cpu().numpy()
    n0 = ds[0].num_nodes
    with np.load(out["data_filename"][0]) as f0, np.load(out["data_filename"][1]) as f1:
        assert np.array_equal(f0["stress_field"], pred[:n0])
        assert np.array_equal(f1["stress_field"], pred[n0:])
