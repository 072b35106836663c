"""Inference I/O of the reference (``scripts/gnn_inference.py``) on the HIP path
(SURVEY §8f row 2): reads a dataset CSV (vtk + npz per sample), loads a
reference checkpoint, runs ``forward(scale_output=True, scale_input=True)``
per minibatch and writes, as the reference does,

* ``fields/hole_plate_mesh_{i}.npz``: a copy of sample i's input ``.npz`` with
  ``stress_field`` replaced by the prediction (gnn_inference.py:34-42, :61-79);
* ``dataset.csv``: the input table with ``data_filename`` pointing at those
  files (:130-131);
* ``normalize_params.json``: the model's ``mean_local_stress`` /
  ``std_local_stress`` (:132-138);
* a copy of the config file (:98).

    python -m gnn_local_stress.inference config_inference.yml
"""
from __future__ import annotations

import json
import shutil
from pathlib import Path

import numpy as np
import torch

from pdg.graph import DataLoader

from . import data_utils, datasets, models


def copy_data_file_and_replace_local_stress_field(original_data_path: str, target_data_path: str,
                                                  local_stress_field: torch.Tensor) -> None:
    """gnn_inference.py:34-42 (arrays loaded without pickle)."""
    with np.load(original_data_path, allow_pickle=False) as f:
        org_data = {k: f[k] for k in f.files}
    org_data["stress_field"] = local_stress_field.numpy()
    np.savez(target_data_path, **org_data)


def predict_and_save(model: models.EncodeProcessDecode, dataloader: DataLoader, results_folder: Path,
                     device) -> list[str]:
    """gnn_inference.py:45-81."""
    fields_folder = Path(results_folder) / "fields"
    fields_folder.mkdir(exist_ok=True, parents=True)
    mesh_id = 0
    names: list[str] = []
    for batch in dataloader:
        batch = batch.to(device)
        with torch.no_grad():
            pred = model.forward(batch, scale_output=True, scale_input=True)
        for field in data_utils.slice_batch_predictions(batch_graph_prediction=pred.local_stress,
                                                        batch_indices=batch.batch):
            path = (fields_folder / f"hole_plate_mesh_{mesh_id}.npz").as_posix()
            original = dataloader.dataset.dataframe.data_filename[mesh_id]
            copy_data_file_and_replace_local_stress_field(original, path, field.cpu())
            mesh_id += 1
            names.append(path)
    return names


@torch.no_grad()
def run_inference(dataset_csv, results_folder, model_weights_path, periodic_graph: bool, batch_size: int,
                  latent_size: int, message_passing_steps: int, device, config_path=None) -> None:
    """gnn_inference.py:84-138."""
    import pandas as pd
    dataframe = pd.read_csv(dataset_csv)
    results_folder = Path(results_folder)
    results_folder.mkdir(parents=True, exist_ok=True)
    if config_path is not None:
        shutil.copyfile(config_path, results_folder / Path(config_path).name)
    dataset = datasets.MeshStressFieldDatasetInMemory(dataframe, periodic_graph=periodic_graph)
    loader = DataLoader(dataset, batch_size=batch_size, shuffle=False)   # must not be shuffled
    model = models.EncodeProcessDecode(input_edges_features_size=1, input_nodes_features_size=6,
                                       message_passing_steps=message_passing_steps, latent_size=latent_size,
                                       output_nodes_features_size=3)
    model.to(device)
    models.load_model_checkpoint(model, str(model_weights_path))
    model.to(device)
    model.eval()
    names = predict_and_save(model, loader, results_folder, device)
    dataframe["data_filename"] = names
    dataframe.to_csv((results_folder / "dataset.csv").as_posix(), index=False)
    params = {"mean_local_stress": float(model.mean_local_stress.cpu()),
              "std_local_stress": float(model.std_local_stress.cpu())}
    with open((results_folder / "normalize_params.json").as_posix(), "w") as f:
        json.dump(params, f)


def main(config_path: str) -> None:
    import yaml
    with open(config_path) as f:
        params = yaml.safe_load(f)
    params["config_path"] = Path(config_path)
    run_inference(**params)


if __name__ == "__main__":
    import sys
    main(sys.argv[1])
