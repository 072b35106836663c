"""Drop-in ``gnn_local_stress.data_utils`` (reference gnn_local_stress/data_utils.py:25-59)."""
from __future__ import annotations

from typing import Generator

import torch


def slice_batch_gt_and_predictions(mesh_graph_batch, prediction: torch.Tensor) -> Generator:
    """data_utils.py:25-33 — per-graph (Data, prediction) pairs of a batch."""
    for i in range(len(mesh_graph_batch)):
        mesh_graph_i = mesh_graph_batch[i]
        yield mesh_graph_i, prediction[mesh_graph_batch.batch.to(prediction.device) == i]


def slice_batch_predictions(batch_graph_prediction: torch.Tensor, batch_indices: torch.Tensor) -> Generator:
    """data_utils.py:36-43."""
    for i in range(len(torch.unique(batch_indices))):
        yield batch_graph_prediction[batch_indices == i]


def standardize(data: torch.Tensor, mean, std) -> torch.Tensor:
    """data_utils.py:46-51."""
    return (data - mean) / std


def unstandardize(data: torch.Tensor, mean, std) -> torch.Tensor:
    """data_utils.py:54-59."""
    return (data * std) + mean
