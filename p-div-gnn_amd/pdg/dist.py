"""Graph-batch data parallelism.

One process per GPU.  Every global minibatch of graphs (the reference's loader order,
gnn_train.py:387-394) is split into `world` shards, whole graphs only, balanced by node count;
every rank runs the full forward/backward on its shard and the flat fp32 gradient bucket is
SUMMED with one all-reduce (RCCL over xGMI on the GPU box, gloo in the CPU tests).

Loss weighting: every rank divides its graphs' losses by the GLOBAL minibatch's graph count B,
so each graph's gradient enters the sum with the reference's weight 1/B (gnn_train.py:193/196)
whichever rank it landed on, also for unequal shards (an odd minibatch, graphs of different
sizes, a last partial batch).  A rank that gets no graph contributes zeros.

LayerNorm statistics ("replica", the default): each graph-global LayerNorm is normalised over the
rank's own shard.  The reference normalises over the whole minibatch (models.py:42-55), so replica
DP equals one device only for B_local = B; Trainer(dp_mode="sync") exchanges the statistics and is
exact.
"""
from __future__ import annotations

import heapq
from typing import Sequence

import torch
import torch.distributed as dist


def shard_graphs(node_counts, world: int) -> list[list[int]]:
    """Deterministic greedy partition of graph indices into `world` shards
    balanced by total node count (largest graph first to the lightest shard)."""
    if world < 1:
        raise ValueError("world must be >= 1")
    order = sorted(range(len(node_counts)), key=lambda i: (-int(node_counts[i]), i))
    heap = [(0, r) for r in range(world)]
    shards: list[list[int]] = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        shards[r].append(i)
        heapq.heappush(heap, (load + int(node_counts[i]), r))
    return [sorted(s) for s in shards]


def shard_minibatch(indices: Sequence[int], node_counts: Sequence[int], world: int, rank: int) -> list[int]:
    """This rank's graphs of one global minibatch: `indices` are the dataset indices the reference's
    loader yields (in its order), `node_counts[i]` the size of dataset graph i.  The shards of all
    ranks partition `indices`; each keeps the loader's relative order."""
    pos = shard_graphs([node_counts[i] for i in indices], world)[rank]
    return [int(indices[p]) for p in pos]


def sync_shardable(indices: Sequence[int], store, world: int) -> bool:
    """Whether every rank's ``shard_minibatch`` share of one minibatch has a graph with edges, as the
    exact dp_mode="sync" LayerNorm exchange needs (every rank joins every statistic collective).
    ``store``: per-graph node counts ``n`` and edge counts ``e`` (pdg.collate.DeviceGraphStore)."""
    if len(indices) < world:
        return False
    shards = shard_graphs([store.n[i] for i in indices], world)
    return all(sum(int(store.e[indices[p]]) for p in sh) > 0 for sh in shards)


def allreduce_sum_(flat: torch.Tensor, group=None) -> torch.Tensor:
    """In-place sum of a flat bucket over the process group (one collective)."""
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    return flat


def allreduce_mean_(flat: torch.Tensor, group=None) -> torch.Tensor:
    """In-place mean of a flat bucket over the process group (one collective)."""
    if not dist.is_available() or not dist.is_initialized():
        return flat
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat.mul_(1.0 / dist.get_world_size(group))
    return flat


def flatten(tensors) -> torch.Tensor:
    return torch.cat([t.reshape(-1) for t in tensors])
