"""Graph-batch data parallelism.

One process per GPU.  A global minibatch of graphs is split into `world`
shards, whole graphs only, balanced by node count; every rank runs the full
forward/backward on its shard and the flat fp32 gradient bucket is averaged
with one all-reduce (RCCL over xGMI on the GPU box, gloo in the CPU tests).

Semantics ("replica", the default): each shard is normalised as its own batch
(the loss is divided by the local batch size, gnn_train.py:193/196, and the
graph-global LayerNorm statistics are those of the shard), and the gradients
are averaged.  For equal shards this is the mean over shards of the gradient
each shard would produce alone, which is what the tests check.  (The
reference's LayerNorm normalises over the whole minibatch, so DP over B graphs
equals one device over B graphs only for B_local = B; DESIGN.md.)
"""
from __future__ import annotations

import heapq

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


def allreduce_mean_(flat: torch.Tensor, group=None) -> torch.Tensor:
    """In-place mean of a flat gradient bucket over the process group (one collective)."""
    if not dist.is_available() or not dist.is_initialized():
        return flat
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat.mul_(1.0 / dist.get_world_size(group))
    return flat


def flatten(tensors) -> torch.Tensor:
    return torch.cat([t.reshape(-1) for t in tensors])
