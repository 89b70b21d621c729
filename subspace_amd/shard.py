"""Multi-GPU sharding of independent messages (DESIGN.md "Multi-GPU").

Messages are independent, so a batch shards with no data-path exchange: rank r of a
world of G owns global message ids r, r + G, r + 2G, ... (round-robin, BASELINE config
E). The only collective is the optional gather of the 4-byte results to one rank
(an all_gather over RCCL on GPUs, gloo in the CPU tests), after which
`interleave` restores global message order.
"""
from __future__ import annotations

import numpy as np


def shard_count(count: int, rank: int, world: int) -> int:
    """Number of messages of a `count`-message batch owned by `rank`."""
    return (count - rank + world - 1) // world if rank < count else 0


def shard_ids(count: int, rank: int, world: int) -> np.ndarray:
    return np.arange(rank, count, world, dtype=np.uint64)


def interleave(shards: list[np.ndarray], count: int) -> np.ndarray:
    """Inverse of the round-robin split: shards[r][j] is global message r + j*world."""
    world = len(shards)
    out = np.empty(count, dtype=np.uint32)
    for r, s in enumerate(shards):
        out[r::world] = np.asarray(s, dtype=np.uint32)[:shard_count(count, r, world)]
    return out


def gather_crcs(local, count: int, rank: int, world: int, dist, dst: int = 0):
    """all_gather the per-rank CRC tensors (padded to equal length) and return the
    global-order numpy array on rank `dst` (None elsewhere). `local` is an int32 tensor."""
    import torch
    per = (count + world - 1) // world
    buf = torch.zeros(per, dtype=torch.int32, device=local.device)
    buf[:local.numel()] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    if rank != dst:
        return None
    return interleave([p.cpu().numpy().view(np.uint32) for p in parts], count)
