"""Multi-GPU sharding of independent messages (DESIGN.md "Multi-GPU").

Messages are independent, so a batch shards with no data-path exchange: rank r of a
world of G owns global message ids r, r + G, r + 2G, ... (round-robin, BASELINE config
E). Ragged batches (config C) shard instead into contiguous message ranges balanced by
byte count, so each rank's slice of the offset/length arrays is one
subspace_crc32_batch call. The only collective is the optional gather of the 4-byte
results to one rank (an all_gather over RCCL on GPUs, gloo in the CPU tests), after
which `interleave` (round-robin) or `concat_ranges` (contiguous) restores global
message order.
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


def ragged_ranges(lengths, world: int) -> np.ndarray:
    """Contiguous shard boundaries of a ragged batch, balanced by bytes: rank r owns
    messages [b[r], b[r+1]). b[r] is the first message whose start (the byte count before
    it) reaches r/world of the total, so every rank's bytes differ from total/world by
    less than the longest message. Returns world + 1 boundaries (b[0] = 0, b[world] = count)."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    if world < 1:
        raise ValueError("world must be >= 1")
    # bytes before message i; built from a uint64 zero so it stays uint64 end to end
    # (np.concatenate of a Python-int list with uint64 promotes to float64)
    starts = np.concatenate([np.zeros(1, dtype=np.uint64), np.cumsum(lengths, dtype=np.uint64)])
    total = int(starts[-1])
    targets = [(total * r + world - 1) // world for r in range(world)]  # ceil(total*r/world)
    b = np.searchsorted(starts[:-1], np.array(targets, dtype=np.uint64), side="left").astype(np.int64)
    b[0] = 0
    return np.concatenate([b, [len(lengths)]]).astype(np.int64)


def concat_ranges(shards: list[np.ndarray], bounds) -> np.ndarray:
    """Inverse of the contiguous split: shards[r] holds messages [bounds[r], bounds[r+1])."""
    out = np.empty(int(bounds[-1]), dtype=np.uint32)
    for r, s in enumerate(shards):
        n = int(bounds[r + 1] - bounds[r])
        out[bounds[r]:bounds[r + 1]] = np.asarray(s, dtype=np.uint32)[:n]
    return out


def gather_ragged_crcs(local, bounds, rank: int, world: int, dist, dst: int = 0):
    """all_gather the per-rank CRC tensors of a contiguous (ragged) split, padded to the
    largest shard, and return the global-order numpy array on rank `dst` (None elsewhere)."""
    import torch
    per = int(max(bounds[r + 1] - bounds[r] for r in range(world)))
    buf = torch.zeros(max(per, 1), dtype=torch.int32, device=local.device)
    buf[:local.numel()] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    if rank != dst:
        return None
    return concat_ranges([p.cpu().numpy().view(np.uint32) for p in parts], bounds)


# ---------------------------------------------------------------- device-resident gathers
def gather_crcs_device(local, count: int, world: int, dist):
    """all_gather the per-rank CRC tensors (padded to equal length) and interleave them into
    global order ON THE DEVICE (every rank gets the full int32 tensor; no host copy). Without
    a process group (dist None) it is one device copy of the local results."""
    import torch
    per = (count + world - 1) // world
    buf = torch.zeros(per, dtype=torch.int32, device=local.device)
    buf[:min(local.numel(), per)] = local[:per]
    if dist is None:
        return buf[:count].clone()
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    # parts[r][j] is global message r + j*world: the (world, per) stack read column-major
    return torch.stack(parts).t().contiguous().view(-1)[:count]


def gather_ragged_crcs_device(local, bounds, world: int, dist):
    """all_gather of a contiguous (ragged) split, padded to the largest shard, concatenated in
    rank order on the device (every rank gets the full int32 tensor)."""
    import torch
    per = int(max(bounds[r + 1] - bounds[r] for r in range(world)))
    buf = torch.zeros(max(per, 1), dtype=torch.int32, device=local.device)
    buf[:local.numel()] = local
    if dist is None:
        return buf[:int(bounds[1])].clone()
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    return torch.cat([parts[r][:int(bounds[r + 1] - bounds[r])] for r in range(world)])
