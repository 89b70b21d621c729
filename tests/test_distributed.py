"""World-size-2 gloo test of the multi-GPU sharding path (CPU).

Each rank checksums its round-robin shard of a synthetic 4 KiB batch with the product
host SubspaceCRC32 (the GPU kernel is covered by tests/test_gpu_parity.py), the shards
are all_gathered with subspace_amd.shard.gather_crcs exactly as bench.py does over RCCL,
and rank 0 compares the global-order list with the oracle.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

COUNT, SEED = 1001, 0x5EED000E


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        from pathlib import Path
        sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
        from subspace_amd import checksum, shard, synth
        ids = shard.shard_ids(COUNT, rank, world)
        assert len(ids) == shard.shard_count(COUNT, rank, world)
        local = np.array([checksum.subspace_crc32(0xFFFFFFFF, synth.synth_bytes(SEED, int(i), 4096)) for i in ids],
                         dtype=np.uint32)
        t = torch.from_numpy(local.view(np.int32).copy())
        full = shard.gather_crcs(t, COUNT, rank, world, dist)
        # timing reduction used by bench.py: max over ranks
        el = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        if rank == 0:
            result_q.put((full, float(el.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_round_robin_shards_gather_to_global_order(world, oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, maxel = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = oracle.synth_crc_batch(SEED, np.full(COUNT, 4096, dtype=np.uint64))
    assert np.array_equal(full, want)
    assert maxel == float(world)


RAGGED_SEED = 0x5EED000C


def _ragged_worker(rank, world, port, lengths, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        from pathlib import Path
        sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
        from subspace_amd import checksum, shard, synth
        b = shard.ragged_ranges(lengths, world)
        local = np.array([checksum.subspace_crc32(0xFFFFFFFF, synth.synth_bytes(RAGGED_SEED, i, int(lengths[i])))
                          for i in range(b[rank], b[rank + 1])], dtype=np.uint32)
        t = torch.from_numpy(local.view(np.int32).copy())
        full = shard.gather_ragged_crcs(t, b, rank, world, dist)
        if rank == 0:
            result_q.put(full)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ragged_contiguous_shards_gather_to_global_order(world, oracle):
    """Config C's sharding: contiguous message ranges balanced by bytes, one ragged call
    per rank, CRCs gathered (padded all_gather) and concatenated in rank order."""
    from subspace_amd import synth
    lengths = (synth.ragged_lengths(RAGGED_SEED, 300) // np.uint64(16)).astype(np.uint64)
    lengths[::29] = 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ragged_worker, args=(r, world, port, lengths, q)) for r in range(world)]
    for p in procs:
        p.start()
    full = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(full, oracle.synth_crc_batch(RAGGED_SEED, lengths))


def test_ragged_ranges_balance_bytes():
    from subspace_amd import shard, synth
    lengths = synth.ragged_lengths(RAGGED_SEED, 20000)
    total, longest = int(lengths.sum()), int(lengths.max())
    for world in (1, 2, 3, 4, 8):
        b = shard.ragged_ranges(lengths, world)
        assert b[0] == 0 and b[-1] == len(lengths) and np.all(np.diff(b) >= 0)
        per = [int(lengths[b[r]:b[r + 1]].sum()) for r in range(world)]
        assert sum(per) == total
        assert max(abs(x - total / world) for x in per) < longest
    # more ranks than messages, empty messages, empty batch
    b = shard.ragged_ranges(np.array([5, 0, 7], dtype=np.uint64), 8)
    assert b[0] == 0 and b[-1] == 3 and np.all(np.diff(b) >= 0)
    assert list(shard.ragged_ranges(np.array([], dtype=np.uint64), 2)) == [0, 0, 0]
    got = shard.concat_ranges([np.array([1, 2]), np.array([], dtype=np.uint32), np.array([3])], [0, 2, 2, 3])
    assert list(got) == [1, 2, 3]


def test_interleave_roundtrip():
    from subspace_amd import shard
    for count in (1, 7, 8, 9, 1000):
        for world in (1, 2, 3, 8):
            g = np.arange(count, dtype=np.uint32) * 7 + 3
            parts = [g[r::world] for r in range(world)]
            assert np.array_equal(shard.interleave(parts, count), g)
            assert sum(shard.shard_count(count, r, world) for r in range(world)) == count
