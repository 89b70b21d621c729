#!/usr/bin/env python3
"""Throughput of the small-message kernel by message size (investigation tool): uniform batches
of n messages of L bytes (stride = L rounded up to 16 B) through subspace_crc32_batch_uniform,
event-timed over `launches` back-to-back calls after `settle` untimed ones, rotated over buffers
large enough to leave the 256 MB MALL behind.

  python tools/small_sizes.py [L,L,...] [launches] [settle] [uniform|uniform_packed|slots|slots_ordered|slots4k|slots4k_rand|ragged_rand]

slots: a channel of L-byte slots (MessagePrefix 64 B + payload, the reference's stride) per
256 MiB, published once, then verified as shuffled device slot lists (subspace_crc32_slots,
max_message_size = L) over four rotated copies; GB/s counts span 0 (44 B) + payload. slots4k:
L-byte messages in a channel of 4 KiB slots (max_message_size 4096); slots4k_rand: message
sizes uniform in [1, L] in 4 KiB slots. ragged_rand: a ragged batch (subspace_crc32_batch) of
messages uniform in [1, L] bytes packed back to back (any alignment), 256 MiB per batch, four
rotated.
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import numpy as np  # noqa: E402

from subspace_amd import gpu, slots  # noqa: E402


def main():
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "64,256,1024,2048,4000").split(",")]
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    settle = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    mode = sys.argv[4] if len(sys.argv) > 4 else "uniform"  # uniform | slots | slots_ordered | slots4k
    ctx = gpu.CrcContext(0)
    dev = torch.device("cuda", 0)
    if mode == "ragged_rand":
        return ragged_rand(ctx, dev, sizes, launches, settle)
    if mode.startswith("slots"):
        return slot_lists(ctx, dev, sizes, launches, settle, ordered=mode == "slots_ordered",
                          slot_size=4096 if mode.startswith("slots4k") else 0, rand=mode == "slots4k_rand")
    for L in sizes:
        stride = L if mode == "uniform_packed" else (L + 15) & ~15
        n = (256 << 20) // stride  # 256 MiB of messages per batch
        nb = 4
        bufs = [torch.empty(n * stride, dtype=torch.uint8, device=dev) for _ in range(nb)]
        for k, b in enumerate(bufs):
            gpu.fill_uniform(b, stride, L, n, seed=0x5153 + k)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        for i in range(settle):
            ctx.crc32_uniform(bufs[i % nb], stride, L, n, out)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(launches):
            ctx.crc32_uniform(bufs[i % nb], stride, L, n, out)
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / launches
        print(json.dumps({"length": L, "stride": stride, "messages": n, "us_per_call": round(us, 2),
                          "GBps": round(n * L / us / 1e3, 1), "Gmsg_per_s": round(n / us / 1e3, 3),
                          "pct_of_hbm_peak": round(100 * n * L / us / 1e3 / 8000, 2)}), flush=True)
        del bufs, out  # (no empty_cache: VRAM handed back is wiped in the background)
    ctx.close()


def ragged_rand(ctx, dev, sizes, launches, settle):
    rng = np.random.default_rng(0x5154)
    for L in sizes:
        n = (256 << 20) // ((L + 1) // 2)
        lens = rng.integers(1, L + 1, n).astype(np.uint64)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        total = int(lens.sum())
        bufs = [torch.randint(0, 256, (total + 64,), dtype=torch.uint8, device=dev) for _ in range(4)]
        d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
        d_len = torch.from_numpy(lens.view(np.int64)).to(dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        for i in range(settle):
            ctx.crc32_ragged(bufs[i % 4], d_off, d_len, out)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(launches):
            ctx.crc32_ragged(bufs[i % 4], d_off, d_len, out)
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / launches
        print(json.dumps({"ragged_max": L, "messages": n, "bytes": total, "us_per_call": round(us, 2),
                          "GBps": round(total / us / 1e3, 1), "Gmsg_per_s": round(n / us / 1e3, 3),
                          "pct_of_hbm_peak": round(100 * total / us / 1e3 / 8000, 2)}), flush=True)
        del bufs, out
    ctx.close()


def slot_lists(ctx, dev, sizes, launches, settle, ordered=False, slot_size=0, rand=False):
    """slot_size: the channel's slot size (max_message_size); 0: each message fills its slot.
    rand: message sizes uniform in [1, L]."""
    rng = np.random.default_rng(0x5153)
    for L in sizes:
        cs, ms = 4, 0
        area = slot_size or L
        ps, stride = slots.compute_prefix_size(cs, ms), slots.slot_stride(area, cs, ms)
        n = (256 << 20) // stride
        msz = rng.integers(1, L + 1, n).astype(np.uint64) if rand else np.full(n, L, dtype=np.uint64)
        host = rng.integers(0, 256, stride * n, dtype=np.uint8)
        host.reshape(n, stride)[:, :ps] = slots.make_prefixes(n, msz, checksum_size=cs, metadata_size=ms, seed=5)
        bufs = [torch.from_numpy(host).to(dev) for _ in range(4)]
        for b in bufs:
            ctx.crc32_slots_strided(b, stride, n, sizes=torch.from_numpy(msz.view(np.int64)).to(dev),
                                    checksum_size=cs, metadata_size=ms, mode=gpu.SLOT_CALCULATE)
        order = np.arange(n, dtype=np.uint64) if ordered else rng.permutation(n).astype(np.uint64)
        recs = []
        for b in bufs:
            b0 = np.uint64(b.data_ptr())
            r = np.stack([b0 + order * np.uint64(stride), b0 + order * np.uint64(stride) + np.uint64(ps),
                          msz[order.astype(np.int64)]], axis=1)
            recs.append(torch.from_numpy(np.ascontiguousarray(r).view(np.int64)).to(dev))
        status = torch.empty(n, dtype=torch.int32, device=dev)
        errs = torch.zeros(1, dtype=torch.int32, device=dev)

        def one(i):
            ctx.crc32_slots(recs[i % 4], max_message_size=area, checksum_size=cs, metadata_size=ms,
                            mode=gpu.SLOT_VERIFY, status=status, error_count=errs)
        for i in range(settle):
            one(i)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(launches):
            one(i)
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / launches
        ok = int(errs.item()) == 0 and bool((status == 0).all().item())
        nbytes = int(msz.sum()) + 44 * n
        print(json.dumps({"order": "channel" if ordered else "shuffled", "slot_area": area,
                          "message": f"1..{L}" if rand else L, "stride": stride, "slots": n, "us_per_call": round(us, 2),
                          "GBps": round(nbytes / us / 1e3, 1), "Gslots_per_s": round(n / us / 1e3, 3),
                          "pct_of_hbm_peak": round(100 * nbytes / us / 1e3 / 8000, 2), "all_pass": ok}), flush=True)
        del bufs, recs, status
    ctx.close()


if __name__ == "__main__":
    main()
