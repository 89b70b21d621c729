#!/usr/bin/env python3
"""Device-resident throughput of every BASELINE config through the production C ABI
(one JSON line per config). Not the driver's headline (that is bench.py, config B);
these are the secondary numbers recorded in DESIGN.md.

  C: 1 Mi ragged messages, 64 B - 1 MiB (~110 GiB), 64-B aligned packing (and --unaligned)
  D: 256 x 64 MiB
  E: one GPU's shard of 8 Mi x 4 KiB (1 Mi messages = 4 GiB, ids r, r+8, ...)
  S: config B in the reference's slot layout on the device (65,536 slots of prefix 64 B +
     4 KiB payload, stride 4,160; 4 rotated channel buffers), the full 3-span checksum
     (44-B prefix span + payload): publish (CALCULATE: flag + checksum written into every
     prefix) and subscriber verify (VERIFY: per-slot status + mismatch count)
The whole call (tile prep kernels + CRC kernel) is timed with HIP events, per call, after
>= 60 ms of warm-up calls; median and best of 21 calls are reported; every run is
checked against tests/golden/configs.json (CRC-list SHA-256) where the fixture covers it.
"""
import argparse
import hashlib
import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from subspace_amd import gpu, synth  # noqa: E402

GOLD = json.loads((ROOT / "tests" / "golden" / "configs.json").read_text())


def u64t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)


def timed(fn, iters, warm_ms=60.0, region=0):
    """Median and best ms per call over `iters` event-bracketed calls, after at least
    warm_ms of back-to-back warm-up calls (the GPU's first ~20 ms of sustained load after an
    idle spell run slower: profiles/r01/sustained.md). region > 0: each of the `iters`
    samples is one event pair around `region` back-to-back calls (per-call event pairs
    cost ~8 us, which matters for sub-0.1 ms calls), divided by `region`."""
    import time
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < warm_ms:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in evs:
        a.record()
        for _ in range(max(region, 1)):
            fn()
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) / max(region, 1) for a, b in evs)
    return ms[len(ms) // 2], ms[0]


def report(name, nbytes, ms_pair, crcs, gold_key, extra=None):
    ms, best = ms_pair
    ok = None
    if gold_key:
        ok = hashlib.sha256(crcs.astype("<u4").tobytes()).hexdigest() == GOLD[gold_key]["sha256_le_u32"]
    line = {"config": name, "bytes": int(nbytes), "ms": round(ms, 4), "GiBps": round(nbytes / ms / 1e-3 / 2**30, 1),
            "TBps": round(nbytes / ms / 1e9, 3), "ms_best": round(best, 4),
            "TBps_best": round(nbytes / best / 1e9, 3), "pct_of_8TBps": round(100 * nbytes / ms / 1e6 / 8000, 1),
            "bitexact_vs_golden": ok}
    if extra:
        line.update(extra)
    print(json.dumps(line), flush=True)


def slot_bench(ctx, dev, iters):
    """Config S (see the module docstring). Checked: after a publish, a verify of every slot
    reports no mismatch, and 64 sampled slots' stored checksums equal the host
    CalculateCRC32Checksum<3> over GetMessageChecksumData's spans (subspace_amd.checksum)."""
    from subspace_amd import checksum, slots
    n, size, cs, ms, nbuf = 65536, 4096, 4, 0, 4
    ps, stride = slots.compute_prefix_size(cs, ms), slots.slot_stride(size, cs, ms)
    rng = np.random.default_rng(0x5EED0005)
    host = rng.integers(0, 256, stride * n, dtype=np.uint8)
    host.reshape(n, stride)[:, :ps] = slots.make_prefixes(n, np.full(n, size, dtype=np.uint64), checksum_size=cs,
                                                          metadata_size=ms, seed=5)
    bufs = [torch.from_numpy(host).to(dev) for _ in range(nbuf)]
    status = torch.empty(n, dtype=torch.int32, device=dev)
    errs = torch.zeros(1, dtype=torch.int32, device=dev)
    nbytes = n * (size + 44)  # checksummed bytes: span 0 (44 B) + payload
    for mode, name in ((gpu.SLOT_CALCULATE, "S publish (CALCULATE)"), (gpu.SLOT_VERIFY, "S verify (VERIFY)")):
        i = [0]

        def call():
            b = bufs[i[0] % nbuf]
            i[0] += 1
            ctx.crc32_slots_strided(b, stride, n, message_size=size, checksum_size=cs, metadata_size=ms, mode=mode,
                                    status=status if mode == gpu.SLOT_VERIFY else None,
                                    error_count=errs if mode == gpu.SLOT_VERIFY else None)
        ms_pair = timed(call, iters, region=100)
        ok = None
        if mode == gpu.SLOT_VERIFY:
            torch.cuda.synchronize()
            ok = int(errs.item()) == 0 and bool((status == 0).all().item())
            chan = bufs[0].cpu().numpy()
            for k in rng.choice(n, 64, replace=False):
                pre = chan[k * stride:k * stride + ps]
                pay = chan[k * stride + ps:k * stride + ps + size]
                want = checksum.calculate_crc32_checksum(checksum.get_message_checksum_data(pre, pay, size, cs, ms))
                ok = ok and bytes(pre[48:52]) == want
        ms_v, best = ms_pair
        print(json.dumps({"config": name, "slots": n, "slot_stride": stride, "bytes": nbytes, "ms": round(ms_v, 4),
                          "GiBps": round(nbytes / ms_v / 1e-3 / 2**30, 1), "TBps": round(nbytes / ms_v / 1e9, 3),
                          "ms_best": round(best, 4), "pct_of_8TBps": round(100 * nbytes / ms_v / 1e6 / 8000, 1),
                          "verified": ok, "timing": "event pair around 100 back-to-back calls"}), flush=True)
    del bufs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C,D,E")
    ap.add_argument("--iters", type=int, default=21)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    for cfg in args.configs.split(","):
        if cfg in ("C", "Cu", "C16"):
            lengths = synth.ragged_lengths(synth.SEED_C, GOLD["C"]["count"])
            if cfg == "C16":  # probe (no fixture): every message end 16-B aligned
                lengths = lengths & ~np.uint64(15)
            offsets, total = synth.packed_offsets(lengths, 1 if cfg == "Cu" else 64)
            buf = torch.empty(total + 64, dtype=torch.uint8, device=dev)
            d_off, d_len = u64t(offsets, dev), u64t(lengths, dev)
            gpu.fill_ragged(buf, d_off, d_len, seed=synth.SEED_C)
            out = torch.empty(len(lengths), dtype=torch.int32, device=dev)
            ms = timed(lambda: ctx.crc32_ragged(buf, d_off, d_len, out), args.iters)
            name = {"C": "C", "Cu": "C unaligned", "C16": "C, lengths rounded to 16 B (probe)"}[cfg]
            report(name, int(lengths.sum()), ms, out.cpu().numpy().view(np.uint32), "C" if cfg != "C16" else None,
                   {"messages": len(lengths)})
            del buf, d_off, d_len, out
        elif cfg == "D":
            n, L = GOLD["D"]["count"], 64 << 20
            buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
            gpu.fill_uniform(buf, L, L, n, seed=synth.SEED_D)
            offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
            lens = np.full(n, L, dtype=np.uint64)
            d_off, d_len = u64t(offs, dev), u64t(lens, dev)
            out = torch.empty(n, dtype=torch.int32, device=dev)
            ms = timed(lambda: ctx.crc32_ragged(buf, d_off, d_len, out), args.iters)
            report("D", n * L, ms, out.cpu().numpy().view(np.uint32), "D", {"messages": n})
            ms_u = timed(lambda: ctx.crc32_uniform(buf, L, L, n, out), args.iters)
            report("D via batch_uniform (long-message kernel)", n * L, ms_u, out.cpu().numpy().view(np.uint32), "D")
            del buf, d_off, d_len, out
        elif cfg == "E":
            n, G = GOLD["E"]["count"], 8
            per = n // G
            buf = torch.empty(per * 4096, dtype=torch.uint8, device=dev)
            gpu.fill_uniform(buf, 4096, 4096, per, seed=synth.SEED_E, first_id=0, id_stride=G)
            out = torch.empty(per, dtype=torch.int32, device=dev)
            ms = timed(lambda: ctx.crc32_uniform(buf, 4096, 4096, per, out), args.iters)
            report("E shard (1 of 8)", per * 4096, ms, out.cpu().numpy().view(np.uint32), None,
                   {"messages": per})
            del buf, out
        elif cfg == "S":
            slot_bench(ctx, dev, args.iters)
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
