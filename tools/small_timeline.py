#!/usr/bin/env python3
"""Per-wave timeline of the small-message kernel over config S's channel as a device slot list
(investigation tool; the kernel's experiment hook, subspace_crc_testutil_probe: realtime-clock
stamps per wave at entry, when the window's records had landed, after the LDS fill + barrier,
at the tile loop's end, after the flush, at exit).

Runs back-to-back verify calls over four rotated channel copies (shuffled or ordered lists)
after a settle, the last `--launches` of them with the probe on (each its own record buffer),
and prints, as medians over launches, the percentiles over waves of each stamp relative to the
launch's first entry, and per-wave phase durations. Clock: s_memrealtime, 100 MHz.

  python tools/small_timeline.py [--launches 20] [--order shuffled|ordered] [--mode verify|publish]
                                 [--sizes 4096|256|mixed]
--sizes: the channel's messages -- 4096 (config S), 256 (S_short: 256-B messages in the 4 KiB
slots) or mixed (S_mixed: 1 .. 4,096 B uniformly random); the slot list's max_message_size is
4,096 for all. With the repack loop (S_short, S_mixed) the record also carries each wave's
packed tile count (rnt), and the output relates it to the wave's loop time.
"""
import argparse
import ctypes
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import _lib, gpu, slots  # noqa: E402

N, SIZE, NB, WORDS, TICK_US = 65536, 4096, 4, 8, 0.01
STAMPS = ("entry", "records", "barrier", "tile0", "loop_end", "flush_end", "exit")


def pct(a, q):
    return round(float(np.percentile(a, q)), 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--settle", type=int, default=600)
    ap.add_argument("--order", default="shuffled", choices=["shuffled", "ordered", "alias"],
                    help="alias: every record points at slot 0 of copy 0 (the compute-only run)")
    ap.add_argument("--mode", default="verify", choices=["verify", "publish"])
    ap.add_argument("--sizes", default="4096", help="4096, 256 or any fixed size <= 4096, or mixed")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    lib = _lib.load()
    waves = int(_lib.load_dev().subspace_crc_testutil_probe_waves(ctx._h, N))
    ps, stride = slots.compute_prefix_size(4, 0), slots.slot_stride(SIZE, 4, 0)
    rng = np.random.default_rng(0x5EED0005)
    sizes = (rng.integers(1, SIZE + 1, N).astype(np.uint64) if a.sizes == "mixed"
             else np.full(N, int(a.sizes), dtype=np.uint64))
    host = rng.integers(0, 256, stride * N, dtype=np.uint8)
    host.reshape(N, stride)[:, :ps] = slots.make_prefixes(N, sizes, checksum_size=4, metadata_size=0, seed=5)
    bufs = [torch.from_numpy(host).to(dev) for _ in range(NB)]
    d_sizes = torch.from_numpy(sizes.view(np.int64)).to(dev)
    for b in bufs:
        ctx.crc32_slots_strided(b, stride, N, sizes=d_sizes, checksum_size=4, metadata_size=0,
                                mode=gpu.SLOT_CALCULATE)
    order = {"shuffled": rng.permutation(N).astype(np.uint64), "ordered": np.arange(N, dtype=np.uint64),
             "alias": np.zeros(N, dtype=np.uint64)}[a.order]
    recs = []
    for b in (bufs if a.order != "alias" else bufs[:1] * NB):
        b0 = np.uint64(b.data_ptr())
        r = np.stack([b0 + order * np.uint64(stride), b0 + order * np.uint64(stride) + np.uint64(ps),
                      sizes[order.astype(np.int64)]], axis=1)
        recs.append(torch.from_numpy(np.ascontiguousarray(r).view(np.int64)).to(dev))
    status = torch.empty(N, dtype=torch.int32, device=dev)
    errs = torch.zeros(1, dtype=torch.int32, device=dev)
    mode = gpu.SLOT_VERIFY if a.mode == "verify" else gpu.SLOT_CALCULATE

    def launch(i):
        ctx.crc32_slots(recs[i % NB], max_message_size=SIZE, checksum_size=4, metadata_size=0, mode=mode,
                        status=status, error_count=errs if mode == gpu.SLOT_VERIFY else None)

    for i in range(a.settle):
        launch(i)
    rec_bufs = [torch.zeros(waves * WORDS, dtype=torch.int64, device=dev) for _ in range(a.launches)]
    torch.cuda.synchronize()
    for i, rb in enumerate(rec_bufs):
        _lib.load_dev().subspace_crc_testutil_probe(ctx._h, rb.data_ptr())
        launch(a.settle + i)
    _lib.load_dev().subspace_crc_testutil_probe(ctx._h, None)
    torch.cuda.synchronize()
    per = {k: [] for k in STAMPS}
    dur = {"records": [], "fill": [], "tile0": [], "loop": [], "flush": [], "tail": [], "total": []}
    gaps = []
    prev_exit = None
    for rb in rec_bufs:
        r = rb.cpu().numpy().view(np.uint64).reshape(waves, WORDS).astype(np.int64)
        live = r[:, 0] > 0
        r = r[live]
        t0 = r[:, 0].min()
        if prev_exit is not None:
            gaps.append((t0 - prev_exit) * TICK_US)
        prev_exit = r[:, 6].max()
        for j, k in enumerate(STAMPS):
            per[k].append([pct((r[:, j] - t0) * TICK_US, q) for q in (0, 10, 50, 90, 100)])
        dur["records"].append(np.median((r[:, 1] - r[:, 0]) * TICK_US))
        dur["fill"].append(np.median((r[:, 2] - r[:, 1]) * TICK_US))
        dur["tile0"].append(np.median((r[:, 3] - r[:, 2]) * TICK_US))
        dur["loop"].append(np.median((r[:, 4] - r[:, 2]) * TICK_US))
        dur["flush"].append(np.median((r[:, 5] - r[:, 4]) * TICK_US))
        dur["tail"].append(np.median((r[:, 6] - r[:, 5]) * TICK_US))
        dur["total"].append((r[:, 6].max() - t0) * TICK_US)
    fast = int(((rec_bufs[-1].cpu().numpy().view(np.uint64).reshape(waves, WORDS)[:, 7] >> 48) & 1).sum())
    by_wave = {"loop_end": [], "exit": []}  # medians over launches of each wave-in-workgroup's median
    for rb in rec_bufs:
        r = rb.cpu().numpy().view(np.uint64).reshape(waves, WORDS).astype(np.int64)
        t0 = r[r[:, 0] > 0, 0].min()
        w = np.arange(waves) % 8
        by_wave["loop_end"].append([np.median((r[w == i, 4] - t0) * TICK_US) for i in range(8)])
        by_wave["exit"].append([np.median((r[w == i, 6] - t0) * TICK_US) for i in range(8)])
    # the repack loop's packed tiles per wave (record word 7 bits 52..) against the wave's loop time
    last = rec_bufs[-1].cpu().numpy().view(np.uint64).reshape(waves, WORDS)
    rnt = ((last[:, 7] >> 52) & 0xFFF).astype(np.int64)
    nk = ((last[:, 7] >> 32) & 0xFFFF).astype(np.int64)
    lr = last.astype(np.int64)
    loop_us = (lr[:, 4] - lr[:, 2]) * TICK_US
    live = lr[:, 0] > 0
    rep = {}
    if (rnt[live] > 0).any():
        t0l = lr[live, 0].min()
        rep = {"rnt_p0_p50_p100": [int(np.percentile(rnt[live], q)) for q in (0, 50, 100)],
               "nk_p50": int(np.median(nk[live])),
               "loop_us_by_rnt": {int(v): round(float(np.median(loop_us[live & (rnt == v)])), 2)
                                  for v in np.unique(rnt[live])},
               "flush_end_us_by_rnt": {int(v): round(float(np.median((lr[live & (rnt == v), 5] - t0l) * TICK_US)), 2)
                                       for v in np.unique(rnt[live])},
               # the two waves of a SIMD (wave slots w, w + 4 of a workgroup: front_slot pairs)
               "simd_pair_tiles_p50_p100": [int(np.percentile((rnt.reshape(-1, 8)[:, :4] + rnt.reshape(-1, 8)[:, 4:]), q))
                                            for q in (50, 100)],
               "cu_tiles_p50_p100": [int(np.percentile(rnt.reshape(-1, 8).sum(1), q)) for q in (50, 100)]}
    # the last waves to exit in the last launch: their workgroup, wave, XCC and every stamp
    t0l = lr[lr[:, 0] > 0, 0].min()
    order_exit = np.argsort(-(lr[:, 6] * (lr[:, 0] > 0)))[:6]
    slowest = [{"wg": int(w // 8), "wave": int(w % 8), "xcc": int(last[w, 7] & 0xFF),
                "stamps_us": [round(float((lr[w, i] - t0l) * TICK_US), 2) for i in range(7)]} for w in order_exit]
    out = {"order": a.order, "mode": a.mode, "sizes": a.sizes, "launches": a.launches, "waves": waves,
           "slowest_waves_last_launch": slowest,
           "fast_waves": fast, "repack": rep,
           "stamp_us_p0_p10_p50_p90_p100": {k: np.median(np.array(v), axis=0).round(2).tolist()
                                             for k, v in per.items() if v},
           "median_wave_phase_us": {k: round(float(np.median(v)), 2) for k, v in dur.items()},
           "gap_to_next_launch_us": round(float(np.median(gaps)), 2) if gaps else None,
           "by_wave_in_wg_us": {k: np.median(np.array(v), axis=0).round(2).tolist() for k, v in by_wave.items()}}
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
