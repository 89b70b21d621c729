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
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    lib = _lib.load()
    lib.subspace_crc_testutil_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.subspace_crc_testutil_probe_waves.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    lib.subspace_crc_testutil_probe_waves.restype = ctypes.c_uint64
    waves = int(lib.subspace_crc_testutil_probe_waves(ctx._h, N))
    ps, stride = slots.compute_prefix_size(4, 0), slots.slot_stride(SIZE, 4, 0)
    rng = np.random.default_rng(0x5EED0005)
    host = rng.integers(0, 256, stride * N, dtype=np.uint8)
    host.reshape(N, stride)[:, :ps] = slots.make_prefixes(N, np.full(N, SIZE, dtype=np.uint64), checksum_size=4,
                                                          metadata_size=0, seed=5)
    bufs = [torch.from_numpy(host).to(dev) for _ in range(NB)]
    for b in bufs:
        ctx.crc32_slots_strided(b, stride, N, message_size=SIZE, checksum_size=4, metadata_size=0,
                                mode=gpu.SLOT_CALCULATE)
    order = {"shuffled": rng.permutation(N).astype(np.uint64), "ordered": np.arange(N, dtype=np.uint64),
             "alias": np.zeros(N, dtype=np.uint64)}[a.order]
    recs = []
    for b in (bufs if a.order != "alias" else bufs[:1] * NB):
        b0 = np.uint64(b.data_ptr())
        r = np.stack([b0 + order * np.uint64(stride), b0 + order * np.uint64(stride) + np.uint64(ps),
                      np.full(N, SIZE, dtype=np.uint64)], axis=1)
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
        lib.subspace_crc_testutil_probe(ctx._h, rb.data_ptr())
        launch(a.settle + i)
    lib.subspace_crc_testutil_probe(ctx._h, None)
    torch.cuda.synchronize()
    per = {k: [] for k in STAMPS}
    dur = {"records": [], "fill": [], "loop": [], "flush": [], "tail": [], "total": []}
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
            if k == "tile0":
                continue
            per[k].append([pct((r[:, j] - t0) * TICK_US, q) for q in (0, 10, 50, 90, 100)])
        dur["records"].append(np.median((r[:, 1] - r[:, 0]) * TICK_US))
        dur["fill"].append(np.median((r[:, 2] - r[:, 1]) * TICK_US))
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
    out = {"order": a.order, "mode": a.mode, "launches": a.launches, "waves": waves, "fast_waves": fast,
           "stamp_us_p0_p10_p50_p90_p100": {k: np.median(np.array(v), axis=0).round(2).tolist()
                                             for k, v in per.items() if v},
           "median_wave_phase_us": {k: round(float(np.median(v)), 2) for k, v in dur.items()},
           "gap_to_next_launch_us": round(float(np.median(gaps)), 2) if gaps else None,
           "by_wave_in_wg_us": {k: np.median(np.array(v), axis=0).round(2).tolist() for k, v in by_wave.items()}}
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
