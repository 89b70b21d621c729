#!/usr/bin/env python3
"""Per-wave timeline of the config-B uniform launch, or of config S through the fused slot
kernel (the kernel's PROBE instantiation: realtime-clock stamps at entry, after the table and
tile-0 loads were issued, after the LDS fill + barrier, when tile 0 had landed, after the tile
loop, before the last slot flush, at exit).

Runs back-to-back config-B launches (4 rotated 256 MiB batches) after the power-management
settle, the last `--launches` of them with the probe on (each its own record buffer), and
prints, per launch and as medians over launches: dispatch ramp (entry spread), fill time,
loop time, tail (loop end -> exit), the exit spread, per-XCD exit times and the gap between a
launch's last exit and the next launch's first entry. Clock: s_memrealtime, 100 MHz.
"""
import argparse
import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import _lib, gpu, slots  # noqa: E402

N, SIZE, NBUF, WORDS, TICK_US = 65536, 4096, 4, 8, 0.01


def pct(a, q):
    return round(float(np.percentile(a, q)), 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--settle", type=int, default=600)
    ap.add_argument("--out", default=None, help="write the raw records (npz)")
    ap.add_argument("--mode", default="uniform", choices=["uniform", "uniform4160", "publish", "verify"],
                    help="config B (uniform kernel), config S's payloads through the uniform kernel, "
                         "or config S through the fused slot kernel")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    lib = _lib.load()
    _lib.load_dev().subspace_crc_testutil_probe.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    _lib.load_dev().subspace_crc_testutil_probe_waves.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    _lib.load_dev().subspace_crc_testutil_probe_waves.restype = ctypes.c_uint64
    waves = int(_lib.load_dev().subspace_crc_testutil_probe_waves(ctx._h, N))
    out = torch.empty(N, dtype=torch.int32, device=dev)
    errs = torch.zeros(1, dtype=torch.int32, device=dev)
    if a.mode == "uniform":
        bufs = [torch.empty(N * SIZE, dtype=torch.uint8, device=dev) for _ in range(NBUF)]
        for k, b in enumerate(bufs):
            gpu.fill_uniform(b, SIZE, SIZE, N, seed=0x5EED000B, first_id=k * N)

        def launch(b, res):
            ctx.crc32_uniform(b, SIZE, SIZE, N, res)
    else:  # config S: PrefixSize 64 + 4 KiB payload per slot, stride 4,160
        ps, stride = slots.compute_prefix_size(4, 0), slots.slot_stride(SIZE, 4, 0)
        host = np.random.default_rng(7).integers(0, 256, stride * N, dtype=np.uint8)
        host.reshape(N, stride)[:, :ps] = slots.make_prefixes(N, np.full(N, SIZE, dtype=np.uint64),
                                                              checksum_size=4, metadata_size=0, seed=5)
        bufs = [torch.from_numpy(host).to(dev) for _ in range(NBUF)]
        for b in bufs:  # valid stored checksums, so verify passes
            ctx.crc32_slots_strided(b, stride, N, message_size=SIZE, mode=gpu.SLOT_CALCULATE)

        def launch(b, res):
            if a.mode == "uniform4160":  # the payloads of config S through the plain uniform kernel
                ctx.crc32_uniform(b, stride, SIZE, N, res, base_offset=ps)
            elif a.mode == "publish":
                ctx.crc32_slots_strided(b, stride, N, message_size=SIZE, mode=gpu.SLOT_CALCULATE)
            else:
                ctx.crc32_slots_strided(b, stride, N, message_size=SIZE, mode=gpu.SLOT_VERIFY, status=res,
                                        error_count=errs)
    rec = torch.zeros((a.launches, waves, WORDS), dtype=torch.int64, device=dev)
    ref = torch.empty(N, dtype=torch.int32, device=dev)
    launch(bufs[0], ref)
    torch.cuda.synchronize()
    for i in range(a.settle):
        launch(bufs[i % NBUF], out)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for i in range(a.launches):
        _lib.load_dev().subspace_crc_testutil_probe(ctx._h, ctypes.c_void_p(rec[i].data_ptr()))
        launch(bufs[(a.settle + i) % NBUF], out)
    ev1.record()
    _lib.load_dev().subspace_crc_testutil_probe(ctx._h, None)
    torch.cuda.synchronize()
    span_ms = ev0.elapsed_time(ev1) / a.launches
    # the probe launch computes the same results
    _lib.load_dev().subspace_crc_testutil_probe(ctx._h, ctypes.c_void_p(rec[0].data_ptr()))
    launch(bufs[0], out)
    _lib.load_dev().subspace_crc_testutil_probe(ctx._h, None)
    torch.cuda.synchronize()
    check = not os.environ.get("SLOT_GAP_NOCHECK")  # (timing-only builds compute nothing valid)
    if a.mode != "publish" and check:
        assert torch.equal(out, ref), "PROBE instantiation results differ"
    if a.mode in ("uniform", "uniform4160"):
        _lib.load_dev().subspace_crc_testutil_probe(ctx._h, None)
    assert int(errs.item()) == 0 or not check
    r = rec.cpu().numpy()[1:]  # launch 0 was overwritten by the check above
    if a.out:
        np.savez_compressed(a.out, rec=r)
    rows = []
    for i in range(r.shape[0]):
        t = r[i, :, :4].astype(np.float64) * TICK_US
        base = t[:, 0].min()
        t -= base
        xcc = r[i, :, 5] & 0xF
        row = {
            "launch": i + 1,
            "entry_p50": pct(t[:, 0], 50), "entry_max": pct(t[:, 0], 100),
            "fill_p50": pct(t[:, 1] - t[:, 0], 50), "fill_max": pct(t[:, 1] - t[:, 0], 100),
            "issued_p50": pct(r[i, :, 4] * TICK_US - base, 50), "issued_max": pct(r[i, :, 4] * TICK_US - base, 100),
            "tile0_landed_p50": pct(r[i, :, 7] * TICK_US - base, 50),
            "tile0_landed_max": pct(r[i, :, 7] * TICK_US - base, 100),
            "loop_end_p50": pct(t[:, 2], 50), "loop_end_max": pct(t[:, 2], 100),
            "exit_p10": pct(t[:, 3], 10), "exit_p50": pct(t[:, 3], 50), "exit_p90": pct(t[:, 3], 90),
            "exit_max": pct(t[:, 3], 100),
            "tail_p50": pct(t[:, 3] - t[:, 2], 50),
            "xcd_exit_max": [pct(t[xcc == x, 3], 100) if (xcc == x).any() else None for x in range(8)],
            "xcd_entry_p50": [pct(t[xcc == x, 0], 50) if (xcc == x).any() else None for x in range(8)],
        }
        if i + 1 < r.shape[0]:
            nxt = r[i + 1, :, 0].min() * TICK_US - base
            row["gap_to_next_entry"] = round(nxt - t[:, 3].max(), 2)
            row["period"] = round(nxt, 2)
        rows.append(row)
    for row in rows:
        print(json.dumps(row), flush=True)
    keys = [k for k in rows[0] if k not in ("launch", "xcd_exit_max", "xcd_entry_p50")]
    med = {k: round(float(np.median([row[k] for row in rows if row.get(k) is not None])), 2)
           for k in keys if any(row.get(k) is not None for row in rows)}
    wid = np.arange(waves) % 8
    t2 = np.stack([(r[i, :, 2] - r[i, :, 0].min()) * TICK_US for i in range(r.shape[0])])
    med["loop_end_by_wave_in_wg"] = [round(float(np.median(t2[:, wid == w])), 2) for w in range(8)]
    # the same per wave of a workgroup for entry, tile 0's loads issued, tile 0 landed and exit
    for name, col in (("entry", 0), ("issued", 4), ("tile0_landed", 7), ("exit", 3)):
        tt = np.stack([(r[i, :, col].astype(np.float64) - r[i, :, 0].min()) * TICK_US for i in range(r.shape[0])])
        med[f"{name}_by_wave_in_wg"] = [round(float(np.median(tt[:, wid == w])), 2) for w in range(8)]
    # placement of wave w of a workgroup (HW_ID of launch 1): SIMD and wave slot, as counts
    hw = r[0, :, 6].astype(np.int64)
    simd, slot = (hw >> 4) & 3, hw & 15
    med["simd_by_wave_in_wg"] = [dict(zip(*[x.tolist() for x in np.unique(simd[wid == w], return_counts=True)]))
                                 for w in range(8)]
    med["slot_by_wave_in_wg"] = [dict(zip(*[x.tolist() for x in np.unique(slot[wid == w], return_counts=True)]))
                                 for w in range(8)]
    med["event_span_us_per_launch"] = round(span_ms * 1e3, 2)
    med["waves"] = waves
    med["tiles_per_wave"] = sorted(set(int(x) >> 32 for x in r[0, :, 5]))
    print(json.dumps({"median_over_launches": med}), flush=True)


if __name__ == "__main__":
    main()
