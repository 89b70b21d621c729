#!/usr/bin/env python3
"""Config S launch by launch: bench.py's S publish / verify timing loop (400 back-to-back
calls over 4 rotated channel buffers after ~60 ms of warm-up calls), with the host's
enqueue time per call next to the event span, so a rocprofv3 --kernel-trace of this script
gives every launch's duration and its gap to the next (tools/s_launches.py --analyze <csv>).

  python tools/s_launches.py [calls] [--prealloc=GiB [--hold=s]] [--keep=GiB] [--sleep=s] [--after=GiB]
      one JSON line per mode; optionally after allocating GiB (held s seconds) and freeing it
      before the channel buffers, or allocating GiB and keeping it, then sleeping s seconds;
      or allocating and freeing GiB after the channel buffers
  python tools/s_launches.py --analyze run_kernel_trace.csv
"""
import csv
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

N, SIZE, NBUF = 65536, 4096, 4


def big_alloc_free(gib: float, hold_s: float = 0.0, keep: bool = False):
    """As bench.py's configs C/D before S: a large allocation, touched, held hold_s seconds,
    then freed back to the driver (or kept, and returned)."""
    import torch
    big = torch.empty(int(gib * 2**30), dtype=torch.uint8, device="cuda")
    big[::1 << 20].fill_(1)
    torch.cuda.synchronize()
    time.sleep(hold_s)
    if keep:
        return big
    del big
    torch.cuda.empty_cache()
    return None


def run(calls: int, prealloc_gib: float = 0.0, sleep_s: float = 0.0, after_gib: float = 0.0, hold_s: float = 0.0,
        keep_gib: float = 0.0) -> None:
    import torch
    from subspace_amd import gpu, slots
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    if prealloc_gib:
        big_alloc_free(prealloc_gib, hold_s)
    kept = big_alloc_free(keep_gib, keep=True) if keep_gib else None  # allocated, never freed
    time.sleep(sleep_s)
    cs, ms_ = 4, 0
    ps, stride = slots.compute_prefix_size(cs, ms_), slots.slot_stride(SIZE, cs, ms_)
    rng = np.random.default_rng(0x5EED0005)
    host = rng.integers(0, 256, stride * N, dtype=np.uint8)
    host.reshape(N, stride)[:, :ps] = slots.make_prefixes(N, np.full(N, SIZE, dtype=np.uint64), checksum_size=cs,
                                                          metadata_size=ms_, seed=5)
    bufs = [torch.from_numpy(host).to(dev) for _ in range(NBUF)]
    status = torch.empty(N, dtype=torch.int32, device=dev)
    errs = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.empty(N, dtype=torch.int32, device=dev)
    nbytes = N * (SIZE + 44)
    if after_gib:  # the same, after the channel buffers exist (placement vs. what follows a free)
        big_alloc_free(after_gib)
    print(json.dumps({"buffers": [hex(b.data_ptr()) for b in bufs], "prealloc_gib": prealloc_gib, "sleep_s": sleep_s,
                      "after_gib": after_gib, "hold_s": hold_s, "keep_gib": keep_gib, "kept": kept is not None}),
          flush=True)
    st = torch.cuda.current_stream()
    modes = [("uniform_4160", None), ("S_publish", gpu.SLOT_CALCULATE), ("S_verify", gpu.SLOT_VERIFY),
             ("S_publish", gpu.SLOT_CALCULATE)]
    for name, mode in modes:
        i = [0]

        def call():
            b = bufs[i[0] % NBUF]
            i[0] += 1
            if mode is None:
                ctx.crc32_uniform(b, stride, SIZE, N, out, base_offset=ps)
            else:
                ctx.crc32_slots_strided(b, stride, N, message_size=SIZE, checksum_size=cs, metadata_size=ms_,
                                        mode=mode, status=status if mode == gpu.SLOT_VERIFY else None,
                                        error_count=errs if mode == gpu.SLOT_VERIFY else None, stream=st)
        for _ in range(1300):  # ~60 ms back to back, as bench.py's time_calls
            call()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        t0 = time.perf_counter()
        for _ in range(calls):
            call()
        t1 = time.perf_counter()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / calls
        print(json.dumps({"mode": name, "event_us_per_call": round(ms * 1e3, 2),
                          "host_enqueue_us_per_call": round((t1 - t0) / calls * 1e6, 2),
                          "pct_of_8TBs": round(100 * nbytes / (ms * 1e-3) / 8e12, 2)}), flush=True)


def analyze(path: str) -> None:
    rows = [r for r in csv.DictReader(open(path)) if "crc32_uniform4k" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    kinds = {}
    for r in rows:
        kinds.setdefault(r["Kernel_Name"], []).append(r)
    for name, rs in kinds.items():
        d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rs])
        s = np.array([int(r["Start_Timestamp"]) for r in rs]) / 1e3
        gaps = np.diff(s) - d[:-1]
        # runs of back-to-back launches: split where the gap exceeds 1 ms (between modes)
        cut = np.where(gaps > 1000)[0]
        starts = np.concatenate([[0], cut + 1])
        ends = np.concatenate([cut + 1, [len(d)]])
        for a, b in zip(starts, ends):
            seg = d[a:b][-400:]
            g = gaps[a:b - 1][-399:]
            by_buf = [float(np.mean(seg[k::4])) for k in range(4)]
            print(json.dumps({"kernel": name[:70], "launches": int(b - a), "mean_us": round(float(seg.mean()), 2),
                              "median_us": round(float(np.median(seg)), 2),
                              "p10": round(float(np.percentile(seg, 10)), 2),
                              "p90": round(float(np.percentile(seg, 90)), 2), "max": round(float(seg.max()), 2),
                              "gap_mean_us": round(float(g.mean()), 2) if len(g) else None,
                              "gap_p90_us": round(float(np.percentile(g, 90)), 2) if len(g) else None,
                              "mean_by_launch_mod4": [round(x, 2) for x in by_buf],
                              "first50_mean": round(float(seg[:50].mean()), 2),
                              "last50_mean": round(float(seg[-50:].mean()), 2)}))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        opts = {a.split("=")[0][2:]: float(a.split("=")[1]) for a in sys.argv[1:] if a.startswith("--")}
        args = [a for a in sys.argv[1:] if not a.startswith("--")]
        run(int(args[0]) if args else 400, opts.get("prealloc", 0.0), opts.get("sleep", 0.0), opts.get("after", 0.0),
            opts.get("hold", 0.0), opts.get("keep", 0.0))
