#!/usr/bin/env python3
"""What a large VRAM free does to the next seconds: allocate, touch and free GIB of device
memory, then every ~0.25 s print the device's free memory (hipMemGetInfo) and the time of
100 back-to-back config-B launches (uniform 4 KiB kernel, 256 MiB each), for SECONDS.

  python tools/wipe_watch.py [GIB] [SECONDS]
"""
import json
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import gpu  # noqa: E402

N, SIZE = 65536, 4096


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 110.0
    secs = float(sys.argv[2]) if len(sys.argv) > 2 else 12.0
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    bufs = [torch.empty(N * SIZE, dtype=torch.uint8, device=dev) for _ in range(4)]
    for k, b in enumerate(bufs):
        gpu.fill_uniform(b, SIZE, SIZE, N, seed=11, first_id=k * N)
    out = torch.empty(N, dtype=torch.int32, device=dev)

    def launches_us(n=100):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(n):
            ctx.crc32_uniform(bufs[i % 4], SIZE, SIZE, N, out)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / n * 1e3

    for _ in range(40):  # power-management settle
        launches_us()
    free0, total = torch.cuda.mem_get_info()
    print(json.dumps({"phase": "before", "free_gib": round(free0 / 2**30, 2), "total_gib": round(total / 2**30, 2),
                      "us_per_launch": round(launches_us(), 2)}), flush=True)
    big = torch.empty(int(gib * 2**30), dtype=torch.uint8, device=dev)
    big[::1 << 20].fill_(1)
    torch.cuda.synchronize()
    print(json.dumps({"phase": "allocated", "free_gib": round(torch.cuda.mem_get_info()[0] / 2**30, 2),
                      "us_per_launch": round(launches_us(), 2)}), flush=True)
    del big
    torch.cuda.empty_cache()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < secs:
        f = torch.cuda.mem_get_info()[0]
        us = launches_us()
        print(json.dumps({"t_s": round(time.perf_counter() - t0, 2), "free_gib": round(f / 2**30, 2),
                          "us_per_launch": round(us, 2)}), flush=True)
        time.sleep(0.2)


if __name__ == "__main__":
    main()
