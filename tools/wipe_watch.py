#!/usr/bin/env python3
"""What a large VRAM free does to the next seconds: allocate, touch and free GIB of device
memory while config-B launches (uniform 4 KiB kernel, 256 MiB each) run back to back without
pause (an idle spell would restart the power-management ramp), and every ~0.25 s print the
device's free memory (hipMemGetInfo) and the mean time per launch of that interval, for
SECONDS; the same for SECONDS before the free, as the reference.

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

    def watch(phase, seconds):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            t1, us = time.perf_counter(), []
            while time.perf_counter() - t1 < 0.25:
                us.append(launches_us())
            print(json.dumps({"phase": phase, "t_s": round(time.perf_counter() - t0, 2),
                              "free_gib": round(torch.cuda.mem_get_info()[0] / 2**30, 2),
                              "us_per_launch": round(sum(us) / len(us), 2)}), flush=True)

    for _ in range(100):  # power-management settle
        launches_us()
    big = torch.empty(int(gib * 2**30), dtype=torch.uint8, device=dev)
    big[::1 << 20].fill_(1)
    torch.cuda.synchronize()
    watch("allocated", secs / 2)
    del big
    torch.cuda.empty_cache()
    watch("freed", secs)


if __name__ == "__main__":
    main()
