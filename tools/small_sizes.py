#!/usr/bin/env python3
"""Throughput of the small-message kernel by message size (investigation tool): uniform batches
of n messages of L bytes (stride = L rounded up to 16 B) through subspace_crc32_batch_uniform,
event-timed over `launches` back-to-back calls after `settle` untimed ones, rotated over buffers
large enough to leave the 256 MB MALL behind.

  python tools/small_sizes.py [L,L,...] [launches] [settle]
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import gpu  # noqa: E402


def main():
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "64,256,1024,2048,4000").split(",")]
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    settle = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    ctx = gpu.CrcContext(0)
    dev = torch.device("cuda", 0)
    for L in sizes:
        stride = (L + 15) & ~15
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
        del bufs, out
        torch.cuda.empty_cache()
    ctx.close()


if __name__ == "__main__":
    main()
