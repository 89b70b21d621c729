#!/usr/bin/env python3
"""Read ceiling of a large batch (investigation tool): gpu.stream_read (the CRC kernels' load
shape with an XOR fold) over config D's 16 GiB against the long-message kernel
(subspace_crc32_batch_uniform) and the ragged kernel (subspace_crc32_batch) on the same bytes,
event-timed, `iters` calls each after a warm-up.

  python tools/read_ceiling_large.py [iters]
"""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import gpu, synth  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    n, L = 256, 64 << 20
    buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
    gpu.fill_uniform(buf, L, L, n, seed=synth.SEED_D)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    sink = torch.empty(256 * 512, dtype=torch.int32, device=dev)
    d_off = torch.from_numpy((np.arange(n, dtype=np.uint64) * np.uint64(L)).view(np.int64)).to(dev)
    d_len = torch.from_numpy(np.full(n, L, dtype=np.uint64).view(np.int64)).to(dev)
    res = {"bytes": n * L}
    res["read_ms"] = round(timed(lambda: gpu.stream_read(buf, sink), iters), 4)
    res["long_ms"] = round(timed(lambda: ctx.crc32_uniform(buf, L, L, n, out), iters), 4)
    res["ragged_ms"] = round(timed(lambda: ctx.crc32_ragged(buf, d_off, d_len, out), iters), 4)
    for k in ("read", "long", "ragged"):
        res[k + "_pct_of_hbm_peak"] = round(100 * n * L / (res[k + "_ms"] * 1e-3) / 8e12, 2)
    res["long_frac_of_read"] = round(res["read_ms"] / res["long_ms"], 4)
    res["ragged_frac_of_read"] = round(res["read_ms"] / res["ragged_ms"], 4)
    print(json.dumps(res))
    ctx.close()


if __name__ == "__main__":
    main()
