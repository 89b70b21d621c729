#!/usr/bin/env python3
"""Small fixed workload for PMC passes (investigation tool): 3 launches each of the
uniform kernel (1 Mi x 4 KiB = 4 GiB), the ragged kernel on config D's shape (32 x 64 MiB
= 2 GiB) and on config C's shape (10,000 log-uniform messages, ~1 GiB, unaligned ends).
Run under `rocprofv3 --pmc ...`, one counter group per pass."""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import gpu  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    n = 1 << 20
    buf = torch.empty(n * 4096, dtype=torch.uint8, device=dev)
    gpu.fill_uniform(buf, 4096, 4096, n, seed=0x5EED000E)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(3):
        ctx.crc32_uniform(buf, 4096, 4096, n, out)
    torch.cuda.synchronize()
    m, L = 32, 64 << 20
    lens = torch.full((m,), L, dtype=torch.int64, device=dev)
    offs = torch.arange(m, dtype=torch.int64, device=dev) * L
    rout = torch.empty(m, dtype=torch.int32, device=dev)
    for _ in range(3):
        ctx.crc32_ragged(buf[: m * L], offs, lens, rout)
    torch.cuda.synchronize()
    # config D's shape through the uniform API: the long-message kernel
    for _ in range(3):
        ctx.crc32_uniform(buf[: m * L], L, L, m, rout)
    torch.cuda.synchronize()
    # config C's shape (log-uniform 64 B - 1 MiB, unaligned ends) over ~1 GiB
    from subspace_amd import synth
    lens = synth.ragged_lengths(synth.SEED_C, 10000)
    offs, total = synth.packed_offsets(lens, 64)
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int64)).to(dev)
    cout = torch.empty(len(lens), dtype=torch.int32, device=dev)
    for _ in range(3):
        ctx.crc32_ragged(buf[: int(total) + 64], d_off, d_len, cout)
    torch.cuda.synchronize()
    print("ok", int(out[0].item()) & 0xFFFFFFFF, int(rout[0].item()) & 0xFFFFFFFF, int(total), "C payload bytes",
          int(lens.sum()))
    ctx.close()


if __name__ == "__main__":
    main()
