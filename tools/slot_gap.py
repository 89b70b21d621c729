#!/usr/bin/env python3
"""Where config S's extra time over config B goes: the uniform kernel over the same channel
buffers at strides 4,096 / 4,160 (payload offsets 64 and 0) / 4,224, against the fused slot
kernel (verify, publish), interleaved rounds in one process. One JSON line per variant
(median / best us per 65,536-message call)."""
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import gpu, slots  # noqa: E402

N, SIZE, NBUF = 65536, 4096, 4


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    iters = 100
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    ps, stride = slots.compute_prefix_size(4, 0), slots.slot_stride(SIZE, 4, 0)
    assert (ps, stride) == (64, 4160)
    rng = np.random.default_rng(7)
    host = rng.integers(0, 256, 4224 * N, dtype=np.uint8)
    host[:stride * N].reshape(N, stride)[:, :ps] = slots.make_prefixes(
        N, np.full(N, SIZE, dtype=np.uint64), checksum_size=4, metadata_size=0, seed=5)
    bufs = [torch.from_numpy(host).to(dev) for _ in range(NBUF)]
    out = torch.empty(N, dtype=torch.int32, device=dev)
    status = torch.empty(N, dtype=torch.int32, device=dev)
    errs = torch.zeros(1, dtype=torch.int32, device=dev)
    variants = {
        "uniform_4096": lambda b: ctx.crc32_uniform(b, 4096, SIZE, N, out),
        "uniform_4160_off64": lambda b: ctx.crc32_uniform(b, 4160, SIZE, N, out, base_offset=64),
        "uniform_4160_off0": lambda b: ctx.crc32_uniform(b, 4160, SIZE, N, out),
        "uniform_4224_off64": lambda b: ctx.crc32_uniform(b, 4224, SIZE, N, out, base_offset=64),
        "uniform_4224_off128": lambda b: ctx.crc32_uniform(b, 4224, SIZE, N, out, base_offset=128),
        "slot_publish": lambda b: ctx.crc32_slots_strided(b, stride, N, message_size=SIZE, mode=gpu.SLOT_CALCULATE),
        "slot_verify": lambda b: ctx.crc32_slots_strided(b, stride, N, message_size=SIZE, mode=gpu.SLOT_VERIFY,
                                                         status=status, error_count=errs),
    }
    for i in range(600):  # power-management settle (profiles/DESIGN_r01-r03.md 4.0)
        variants["uniform_4096"](bufs[i % NBUF])
    torch.cuda.synchronize()
    res = {}
    for r in range(rounds):
        for name, f in variants.items():
            for i in range(5):
                f(bufs[i % NBUF])
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(iters):
                f(bufs[i % NBUF])
            b.record()
            torch.cuda.synchronize()
            res.setdefault(name, []).append(a.elapsed_time(b) / iters * 1e3)
    if not os.environ.get("SLOT_GAP_NOCHECK"):  # (timing-only builds of the slot kernel)
        assert int(errs.item()) == 0
    for name, v in res.items():
        print(json.dumps({"variant": name, "median_us": round(float(np.median(v)), 2),
                          "best_us": round(float(np.min(v)), 2)}), flush=True)


if __name__ == "__main__":
    main()
