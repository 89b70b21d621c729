#!/usr/bin/env python3
"""Where config B's gap to the read ceiling goes: the streaming-read probe (the CRC kernel's
load shape, one tile in flight, no CRC) with 0 / 64 / 152 KiB of unused dynamic LDS per
workgroup, against the CRC kernel, interleaved rounds in one process (us per 256 MiB launch,
400 launches back to back after 1,400).

  python tools/lds_probe.py [rounds]
"""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import _lib, gpu  # noqa: E402

N, SIZE = 65536, 4096


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    bufs = [torch.empty(N * SIZE, dtype=torch.uint8, device=dev) for _ in range(4)]
    for k, b in enumerate(bufs):
        gpu.fill_uniform(b, SIZE, SIZE, N, seed=11, first_id=k * N)
    sink = torch.empty(256 * 512, dtype=torch.int32, device=dev)
    out = torch.empty(N, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def lds(nbytes):
        def f(b):
            rc = _lib.load_dev().subspace_crc_testutil_stream_read_lds(b.data_ptr(), N * SIZE, sink.data_ptr(), nbytes, st)
            assert rc == 0
        return f
    variants = {"read": lambda b: gpu.stream_read(b, sink), "read_lds0": lds(0), "read_lds64k": lds(64 << 10),
                "read_lds152k": lds(152 << 10), "crc": lambda b: ctx.crc32_uniform(b, SIZE, SIZE, N, out)}
    res = {}
    for _ in range(rounds):
        for name, f in variants.items():
            for i in range(1400):
                f(bufs[i % 4])
            a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for i in range(400):
                f(bufs[i % 4])
            e.record()
            torch.cuda.synchronize()
            res.setdefault(name, []).append(round(a.elapsed_time(e) / 400 * 1e3, 2))
    for name, v in res.items():
        print(json.dumps({"variant": name, "us_per_launch": v}), flush=True)


if __name__ == "__main__":
    main()
