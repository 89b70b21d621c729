#!/usr/bin/env python3
"""Sustained-launch behaviour of the uniform kernel variants (investigation tool).

Phases of N back-to-back config-B launches (4 rotated 256 MiB batches), separated by idle
pauses, alternating the CRC kernel (1) and the streaming-read probe over the same batches
(0, no CRC). Prints wall-clock GiB/s per phase; run under `rocprofv3 --kernel-trace` for
per-launch durations.

  python tools/throttle_trace.py [--launches 300] [--pause 3] [--variants 0,1,0,1]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from subspace_amd import gpu  # noqa: E402

MSGS, MSG = 65536, 4096


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=300)
    ap.add_argument("--pause", type=float, default=3.0)
    ap.add_argument("--variants", default="0,1,0,1")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    bufs = [torch.empty(MSGS * MSG, dtype=torch.uint8, device=dev) for _ in range(4)]
    outs = [torch.empty(MSGS, dtype=torch.int32, device=dev) for _ in range(4)]
    for k, b in enumerate(bufs):
        gpu.fill_uniform(b, MSG, MSG, MSGS, seed=0x5EED000B, first_id=k * MSGS)
    torch.cuda.synchronize()
    ref = None
    sink = torch.empty(256 * 512, dtype=torch.int32, device=dev)
    for ph, v in enumerate(int(x) for x in args.variants.split(",")):
        time.sleep(args.pause)
        t0 = time.perf_counter()
        for i in range(args.launches):
            if v:
                ctx.crc32_uniform(bufs[i % 4], MSG, MSG, MSGS, outs[i % 4])
            else:  # 0: the streaming-read probe over the same batches (no CRC)
                gpu.stream_read(bufs[i % 4], sink)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        same = None
        if v:
            crcs = outs[0].cpu()
            same = None if ref is None else bool(torch.equal(crcs, ref))
            ref = crcs if ref is None else ref
        print(json.dumps({"phase": ph, "crc": bool(v), "launches": args.launches, "us_per_launch": round(dt / args.launches * 1e6, 2),
                          "GiBps": round(MSGS * MSG * args.launches / dt / 2**30, 1), "same_crcs_as_phase0": same}),
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
