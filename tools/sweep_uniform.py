#!/usr/bin/env python3
"""Tuning sweep for the uniform 4 KiB kernel: batch size x workgroup size, interleaved
rounds in one process (cdna_hip_programming.md section 5.4 rule 24). Prints one JSON line
per variant with median / best kernel time and HBM rate."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import _lib, gpu  # noqa: E402


def main():
    counts = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["65536", "262144", "1048576"])]
    wgs = [int(x) for x in (sys.argv[2].split(",") if len(sys.argv) > 2 else ["512", "768", "1024"])]
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    orders = [int(x) for x in (sys.argv[4].split(",") if len(sys.argv) > 4 else ["0"])]
    blocks = [int(x) for x in (sys.argv[5].split(",") if len(sys.argv) > 5 else ["0"])]
    ctx = gpu.CrcContext(0)
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    res = {}
    for count in counts:
        nb = max(2, (1 << 30) // (count * 4096) + 1)  # >= 1 GiB rotated so the MALL cannot serve re-reads
        bufs = [torch.empty(count * 4096, dtype=torch.uint8, device=dev) for _ in range(nb)]
        for k, b in enumerate(bufs):
            gpu.fill_uniform(b, 4096, 4096, count, seed=0x5EED000B, first_id=k * count)
        out = torch.empty(count, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        iters = max(8, int(2e9 // (count * 4096)))
        for i in range(max(400, int(16e9 // (count * 4096)))):  # >= ~20 ms of warm-up (sustained.md)
            ctx.crc32_uniform(bufs[i % nb], 4096, 4096, count, out)
        torch.cuda.synchronize()
        ref = None
        for r in range(rounds):
            for wg, order, nb_cap in [(a, b, c) for a in wgs for b in orders for c in blocks]:
                if _lib.load_dev().subspace_crc_testutil_tune(ctx._h, wg, nb_cap, order) != 0:
                    raise SystemExit(f"bad variant wg={wg} order={order}")
                if r == 0:  # every variant must produce the same CRCs
                    ctx.crc32_uniform(bufs[0], 4096, 4096, count, out)
                    got = out.clone()
                    if ref is None:
                        ref = got
                    elif not torch.equal(ref, got):
                        raise SystemExit(f"variant wg={wg} order={order} blocks={nb_cap} differs")
                for i in range(3):
                    ctx.crc32_uniform(bufs[i % nb], 4096, 4096, count, out)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for i in range(iters):
                    ctx.crc32_uniform(bufs[i % nb], 4096, 4096, count, out)
                b.record()
                torch.cuda.synchronize()
                ms = a.elapsed_time(b) / iters
                res.setdefault((count, wg, order, nb_cap), []).append(ms)
        del bufs
        torch.cuda.empty_cache()
    for (count, wg, order, nb_cap), v in sorted(res.items()):
        med, best = float(np.median(v)), float(np.min(v))
        print(json.dumps({"count": count, "wg": wg, "order": order, "blocks": nb_cap or "all CUs",
                          "median_ms": round(med, 4), "best_ms": round(best, 4),
                          "TBps_median": round(count * 4096 / med / 1e9, 3),
                          "TBps_best": round(count * 4096 / best / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
