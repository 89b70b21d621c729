#!/usr/bin/env python3
"""Fixed workloads for the headline kernel's compute ledger (investigation tool; run under
`rocprofv3 --kernel-trace` or `--pmc`, one mode per process, tools/pmc_ledger.sh):

  hbm   -- config B: the uniform 4 KiB kernel over 65,536 messages per launch, rotated over
           five 256 MiB batches (1.25 GiB: no launch is served from the MALL)
  l2    -- the same kernel, grid and tile count, every message aliasing one 4 KiB message
           (subspace_crc_testutil_uniform_alias): its compute-only time
  read  -- stream_read_kernel (testutil.hip) over the same batches: the kernel's load shape
           with an XOR fold instead of the CRC (bench.py's read ceiling)

Each mode runs `settle` untimed launches then `launches` more, and prints one JSON line with
the event-timed mean of the latter (the PMC passes read the per-dispatch counters)."""
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import _lib, gpu  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "hbm"
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    settle = int(sys.argv[3]) if len(sys.argv) > 3 else 400
    count, nb = 65536, 5
    ctx = gpu.CrcContext(0)
    lib = _lib.load()
    wg = int(os.environ.get("UNIFORM_WG", "512"))  # the tuning hook's workgroup size (512: the product's)
    if wg != 512 and _lib.load_dev().subspace_crc_testutil_tune(ctx._h, wg, 0, 0) != 0:
        raise SystemExit(f"tune failed: {_lib.last_error()}")
    dev = torch.device("cuda", 0)
    bufs = [torch.empty(count * 4096, dtype=torch.uint8, device=dev) for _ in range(nb)]
    for k, b in enumerate(bufs):
        gpu.fill_uniform(b, 4096, 4096, count, seed=0x5EED000B, first_id=k * count)
    out = torch.empty(count, dtype=torch.int32, device=dev)
    sink = torch.empty(256 * 512, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()

    def one(i):
        if mode == "hbm":
            ctx.crc32_uniform(bufs[i % nb], 4096, 4096, count, out)
        elif mode == "l2":
            rc = _lib.load_dev().subspace_crc_testutil_uniform_alias(ctx._h, bufs[0].data_ptr(), count, out.data_ptr(),
                                                         st.cuda_stream)
            if rc != 0:
                raise SystemExit(f"uniform_alias failed: {_lib.last_error()}")
        else:
            gpu.stream_read(bufs[i % nb], sink)

    torch.cuda.synchronize()
    for i in range(settle):
        one(i)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(launches):
        one(i)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / launches
    line = {"mode": mode, "wg": wg, "launches": launches, "settle": settle, "us_per_launch": round(us, 3),
            "GBps": round(count * 4096 / us / 1e3, 1)}
    if mode == "l2":  # every message is message 0 of batch 0
        line["alias_crc_equal"] = bool((out == out[0]).all().item())
    print(json.dumps(line))
    ctx.close()


if __name__ == "__main__":
    main()
