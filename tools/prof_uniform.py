#!/usr/bin/env python3
"""A fixed number of uniform-kernel launches for PMC profiling (investigation tool):
  rocprofv3 --pmc SQ_WAVE_CYCLES ... -- python3 tools/prof_uniform.py [count] [launches]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import gpu  # noqa: E402

count = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
launches = int(sys.argv[2]) if len(sys.argv) > 2 else 6
ctx = gpu.CrcContext(0)
nb = max(1, (1 << 30) // (count * 4096) + 1)
bufs = [torch.empty(count * 4096, dtype=torch.uint8, device="cuda") for _ in range(nb)]
for k, b in enumerate(bufs):
    gpu.fill_uniform(b, 4096, 4096, count, seed=0x5EED000B, first_id=k * count)
out = torch.empty(count, dtype=torch.int32, device="cuda")
for i in range(launches):
    ctx.crc32_uniform(bufs[i % nb], 4096, 4096, count, out)
torch.cuda.synchronize()
print("ok", count, launches)
ctx.close()
