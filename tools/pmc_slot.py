#!/usr/bin/env python3
"""Small fixed workload for PMC passes on the fused slot kernel (investigation tool): after a
settle, 20 launches each of config S publish, config S verify and the plain uniform kernel
over the same stride-4,160 payloads. The library comes from SUBSPACE_CRC_PROBE_LIB when set.
Run under `rocprofv3 --pmc ...`, one counter group per pass (tools/session_pmc_slot.sh)."""
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import gpu, slots  # noqa: E402

N, SIZE = 65536, 4096


def main():
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    ps, stride = slots.compute_prefix_size(4, 0), slots.slot_stride(SIZE, 4, 0)
    rng = np.random.default_rng(7)
    host = rng.integers(0, 256, stride * N, dtype=np.uint8)
    host.reshape(N, stride)[:, :ps] = slots.make_prefixes(
        N, np.full(N, SIZE, dtype=np.uint64), checksum_size=4, metadata_size=0, seed=5)
    buf = torch.from_numpy(host).to(dev)
    out = torch.empty(N, dtype=torch.int32, device=dev)
    status = torch.empty(N, dtype=torch.int32, device=dev)
    errs = torch.zeros(1, dtype=torch.int32, device=dev)
    for _ in range(200):
        ctx.crc32_uniform(buf, stride, SIZE, N, out, base_offset=ps)
    for _ in range(20):
        ctx.crc32_slots_strided(buf, stride, N, message_size=SIZE, mode=gpu.SLOT_CALCULATE)
    for _ in range(20):
        ctx.crc32_slots_strided(buf, stride, N, message_size=SIZE, mode=gpu.SLOT_VERIFY, status=status,
                                error_count=errs)
    for _ in range(20):
        ctx.crc32_uniform(buf, stride, SIZE, N, out, base_offset=ps)
    torch.cuda.synchronize()
    assert int(errs.item()) == 0


if __name__ == "__main__":
    main()
