#!/usr/bin/env python3
"""Fixed workloads for the slot-list drain's compute ledger (investigation
tool, run directly or under `rocprofv3 --kernel-trace` / `--pmc`, tools/pmc_ledger.sh with
LEDGER=small). Config S's channel (65,536 slots of MessagePrefix 64 B + 4 KiB payload, stride
4,160), in four device copies (1.09 GB, beyond the 256 MB MALL), verified through
subspace_crc32_slots (the small-message kernel, crc_small.hip) or read by the probes:

  list     -- the slots as a shuffled device slot list, rotated over the four copies
  list1    -- the same, every call over copy 0 (round 4's bench.py S_list)
  ordered  -- the slot list in channel order, rotated
  alias    -- every record pointing at slot 0 of copy 0: the kernel's compute-only time at
              the same grid and tile count (every line load an L2 hit)
  probe0   -- slot_list_read_kernel<0> (testutil.hip) over the shuffled rotated lists: the
              kernel's loads (records one tile ahead, clamped lines, first-window prefix
              words) with an XOR fold instead of the CRC -- the access shape's read ceiling
  probe1   -- slot_list_read_kernel<1>: the same with the wave's records held in registers
  probe0o  -- probe0 over the ordered lists (probe1o: probe1's)
  probe2   -- no records: slot m's payload from the channel stride, clamped block addresses
  probe3   -- as probe2 with one address and immediate offsets (the uniform kernel's loads);
              probe3n without the kernel's LDS allocation
  probe4   -- the window's records in registers, one address and immediate offsets (the
              small kernel's FAST loop), shuffled; probe4o ordered, probe4n ordered without LDS
  probe5   -- probe4 with two tiles in flight per wave (probe5o ordered); probe6: probe3 so
  list_ns, ordered_ns, strided_ns -- the same without the per-slot status array (the
              mismatch count only)
  strided  -- the fused uniform slot kernel (subspace_crc32_slots_strided), verify, rotated:
              config S's S_verify, the same slots read in channel order
  mixed    -- the shuffled lists with message sizes 1 .. 4,096 B (uniformly random; bench.py's
              S_mixed shape: the repack by size), verify (mismatches: the same reads);
              mixed_alias its compute-only twin (every record at slot 0 of copy 0, the same
              sizes); mixed_probe0 slot_list_read_kernel<0> over the mixed lists (clamped lines
              of each message's length: the access shape's read ceiling, no CRC)

  python tools/ledger_small.py <mode>[,<mode>...] [launches] [settle] [rounds]

One JSON line per mode and round: the event-timed mean of `launches` back-to-back calls after
`settle` untimed ones. SUBSPACE_CRC_PROBE_LIB selects a library variant (tools/ab_lib.sh)."""
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import _lib, gpu, slots  # noqa: E402

N, SIZE, CS, MS, NB = 65536, 4096, 4, 0, 4


def main():
    modes = (sys.argv[1] if len(sys.argv) > 1 else "list").split(",")
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    settle = int(sys.argv[3]) if len(sys.argv) > 3 else 400
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 1
    check = not os.environ.get("SLOT_LIST_NOCHECK")
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)
    lib = _lib.load()
    ps, stride = slots.compute_prefix_size(CS, MS), slots.slot_stride(SIZE, CS, MS)
    rng = np.random.default_rng(0x5EED0005)
    host = rng.integers(0, 256, stride * N, dtype=np.uint8)
    host.reshape(N, stride)[:, :ps] = slots.make_prefixes(N, np.full(N, SIZE, dtype=np.uint64), checksum_size=CS,
                                                          metadata_size=MS, seed=5)
    bufs = [torch.from_numpy(host).to(dev) for _ in range(NB)]
    for b in bufs:  # published: every slot verifies
        ctx.crc32_slots_strided(b, stride, N, message_size=SIZE, checksum_size=CS, metadata_size=MS,
                                mode=gpu.SLOT_CALCULATE)
    status = torch.empty(N, dtype=torch.int32, device=dev)
    errs = torch.zeros(1, dtype=torch.int32, device=dev)
    perm = rng.permutation(N).astype(np.uint64)

    def recs(buf, order, sizes=None):
        b0 = np.uint64(buf.data_ptr())
        r = np.stack([b0 + order * np.uint64(stride), b0 + order * np.uint64(stride) + np.uint64(ps),
                      np.full(len(order), SIZE, dtype=np.uint64) if sizes is None else sizes], axis=1)
        return torch.from_numpy(np.ascontiguousarray(r).view(np.int64)).to(dev)

    shuffled = [recs(b, perm) for b in bufs]
    msz = np.random.default_rng(0x5EED0258).integers(1, SIZE + 1, N).astype(np.uint64)
    mixed = [recs(b, perm, msz) for b in bufs] if any(m.startswith("mixed") for m in modes) else []
    mixed_alias = recs(bufs[0], np.zeros(N, dtype=np.uint64), msz) if "mixed_alias" in modes else None
    ordered = [recs(b, np.arange(N, dtype=np.uint64)) for b in bufs]
    alias = recs(bufs[0], np.zeros(N, dtype=np.uint64))
    sink = torch.empty(2048 * 512, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()

    def slot_list(r, st_out=True):
        ctx.crc32_slots(r, max_message_size=SIZE, checksum_size=CS, metadata_size=MS, mode=gpu.SLOT_VERIFY,
                        status=status if st_out else None, error_count=errs)

    def probe(r, rec, lds=1):
        rc = _lib.load_dev().subspace_crc_testutil_slot_list_read(r.data_ptr(), N, rec, stride, lds, sink.data_ptr(), sink.numel(),
                                                      st.cuda_stream)
        if rc != 0:
            raise SystemExit(f"slot_list_read failed: {rc}")

    calls = {
        "list": lambda i: slot_list(shuffled[i % NB]),
        "list1": lambda i: slot_list(shuffled[0]),
        "list_ns": lambda i: slot_list(shuffled[i % NB], False),
        "ordered_ns": lambda i: slot_list(ordered[i % NB], False),
        "strided_ns": lambda i: ctx.crc32_slots_strided(bufs[i % NB], stride, N, message_size=SIZE, checksum_size=CS,
                                                        metadata_size=MS, mode=gpu.SLOT_VERIFY, status=None,
                                                        error_count=errs),
        "ordered": lambda i: slot_list(ordered[i % NB]),
        "alias": lambda i: slot_list(alias),
        "probe0": lambda i: probe(shuffled[i % NB], 0),
        "probe1": lambda i: probe(shuffled[i % NB], 1),
        "probe0o": lambda i: probe(ordered[i % NB], 0),
        "probe1o": lambda i: probe(ordered[i % NB], 1),
        "probe2": lambda i: probe(ordered[i % NB], 2),
        "probe3": lambda i: probe(ordered[i % NB], 3),
        "probe3n": lambda i: probe(ordered[i % NB], 3, 0),
        "probe4": lambda i: probe(shuffled[i % NB], 4),
        "probe4o": lambda i: probe(ordered[i % NB], 4),
        "probe4n": lambda i: probe(ordered[i % NB], 4, 0),
        "probe5": lambda i: probe(shuffled[i % NB], 5),
        "probe5o": lambda i: probe(ordered[i % NB], 5),
        "probe6": lambda i: probe(ordered[i % NB], 6),
        "mixed": lambda i: slot_list(mixed[i % NB]),
        "mixed_alias": lambda i: slot_list(mixed_alias),
        "mixed_probe0": lambda i: probe(mixed[i % NB], 0),
        "strided": lambda i: ctx.crc32_slots_strided(bufs[i % NB], stride, N, message_size=SIZE, checksum_size=CS,
                                                     metadata_size=MS, mode=gpu.SLOT_VERIFY, status=status,
                                                     error_count=errs),
    }
    for r in range(rounds):
        for mode in modes:
            one = calls[mode]
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
            nbytes = (int(msz.sum()) + 44 * N) if mode.startswith("mixed") else N * (SIZE + 44)  # checksummed bytes
            line = {"mode": mode, "round": r, "launches": launches, "settle": settle, "us_per_launch": round(us, 3),
                    "pct_of_hbm_peak": round(100 * nbytes / us / 1e3 / 8000.0, 2)}
            if check and mode in ("list", "list1", "ordered", "alias", "strided", "list_ns", "ordered_ns", "strided_ns"):
                line["all_pass"] = int(errs.item()) == 0 and (mode.endswith("_ns") or bool((status == 0).all().item()))
            print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
