#!/usr/bin/env python3
"""One secondary bench configuration's C-ABI call, repeated, for a PMC pass (VERDICT r04 item 5:
the secondary configs' roofline.traffic). Run under `rocprofv3 --pmc FETCH_SIZE` (and a second
pass with WRITE_SIZE), one process per configuration (tools/pmc_configs.sh); the summary,
tools/summarize_configs_traffic.py, divides every dispatch's bytes of the call's kernels by the
calls made and writes profiles/traffic_configs.json, which bench.py reads.

  python tools/pmc_configs.py <config> [calls]
  config: C, Cu, D, Du, S_publish, S_verify, S_meta_publish, S_meta_verify, S_list_publish,
          S_list_verify, Usmall, S_short, S_mixed, S_large_verify, S_large_publish (bench.py's
          secondary configs, the same shapes and
          synthetic data)

Prints one JSON line: the config, the calls made and the algorithmic bytes per call (bench.py's
"bytes"). Verify legs run over unpublished slots (every slot a mismatch): the same reads."""
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from subspace_amd import gpu, slots, synth  # noqa: E402

GOLD = json.loads((Path(__file__).resolve().parent.parent / "tests" / "golden" / "configs.json").read_text())


def main():
    name = sys.argv[1]
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda", 0)
    ctx = gpu.CrcContext(0)

    def u64t(a):
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)

    if name in ("C", "Cu"):
        lengths = synth.ragged_lengths(synth.SEED_C, GOLD["C"]["count"])
        offsets, total = synth.packed_offsets(lengths, 1 if name == "Cu" else 64)
        buf = torch.empty(total + 64, dtype=torch.uint8, device=dev)
        d_off, d_len = u64t(offsets), u64t(lengths)
        gpu.fill_ragged(buf, d_off, d_len, seed=synth.SEED_C)
        out = torch.empty(len(lengths), dtype=torch.int32, device=dev)
        fn, nbytes = (lambda: ctx.crc32_ragged(buf, d_off, d_len, out)), int(lengths.sum())
    elif name in ("D", "Du"):
        n, L = GOLD["D"]["count"], 64 << 20
        buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
        gpu.fill_uniform(buf, L, L, n, seed=synth.SEED_D)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        if name == "D":
            d_off = u64t(np.arange(n, dtype=np.uint64) * np.uint64(L))
            d_len = u64t(np.full(n, L, dtype=np.uint64))
            fn = lambda: ctx.crc32_ragged(buf, d_off, d_len, out)  # noqa: E731
        else:
            fn = lambda: ctx.crc32_uniform(buf, L, L, n, out)  # noqa: E731
        nbytes = n * L
    elif name == "Usmall":  # bench.py small_uniform_config: 1 Mi x 256 B, 4 rotated batches
        n, L = 1 << 20, 256
        bufs = [torch.empty(n * L, dtype=torch.uint8, device=dev) for _ in range(4)]
        for k, b in enumerate(bufs):
            gpu.fill_uniform(b, L, L, n, seed=0x5EED0256 + k)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        i = [0]

        def fn():
            ctx.crc32_uniform(bufs[i[0] % 4], L, L, n, out)
            i[0] += 1
        nbytes = n * L
    elif name in ("S_short", "S_mixed"):  # bench.py short_slots_config: 256-B / 1..4096-B messages in 4 KiB slots
        n, area, L, cs = 65536, 4096, 256, 4
        ps, stride = slots.compute_prefix_size(cs, 0), slots.slot_stride(area, cs, 0)
        mixed = name == "S_mixed"
        rng = np.random.default_rng(0x5EED0258 if mixed else 0x5EED0257)
        sizes = rng.integers(1, area + 1, n).astype(np.uint64) if mixed else np.full(n, L, dtype=np.uint64)
        host = rng.integers(0, 256, stride * n, dtype=np.uint8)
        host.reshape(n, stride)[:, :ps] = slots.make_prefixes(n, sizes, checksum_size=cs, metadata_size=0, seed=7)
        bufs = [torch.from_numpy(host).to(dev) for _ in range(4)]
        order = rng.permutation(n).astype(np.uint64)
        recs = []
        for b in bufs:
            b0 = np.uint64(b.data_ptr())
            r = np.stack([b0 + order * np.uint64(stride), b0 + order * np.uint64(stride) + np.uint64(ps),
                          sizes[order.astype(np.int64)]], axis=1)
            recs.append(torch.from_numpy(np.ascontiguousarray(r).view(np.int64)).to(dev))
        status = torch.empty(n, dtype=torch.int32, device=dev)
        errs = torch.zeros(1, dtype=torch.int32, device=dev)
        i = [0]

        def fn():
            ctx.crc32_slots(recs[i[0] % 4], max_message_size=area, checksum_size=cs, metadata_size=0,
                            mode=gpu.SLOT_VERIFY, status=status, error_count=errs)
            i[0] += 1
        nbytes = int(sizes.sum()) + 44 * n
    elif name.startswith("S_large"):  # bench.py large_slots_config: 32 KiB slots, 1..32,767-B payloads
        n, area, cs = 65536, 32768, 4
        ps, stride = slots.compute_prefix_size(cs, 0), slots.slot_stride(area, cs, 0)
        rng = np.random.default_rng(0x5EED0259)
        sizes = rng.integers(1, area, n).astype(np.uint64)
        d_sizes = torch.from_numpy(sizes.view(np.int64)).to(dev)
        d_pre = torch.from_numpy(slots.make_prefixes(n, sizes, checksum_size=cs, metadata_size=0, seed=9)).to(dev)
        d_offs = u64t(np.arange(n, dtype=np.uint64) * np.uint64(stride) + np.uint64(ps))
        bufs = []
        for k in range(4):
            b = torch.empty(n * stride, dtype=torch.uint8, device=dev)
            b.view(n, stride)[:, :ps] = d_pre
            gpu.fill_ragged(b, d_offs, d_sizes, seed=0x5EED0259 + k)
            bufs.append(b)
        order = rng.permutation(n).astype(np.uint64)
        recs = []
        for b in bufs:
            b0 = np.uint64(b.data_ptr())
            r = np.stack([b0 + order * np.uint64(stride), b0 + order * np.uint64(stride) + np.uint64(ps),
                          sizes[order.astype(np.int64)]], axis=1)
            recs.append(torch.from_numpy(np.ascontiguousarray(r).view(np.int64)).to(dev))
        status = torch.empty(n, dtype=torch.int32, device=dev)
        errs = torch.zeros(1, dtype=torch.int32, device=dev)
        mode = gpu.SLOT_CALCULATE if name.endswith("publish") else gpu.SLOT_VERIFY
        i = [0]

        def fn():
            ctx.crc32_slots(recs[i[0] % 4], max_message_size=area, checksum_size=cs, metadata_size=0, mode=mode,
                            status=status, error_count=errs if mode == gpu.SLOT_VERIFY else None)
            i[0] += 1
        nbytes = int(sizes.sum()) + 44 * n
    else:  # config S's slots (bench.py slot_configs): 65,536 x 4 KiB payloads, 4 rotated copies
        n, size, cs = 65536, 4096, 4
        ms_ = 16 if name.startswith("S_meta") else 0
        ps, stride = slots.compute_prefix_size(cs, ms_), slots.slot_stride(size, cs, ms_)
        rng = np.random.default_rng(0x5EED0005)
        host = rng.integers(0, 256, stride * n, dtype=np.uint8)
        host.reshape(n, stride)[:, :ps] = slots.make_prefixes(n, np.full(n, size, dtype=np.uint64), checksum_size=cs,
                                                              metadata_size=ms_, seed=5)
        bufs = [torch.from_numpy(host).to(dev) for _ in range(4)]
        status = torch.empty(n, dtype=torch.int32, device=dev)
        errs = torch.zeros(1, dtype=torch.int32, device=dev)
        mode = gpu.SLOT_CALCULATE if name.endswith("publish") else gpu.SLOT_VERIFY
        i = [0]
        if name.startswith("S_list"):
            order = rng.permutation(n).astype(np.uint64)
            recs = []
            for b in bufs:
                b0 = np.uint64(b.data_ptr())
                r = np.stack([b0 + order * np.uint64(stride), b0 + order * np.uint64(stride) + np.uint64(ps),
                              np.full(n, size, dtype=np.uint64)], axis=1)
                recs.append(torch.from_numpy(np.ascontiguousarray(r).view(np.int64)).to(dev))

            def fn():
                ctx.crc32_slots(recs[i[0] % 4], max_message_size=size, checksum_size=cs, metadata_size=ms_, mode=mode,
                                status=status, error_count=errs if mode == gpu.SLOT_VERIFY else None)
                i[0] += 1
        else:
            def fn():
                ctx.crc32_slots_strided(bufs[i[0] % 4], stride, n, message_size=size, checksum_size=cs,
                                        metadata_size=ms_, mode=mode, status=status if mode == gpu.SLOT_VERIFY else None,
                                        error_count=errs if mode == gpu.SLOT_VERIFY else None)
                i[0] += 1
        nbytes = n * (size + 44 + ms_)
    torch.cuda.synchronize()
    for _ in range(calls):
        fn()
    torch.cuda.synchronize()
    print(json.dumps({"config": name, "calls": calls, "algorithmic_bytes_per_call": nbytes}))
    ctx.close()


if __name__ == "__main__":
    main()
