#!/usr/bin/env python3
"""Headline benchmark: device-resident batched CRC32 on MI355X.

Workload (BASELINE.json configs[1], "config B"): 65,536 independent 4 KiB payloads,
one CRC32 each, bit-exact with the reference's client/checksum.cc. One step = one
launch of the batched kernel over one 256 MiB batch already resident in HBM. Four
distinct batches are rotated so the 256 MiB Infinity Cache cannot serve re-reads
(every step reads HBM). The payloads are synthetic (SURVEY.md 8d generator),
generated on device before timing.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...    (one rank per GPU, weak scaling:
                                                        every rank checksums its own
                                                        65,536-message shard per step)

Prints ONE JSON line (rank 0). `value` = aggregate GiB/s over all ranks (bytes of all
ranks / max-over-ranks time). `roofline` is for the CRC kernel itself (one HIP event
pair around the K launches on their stream, / K; algorithmic bytes = 65,536 x 4,096 per
launch).
`cpu_baseline` times the oracle (a C restatement of the reference table path) on this
host's cores over a bounded sample of the same batches.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "GiB/s CRC32 over batched payloads (device-resident); % of HBM3E read peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md chip table
MSGS, MSG_BYTES = 65536, 4096
BATCH_BYTES = MSGS * MSG_BYTES
ROTATE = 4  # 4 x 256 MiB > the 256 MiB Infinity Cache: every step reads HBM


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    # After an idle spell the first ~300 back-to-back launches of this kernel run up to 25 %
    # slower while the GPU's power management settles (profiles/r01/sustained.md). Before
    # the W warm-up steps the bench runs untimed settle launches until SETTLE launches have
    # run in all; reported as "settle_launches" (0 disables).
    ap.add_argument("--settle", type=int, default=400)
    # --streams 2: consecutive steps alternate between two HIP streams (independent batches)
    # and overlap (45.2 vs 46.7 us per launch in profiles/r01/ceiling.md). Off by default:
    # overlapping dispatches make rocprofv3's per-dispatch duration (~2x, both kernels
    # resident) disagree with the roofline's per-launch interval.
    ap.add_argument("--streams", type=int, default=1, choices=[1, 2])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="budget for the CPU baseline legs")
    ap.add_argument("--event-every", type=int, default=0,
                    help="0 (default): one HIP event pair around the whole timed region, launch duration = "
                         "region / K (an event record between launches costs ~9 us per step on MI355X); "
                         "N > 0: also bracket every N-th launch (perturbs the timed region)")
    ap.add_argument("--workload", default="B", choices=["B", "C", "E"],
                    help="B: 65,536 x 4 KiB per GPU per step (weak scaling, default); "
                         "C: 1 Mi ragged messages 64 B - 1 MiB (117.8 GB) in contiguous shards balanced by "
                         "bytes (strong scaling) + RCCL gather; "
                         "E: 8 Mi x 4 KiB sharded round-robin over the GPUs (strong scaling) + RCCL gather")
    return ap.parse_args()


def cpu_baseline(batches_host: list[np.ndarray], seconds: float) -> dict:
    """Oracle (reference table path restated in C) on this host's cores."""
    sys.path.insert(0, str(ROOT / "tests"))
    import _oracle
    orc = _oracle.load()
    offs = np.arange(MSGS, dtype=np.uint64) * np.uint64(MSG_BYTES)
    lens = np.full(MSGS, MSG_BYTES, dtype=np.uint64)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))

    def rate(nthreads, budget):
        done, t0 = 0, time.perf_counter()
        i = 0
        while True:
            orc.crc32_batch(batches_host[i % len(batches_host)], offs, lens, threads=nthreads)
            done += BATCH_BYTES
            i += 1
            if time.perf_counter() - t0 >= budget:
                break
        return done / (time.perf_counter() - t0) / 2**30, done

    r1, b1 = rate(1, seconds / 2)
    rn, bn = rate(threads, seconds / 2)
    sse = None
    if orc.has_sse42():  # informational: the reference's -msse4.2 path computes CRC-32C
        done, t0, i = 0, time.perf_counter(), 0
        while time.perf_counter() - t0 < min(1.0, seconds / 4):
            orc.crc32c_sse42_batch(batches_host[i % len(batches_host)], offs, lens, threads=threads)
            done += BATCH_BYTES
            i += 1
        sse = round(done / (time.perf_counter() - t0) / 2**30, 3)
    # informational: the library's own host SubspaceCRC32 (PCLMULQDQ body) on one core, over
    # whole 256 MiB batches (per-message calls would time Python's call overhead instead)
    from subspace_amd import checksum
    done, t0, i = 0, time.perf_counter(), 0
    while time.perf_counter() - t0 < min(1.0, seconds / 4):
        checksum.subspace_crc32(0xFFFFFFFF, batches_host[i % len(batches_host)])
        done += BATCH_BYTES
        i += 1
    dropin = round(done / (time.perf_counter() - t0) / 2**30, 3)
    config_a = None  # BASELINE configs[0]: the per-message CPU path (tools/config_a.cpp)
    exe = ROOT / "tools" / "config_a"
    if exe.exists():
        import subprocess
        try:
            r = subprocess.run([str(exe), "20000", str(ROOT / "oracle" / "liboracle_crc.so")], capture_output=True,
                               text=True, timeout=120)
            config_a = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else None
        except (subprocess.SubprocessError, ValueError, IndexError):
            config_a = None
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(rn, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "value_1core": round(r1, 3),
            "sse42_crc32c_value": sse,
            "dropin_host_1core_value": dropin,
            "dropin_host_note": "libsubspace_crc.so's host SubspaceCRC32 (bit-exact IEEE; PCLMULQDQ folding) on one "
                                "core over the same batches; informational",
            "config_a": config_a,
            "sse42_crc32c_note": "client/checksum.cc:56-76 (-msse4.2 builds) restated on the same batches and "
                                 "threads: CRC-32C, NOT bit-exact with the IEEE parity path; informational",
            "sample": f"config-B batches (65,536 x 4 KiB, host copies of the device batches): "
                      f"{bn / 2**30:.2f} GiB on {threads} threads, {b1 / 2**30:.2f} GiB on 1 thread; "
                      f"oracle/crc32_oracle.c byte-table loop (reference client/checksum.cc:125-130), "
                      f"gcc -O2, CPU: {cpu_model}"}


def end_to_end(ctx, gpu) -> dict:
    from subspace_amd import slots
    stride = slots.slot_stride(MSG_BYTES)  # PrefixSize(64) + Aligned64(4096) = 4160
    rng = np.random.default_rng(0x5EED00A)
    host = rng.integers(0, 256, MSGS * stride, dtype=np.uint8)
    host.reshape(MSGS, stride)[:, :64] = slots.make_prefixes(MSGS, np.full(MSGS, MSG_BYTES, dtype=np.uint64), seed=1)
    gpu.host_register(host)
    try:
        def rate(mode, n=5):
            ctx.crc32_host_slots(host, stride, MSGS, message_size=MSG_BYTES, mode=mode)  # warm
            ts = []
            for _ in range(n):
                t = time.perf_counter()
                errors = ctx.crc32_host_slots(host, stride, MSGS, message_size=MSG_BYTES, mode=mode)
                ts.append(time.perf_counter() - t)
                assert errors == 0
            return sorted(ts)[n // 2]
        t_pub = rate(gpu.SLOT_CALCULATE)
        t_ver = rate(gpu.SLOT_VERIFY)
        # the subscriber drain hook: the same slots as a record list (host addresses, here
        # in shuffled order), read in place over PCIe through the registered mapping
        base = host.ctypes.data
        order = rng.permutation(MSGS).astype(np.uint64)
        recs = slots.slot_records(base + order * np.uint64(stride), base + order * np.uint64(stride) + np.uint64(64),
                                  np.full(MSGS, MSG_BYTES, dtype=np.uint64))
        ctx.crc32_host_slot_list(recs, max_message_size=MSG_BYTES, mode=gpu.SLOT_VERIFY)  # warm
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            errors = ctx.crc32_host_slot_list(recs, max_message_size=MSG_BYTES, mode=gpu.SLOT_VERIFY)
            ts.append(time.perf_counter() - t)
            assert errors == 0
        t_drain = sorted(ts)[2]
    finally:
        gpu.host_unregister(host)
    return {"value": round(BATCH_BYTES / t_pub / 2**30, 2), "unit": "GiB/s",
            "verify_value": round(BATCH_BYTES / t_ver / 2**30, 2),
            "drain_hook_verify_value": round(BATCH_BYTES / t_drain / 2**30, 2),
            "slot_bytes_GBps": round(MSGS * stride / t_pub / 1e9, 2),
            "path": "subspace_crc32_host_slots: 65,536 pinned host slots (stride 4,160) -> chunked H2D "
                    "overlapping the kernels -> 4 B per slot D2H -> flag + checksum written into each host "
                    "prefix (publish); value = payload GiB/s, median of 5 calls; drain_hook_verify_value: "
                    "subspace_crc32_host_slot_list over the same slots as shuffled host-address records, read "
                    "zero-copy over PCIe"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from subspace_amd import gpu

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    if world > 1:
        torch.cuda.set_device(local)
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    ctx = gpu.CrcContext(local)
    stream = torch.cuda.current_stream()

    from subspace_amd import shard

    # ---- inputs. B: ROTATE distinct 256 MiB batches per rank (message ids r, r+world, ...).
    #      E: this rank's round-robin shard of the 8 Mi-message batch, one buffer.
    bufs, outs = [], []
    if args.workload == "B":
        nmsg, nbuf = MSGS, ROTATE
        for k in range(nbuf):
            b = torch.empty(nmsg * MSG_BYTES, dtype=torch.uint8, device=dev)
            gpu.fill_uniform(b, MSG_BYTES, MSG_BYTES, nmsg, seed=0x5EED000B, first_id=rank + k * nmsg * world,
                             id_stride=world)
            bufs.append(b)
            outs.append(torch.empty(nmsg, dtype=torch.int32, device=dev))
    elif args.workload == "C":
        # this rank's contiguous, byte-balanced range of config C (one ragged call per step)
        from subspace_amd import synth
        goldens_c = json.loads((ROOT / "tests" / "golden" / "configs.json").read_text())["C"]
        lengths_c = synth.ragged_lengths(synth.SEED_C, goldens_c["count"])
        bounds_c = shard.ragged_ranges(lengths_c, world)
        lo, hi = int(bounds_c[rank]), int(bounds_c[rank + 1])
        local_len = lengths_c[lo:hi]
        offs_c, arena_c = synth.packed_offsets(local_len, 64)
        nmsg, nbuf = hi - lo, 1
        b = torch.empty(int(arena_c) + 64, dtype=torch.uint8, device=dev)
        d_off_c = torch.from_numpy(offs_c.astype(np.int64)).to(dev)
        d_len_c = torch.from_numpy(local_len.astype(np.int64)).to(dev)
        if nmsg:
            gpu.fill_ragged(b, d_off_c, d_len_c, seed=synth.SEED_C, first_id=lo)
        bufs.append(b)
        outs.append(torch.empty(max(nmsg, 1), dtype=torch.int32, device=dev))
        c_total_bytes = int(lengths_c.sum())
    else:
        total_e = 8 << 20
        nmsg, nbuf = shard.shard_count(total_e, rank, world), 1
        b = torch.empty(nmsg * MSG_BYTES, dtype=torch.uint8, device=dev)
        gpu.fill_uniform(b, MSG_BYTES, MSG_BYTES, nmsg, seed=0x5EED000E, first_id=rank, id_stride=world)
        bufs.append(b)
        outs.append(torch.empty(nmsg, dtype=torch.int32, device=dev))
    step_bytes = int(local_len.sum()) if args.workload == "C" else nmsg * MSG_BYTES
    torch.cuda.synchronize()

    if nbuf % args.streams:  # workload E has one buffer: its steps stay on one stream
        args.streams = 1
    streams = [stream] + [torch.cuda.Stream() for _ in range(args.streams - 1)]
    for s2 in streams[1:]:
        s2.wait_stream(stream)

    def step(i):
        # batch i % nbuf always runs on stream i % len(streams): nbuf is a multiple of the
        # stream count, so a batch's buffers are only ever used in order on one stream
        k = i % nbuf
        if args.workload == "C":
            if nmsg:
                ctx.crc32_ragged(bufs[0], d_off_c, d_len_c, outs[0], stream=streams[0])
            return
        ctx.crc32_uniform(bufs[k], MSG_BYTES, MSG_BYTES, nmsg, outs[k], stream=streams[i % len(streams)])

    settle = max(0, args.settle - args.warmup)
    for i in range(settle):
        step(i)
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()

    # ---- timed region: K steps, barrier + sync on both sides, max over ranks
    every = args.event_every
    ev = {i: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for i in range(0, args.steps, every)} if every > 0 else {}
    region = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    region[0].record(stream)
    for s2 in streams[1:]:
        s2.wait_stream(stream)  # every stream starts after the region's first event
    for i in range(args.steps):
        e = ev.get(i)
        if e:
            e[0].record(stream)
        step(i)
        if e:
            e[1].record(stream)
    for s2 in streams[1:]:
        stream.wait_stream(s2)  # ... and the last event after every stream's last launch
    region[1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # Launch interval of the CRC kernel: the HIP-event span of the K back-to-back launches /
    # K (events on the first stream, joined with the second). With two streams consecutive
    # launches overlap, so this effective interval is shorter than rocprofv3's per-dispatch
    # duration (which then counts the overlapped part twice); with one stream it includes
    # the inter-launch gaps.
    avg_kern_ms = region[0].elapsed_time(region[1]) / args.steps
    sampled_ms = float(np.mean([a.elapsed_time(b) for a, b in ev.values()])) if ev else None

    # ---- bit-exactness of what was timed. B at world 1: batch 0 is exactly config B.
    #      E: gather every rank's CRCs to rank 0 over RCCL (timed separately) and compare the
    #      whole 8 Mi list with the fixture.
    goldens = json.loads((ROOT / "tests" / "golden" / "configs.json").read_text())
    bitexact, gather_ms = None, None
    if args.workload == "B" and world == 1:
        crc0 = outs[0].cpu().numpy().view(np.uint32)
        bitexact = hashlib.sha256(crc0.astype("<u4").tobytes()).hexdigest() == goldens["B"]["sha256_le_u32"]
    if args.workload == "C":
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        if world > 1:
            full = shard.gather_ragged_crcs(outs[0][:nmsg], bounds_c, rank, world, dist)
        else:
            full = outs[0][:nmsg].cpu().numpy().view(np.uint32)
        gather_ms = (time.perf_counter() - tg) * 1e3
        if rank == 0:
            bitexact = hashlib.sha256(np.asarray(full, dtype="<u4").tobytes()).hexdigest() == \
                goldens["C"]["sha256_le_u32"]
    if args.workload == "E":
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        if world > 1:
            full = shard.gather_crcs(outs[0], 8 << 20, rank, world, dist)
        else:
            full = outs[0].cpu().numpy().view(np.uint32)
        gather_ms = (time.perf_counter() - tg) * 1e3
        if rank == 0:
            bitexact = hashlib.sha256(np.asarray(full, dtype="<u4").tobytes()).hexdigest() == \
                goldens["E"]["sha256_le_u32"]

    # ---- end-to-end from host shared-memory slots (not `value`): config B in the reference's
    #      channel layout (65,536 slots of PrefixSize 64 + 4 KiB, stride 4,160) in pinned host
    #      memory; subspace_crc32_host_slots streams it to the GPU in ~32 MiB chunks (copies
    #      overlap kernels) and writes flag + checksum back into every host prefix.
    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e and args.workload == "B":
        e2e = end_to_end(ctx, gpu)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "B":
        cpu = cpu_baseline([b.cpu().numpy() for b in bufs], args.cpu_seconds)

    traffic = None
    # PMC-measured HBM bytes per config-B launch (tools/summarize_profile.py); other
    # workloads' launches are a different size, so no figure for them
    tfile = ROOT / "profiles" / "traffic_uniform4k.json"
    if tfile.exists() and args.workload == "B":
        try:
            traffic = json.loads(tfile.read_text()).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if rank == 0:
        if args.workload == "B":
            total_bytes = step_bytes * args.steps * world  # every rank: its own 65,536-message batch
            workload = {"workload": "B: 65,536 x 4 KiB payloads per GPU per step, one CRC32 (IEEE, "
                                    "client/checksum.cc default build) each", "messages_per_gpu": nmsg,
                        "message_bytes": MSG_BYTES, "batches_rotated": ROTATE,
                        "parallelism": f"independent message shards x{world}", "streams": args.streams}
            scaling = "weak"
        elif args.workload == "C":
            total_bytes = c_total_bytes * args.steps  # the whole 1 Mi-message batch per step
            workload = {"workload": "C: 1 Mi messages, 64 B - 1 MiB log-uniform (117.8 GB), one CRC32 each, "
                                    "contiguous shards balanced by bytes", "messages_total": int(bounds_c[-1]),
                        "messages_rank0": nmsg, "bytes_total": c_total_bytes,
                        "parallelism": f"contiguous byte-balanced shards x{world}, RCCL all_gather of CRCs "
                                       "(untimed)",
                        "gather_ms": round(gather_ms, 3) if gather_ms is not None else None}
            scaling = "strong"
        else:
            total_bytes = (8 << 20) * MSG_BYTES * args.steps  # the whole 8 Mi batch per step
            workload = {"workload": "E: 8 Mi x 4 KiB payloads per step, round-robin over the GPUs, one CRC32 each",
                        "messages_total": 8 << 20, "messages_per_gpu": nmsg, "message_bytes": MSG_BYTES,
                        "parallelism": f"round-robin message shards x{world}, RCCL all_gather of CRCs (untimed)",
                        "gather_ms": round(gather_ms, 3) if gather_ms is not None else None,
                        # the same rate with one gather of every step's CRCs to rank 0 added per step
                        "value_incl_gather": round(total_bytes / (elapsed + args.steps * gather_ms * 1e-3) / 2**30, 2)
                        if gather_ms is not None else None}
            scaling = "strong"
        value = total_bytes / elapsed / 2**30
        achieved = step_bytes / (avg_kern_ms * 1e-3) / 1e9
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_launches": settle,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (deterministic splitmix64 payloads generated on device"
                    + ("; 4 rotated 256 MiB batches per GPU)" if args.workload == "B" else ")"),
            "config": workload,
            "pct_of_hbm_peak": round(100.0 * value * 2**30 / 1e9 / (HBM_PEAK_GBS * world), 2),
            "bitexact_vs_golden": bitexact,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "subspace_amd::crc32_ragged_kernel<512> + prep (whole call)" if args.workload == "C"
                         else "subspace_amd::crc32_uniform4k_kernel<512>", "avg_launch_ms": round(avg_kern_ms, 4),
                         "launch_ms_source": f"HIP event span of the timed region / K ({args.streams} stream(s), "
                                             "consecutive launches overlap when 2)",
                         "sampled_launch_ms": round(sampled_ms, 4) if sampled_ms else None},
            "cpu_baseline": cpu,
            "e2e_pcie": e2e,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
