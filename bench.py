#!/usr/bin/env python3
"""Headline benchmark: device-resident batched CRC32 on MI355X.

Workload at N = 1 (BASELINE.json configs[1], "config B"): 65,536 independent 4 KiB
payloads, one CRC32 each, bit-exact with the reference's client/checksum.cc. One step =
one launch of the batched kernel over one 256 MiB batch already resident in HBM. Four
distinct batches are rotated so the 256 MiB Infinity Cache cannot serve re-reads (every
step reads HBM). Payloads are synthetic (SURVEY.md 8d generator), generated on device
before timing. The same run also times configs C (1 Mi ragged messages), D (256 x 64 MiB,
ragged and uniform API) and S (config B in the reference's slot layout: publish and
verify), each checked bit-exact, under "configs".

Workload at N > 1 (BASELINE.json configs[4], "config E"): 8 Mi x 4 KiB payloads sharded
round-robin over the GPUs (strong scaling), one RCCL all_gather of the 4-byte CRCs after
the timed region (timed separately), the whole list checked against the fixture; rank 0
then times the same 8 Mi batch alone on its GPU, and the line reports per-GPU value and
efficiency = value / (N x that single-GPU rate).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload B|C|E]
      With N > 1 and no WORLD_SIZE in the environment, this process only spawns N ranks
      (python -m torch.distributed.run, one process per GPU, RCCL) and exits with their
      status; it never touches a GPU itself.
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
      The driver's form: WORLD_SIZE must equal --gpus (exit 2 otherwise).
  python bench.py --gpus N --dry-run-cpu [--workload E|C|B]
      The same spawn, shard, time and gather code on the CPU (gloo; each rank checksums its
      shard with the library's host SubspaceCRC32 instead of the kernel) over small fixture
      batches (E -> config B's 65,536 messages round-robin, C -> the first 2,048 messages
      of C in byte-balanced ranges), checked against the fixture hash. For tests.

Prints ONE JSON line (rank 0). `value` = aggregate GiB/s over all ranks (bytes of all ranks
/ max-over-ranks time between barriers). `roofline` is for the dominant kernel (one HIP
event pair around the K launches on their stream, / K). `cpu_baseline` times the oracle
(a C restatement of the reference table path) on this host's cores over bounded samples
of configs B, C, D and E (median of 5 runs each, 1 core and all cores available to the
job).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
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
E_COUNT = 8 << 20
GOLD = json.loads((ROOT / "tests" / "golden" / "configs.json").read_text())


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    # After an idle spell the first ~300 back-to-back launches of this kernel run up to 25 %
    # slower while the GPU's power management settles (profiles/r01/sustained.md). Before
    # the W warm-up steps the bench runs untimed settle launches until SETTLE launches have
    # run in all and at least SETTLE_S seconds have passed: a fresh box's first GPU process ran
    # config B at 5,368 GiB/s after 380 settle launches (r02c25) and 5,374 after 1 s of them
    # (r02c27), 5,583 after 0.9 s on another box (r02c26) and 5,550 after 5 s (r02c28), later
    # processes 5,520-5,583; reported as "settle_launches" (--settle 0 disables both). 8 s: a
    # large VRAM free by an earlier process (a test run's 118 GB) is wiped in the background
    # for 4-8 s, slowing every HBM-bound kernel 2-4 % (profiles/DESIGN_r01-r03.md 6, profiles/r03/wipe).
    ap.add_argument("--settle", type=int, default=400)
    ap.add_argument("--settle-s", type=float, default=8.0)
    # --streams 2: consecutive steps alternate between two HIP streams (independent batches)
    # and overlap (45.2 vs 46.7 us per launch in profiles/r01/ceiling.md). Off by default:
    # overlapping dispatches make rocprofv3's per-dispatch duration (~2x, both kernels
    # resident) disagree with the roofline's per-launch interval.
    ap.add_argument("--streams", type=int, default=1, choices=[1, 2])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-runs", type=int, default=5, help="CPU baseline: runs per sample (median reported)")
    ap.add_argument("--event-every", type=int, default=0,
                    help="0 (default): one HIP event pair around the whole timed region, launch duration = "
                         "region / K (an event record between launches costs ~9 us per step on MI355X); "
                         "N > 0: also bracket every N-th launch (perturbs the timed region)")
    ap.add_argument("--roctx-region", action="store_true",
                    help="bracket exactly the timed region with roctxProfilerResume/Pause, so that "
                         "`rocprofv3 --selected-regions` records only the K timed launches")
    ap.add_argument("--workload", default=None, choices=["B", "C", "E"],
                    help="default B at 1 GPU, E at N > 1. "
                         "B: 65,536 x 4 KiB per GPU per step (weak scaling); "
                         "C: 1 Mi ragged messages 64 B - 1 MiB (117.8 GB) in contiguous shards balanced by "
                         "bytes (strong scaling) + RCCL gather; "
                         "E: 8 Mi x 4 KiB sharded round-robin over the GPUs (strong scaling) + RCCL gather")
    ap.add_argument("--configs", default=None,
                    help="secondary configs timed after the headline at N = 1 (comma list of C, Cu, D, Du, S, "
                         "Usmall, S_short, S_mixed, S_large; default C,Cu,D,Du,S,Usmall,S_short,S_mixed,S_large with workload B, none otherwise; "
                         "'none' disables)")
    ap.add_argument("--config-iters", type=int, default=20)
    ap.add_argument("--no-solo", action="store_true", help="N > 1: skip rank 0's single-GPU reference leg")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N > 1 on a one-GPU machine: every rank on cuda:0, gloo instead of RCCL -- the GPU "
                         "workload, timing, gather and single-GPU legs of a multi-GPU run, for tests (the ranks "
                         "share one GPU, so the rates are not scaling numbers)")
    ap.add_argument("--print-rank-env", action="store_true",
                    help="each rank prints the launch environment it got (one JSON line) and exits, for tests")
    ap.add_argument("--dry-run-cpu", action="store_true",
                    help="CPU + gloo rehearsal of the spawn/shard/gather path (host SubspaceCRC32), for tests")
    return ap.parse_args()


def die(msg: str, code: int = 2):
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)
    sys.exit(code)


# ------------------------------------------------------------------------------ launch
def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# Environment every rank runs with, whichever way it was started (the driver's own
# `torch.distributed.run ... bench.py`, or this script spawning its ranks): applied by
# apply_rank_env() at the top of main(), before torch is imported or any HIP call is made --
# ROCm reads HSA_ENABLE_IPC_MODE_LEGACY when HIP initialises (the host driver supports dmabuf
# IPC only, which RCCL's cross-process buffers need), so setting it later has no effect
# (it used to be set after torch.cuda.device_count() in the driver's form).
RANK_ENV_DEFAULTS = {"HSA_ENABLE_IPC_MODE_LEGACY": "0"}
RANK_ENV_REPORTED = ("HSA_ENABLE_IPC_MODE_LEGACY", "OMP_NUM_THREADS", "WORLD_SIZE", "LOCAL_WORLD_SIZE",
                     "MASTER_ADDR")


def apply_rank_env() -> None:
    for k, v in RANK_ENV_DEFAULTS.items():
        os.environ.setdefault(k, v)


def spawn_ranks(args) -> int:
    """--gpus N > 1 without a launcher: start N rank processes (one per GPU) through
    torch.distributed.run as a child and return its exit status. This process never
    initialises a GPU (no exec from a GPU-initialised process). The ranks get the same
    environment as under the driver's own launch (apply_rank_env; tests/test_bench_launch.py)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(Path(__file__).resolve()),
           *sys.argv[1:]]
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def digest(crcs) -> str:
    return hashlib.sha256(np.asarray(crcs, dtype="<u4").tobytes()).hexdigest()


# ------------------------------------------------------------------------------ CPU baseline
def cpu_share() -> dict:
    """Cores this job may use: the process affinity set, limited to the job's CPU share
    where the environment states one (OMP_NUM_THREADS: 16 per GPU on the gpurun boxes,
    whose nproc shows the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    share = int(omp) if omp and omp.isdigit() and int(omp) > 0 else aff
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"cores": max(1, min(aff, share)), "nproc": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": omp, "cpu_model": cpu_model}


def cpu_samples(dev, bufs_b) -> dict:
    """Host copies of bounded samples of configs B, C, D and E (the same generator as the
    device batches): name -> (arena, offsets, lengths, description)."""
    import torch
    from subspace_amd import gpu, synth
    out = {}
    offs = np.arange(MSGS, dtype=np.uint64) * np.uint64(MSG_BYTES)
    lens = np.full(MSGS, MSG_BYTES, dtype=np.uint64)
    out["B"] = (bufs_b[0].cpu().numpy(), offs, lens, "config B's batch 0 (65,536 x 4 KiB, 256 MiB)")
    # C: the first messages of config C up to 256 MiB, 64-B aligned packing as in the GPU run
    lc = synth.ragged_lengths(synth.SEED_C, 4096)
    k = int(np.searchsorted(np.cumsum(lc, dtype=np.uint64), np.uint64(256 << 20), side="right"))
    lc = lc[:k]
    oc, tot = synth.packed_offsets(lc, 64)
    b = torch.empty(tot + 64, dtype=torch.uint8, device=dev)
    gpu.fill_ragged(b, torch.from_numpy(oc.view(np.int64)).to(dev), torch.from_numpy(lc.view(np.int64)).to(dev),
                    seed=synth.SEED_C)
    out["C"] = (b.cpu().numpy(), oc, lc, f"config C's first {k:,} messages ({int(lc.sum()) / 2**20:.0f} MiB)")
    # D: 16 of the 256 x 64 MiB messages (one CRC per message is serial on a CPU, so the
    # all-core leg needs >= one message per worker; the 1-core leg times the first 4)
    b = torch.empty(16 << 26, dtype=torch.uint8, device=dev)
    gpu.fill_uniform(b, 64 << 20, 64 << 20, 16, seed=synth.SEED_D)
    out["D"] = (b.cpu().numpy(), np.arange(16, dtype=np.uint64) << np.uint64(26), np.full(16, 64 << 20, np.uint64),
                "config D's first 16 x 64 MiB messages (1-core leg: the first 4)")
    # E: 65,536 messages of shard 0 of 8 (ids 0, 8, 16, ...)
    b = torch.empty(BATCH_BYTES, dtype=torch.uint8, device=dev)
    gpu.fill_uniform(b, MSG_BYTES, MSG_BYTES, MSGS, seed=synth.SEED_E, first_id=0, id_stride=8)
    out["E"] = (b.cpu().numpy(), offs, lens, "65,536 messages of config E's shard 0 of 8 (256 MiB)")
    del b
    torch.cuda.empty_cache()
    return out


def cpu_baseline(samples: dict, runs: int) -> dict:
    """The oracle (reference table path restated in C) on this host's cores: per sample,
    the median of `runs` runs on 1 core and on all cores of the job's share (one pinned
    worker per core, round-robin message partition, sample pages first touched by their
    worker; BASELINE.md "CPU-baseline plan")."""
    sys.path.insert(0, str(ROOT / "tests"))
    import _oracle
    orc = _oracle.load()
    share = cpu_share()
    threads = share["cores"]
    per, pinned = {}, 0
    for name, (arena, offs, lens, desc) in samples.items():
        nbytes = int(lens.sum())
        ref = orc.crc32_batch(arena, offs, lens, threads=threads)
        k1 = min(len(offs), 4) if name == "D" else len(offs)  # 1-core leg: ~256 MiB
        bytes_1 = int(lens[:k1].sum())
        orc.crc32_batch_pinned(arena, offs[:k1], lens[:k1], threads=1)  # warm (page faults, clocks)
        t1 = []
        for _ in range(runs):
            t = time.perf_counter()
            got, _ = orc.crc32_batch_pinned(arena, offs[:k1], lens[:k1], threads=1)
            t1.append(time.perf_counter() - t)
        touched = orc.first_touch_copy(arena, offs, lens, threads)
        tn = []
        for _ in range(runs):
            t = time.perf_counter()
            got_n, pinned = orc.crc32_batch_pinned(touched, offs, lens, threads=threads)
            tn.append(time.perf_counter() - t)
        assert np.array_equal(got, ref[:k1]) and np.array_equal(got_n, ref)
        per[name] = {"bytes": nbytes, "sample": desc,
                     "value_1core": round(bytes_1 / float(np.median(t1)) / 2**30, 3),
                     "value_all_cores": round(nbytes / float(np.median(tn)) / 2**30, 3)}
        del touched
    arena_b, offs_b, lens_b, _ = samples["B"]
    # informational: config B's sample on every CPU of the affinity set (nproc may count a whole
    # machine shared with other jobs; BASELINE.md's plan says "all cores", `value` keeps the
    # job's share)
    all_aff = None
    aff = share["affinity_cpus"]
    if aff > threads:
        touched = orc.first_touch_copy(arena_b, offs_b, lens_b, aff)
        ta, pinned_a = [], 0
        for _ in range(runs):
            t = time.perf_counter()
            got_a, pinned_a = orc.crc32_batch_pinned(touched, offs_b, lens_b, threads=aff)
            ta.append(time.perf_counter() - t)
        del touched
        all_aff = {"value": round(BATCH_BYTES / float(np.median(ta)) / 2**30, 3), "threads": aff,
                   "workers_pinned": pinned_a, "bitexact": bool(np.array_equal(got_a, orc.crc32_batch(
                       arena_b, offs_b, lens_b, threads=threads))),
                   "note": "config B's sample, one pinned worker per CPU of the affinity set; informational "
                           "(the CPUs beyond the job's share belong to other jobs' GPUs on the gpurun boxes)"}
    sse = None
    if orc.has_sse42():  # informational: the reference's -msse4.2 path computes CRC-32C
        ts = []
        for _ in range(runs):
            t = time.perf_counter()
            orc.crc32c_sse42_batch(arena_b, offs_b, lens_b, threads=threads)
            ts.append(time.perf_counter() - t)
        sse = round(BATCH_BYTES / float(np.median(ts)) / 2**30, 3)
    # informational: the library's own host SubspaceCRC32 (carry-less folding body) on one core, over
    # the whole 256 MiB batch (per-message calls would time Python's call overhead instead)
    from subspace_amd import checksum
    ts = []
    for _ in range(runs):
        t = time.perf_counter()
        checksum.subspace_crc32(0xFFFFFFFF, arena_b)
        ts.append(time.perf_counter() - t)
    dropin = round(BATCH_BYTES / float(np.median(ts)) / 2**30, 3)
    config_a = None  # BASELINE configs[0]: the per-message CPU path (tools/config_a.cpp)
    exe = ROOT / "tools" / "config_a"
    if exe.exists():
        try:
            r = subprocess.run([str(exe), "20000", str(ROOT / "oracle" / "liboracle_crc.so")], capture_output=True,
                               text=True, timeout=120)
            config_a = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else None
        except (subprocess.SubprocessError, ValueError, IndexError):
            config_a = None
    return {"value": per["B"]["value_all_cores"], "unit": "GiB/s", "cores": threads, "kind": "port",
            "value_1core": per["B"]["value_1core"],
            "nproc": share["nproc"], "affinity_cpus": share["affinity_cpus"],
            "omp_num_threads": share["omp_num_threads"], "workers_pinned": pinned,
            "cores_note": "cores = the job's CPU share: the affinity set, limited by OMP_NUM_THREADS where set "
                          "(16 per GPU on the gpurun boxes, where nproc counts the whole machine)",
            "configs": per,
            "all_affinity_cpus": all_aff,
            "sse42_crc32c_value": sse,
            "sse42_crc32c_note": "client/checksum.cc:56-76 (-msse4.2 builds) restated on config B's sample and "
                                 "the same threads: CRC-32C, NOT bit-exact with the IEEE parity path; informational",
            "dropin_host_1core_value": dropin,
            "dropin_host_note": "libsubspace_crc.so's host SubspaceCRC32 (bit-exact IEEE; 4 x 512-bit VPCLMULQDQ "
                                "folding where the CPU has AVX-512 VPCLMULQDQ, else 4 x 128-bit PCLMULQDQ) on one "
                                "core over config B's sample; informational",
            "config_a": config_a,
            "sample": f"bounded samples of configs B, C, D, E (~256 MiB each, host copies of device-generated "
                      f"batches), median of {runs} runs each on 1 core and on {threads} pinned cores; "
                      f"oracle/crc32_oracle.c byte-table loop (reference client/checksum.cc:125-130), gcc -O2, "
                      f"CPU: {share['cpu_model']}; value = config B on all cores"}


# ------------------------------------------------------------------------------ end to end
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
    # the box's plain pinned H2D copy rate for the same bytes (the end-to-end path's bound)
    import torch
    pinned = torch.empty(MSGS * stride, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(MSGS * stride, dtype=torch.uint8, device="cuda")
    dst.copy_(pinned, non_blocking=True)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        dst.copy_(pinned, non_blocking=True)
    b.record()
    torch.cuda.synchronize()
    h2d = MSGS * stride * 5 / (a.elapsed_time(b) * 1e-3) / 1e9
    del pinned, dst
    return {"value": round(BATCH_BYTES / t_pub / 2**30, 2), "unit": "GiB/s",
            "verify_value": round(BATCH_BYTES / t_ver / 2**30, 2),
            "drain_hook_verify_value": round(BATCH_BYTES / t_drain / 2**30, 2),
            "slot_bytes_GBps": round(MSGS * stride / t_pub / 1e9, 2),
            "pcie_h2d_GBps": round(h2d, 2),
            "slot_bytes_frac_of_h2d": round(MSGS * stride / t_pub / 1e9 / h2d, 3),
            "path": "subspace_crc32_host_slots: 65,536 pinned host slots (stride 4,160) -> chunked H2D "
                    "overlapping the kernels -> 4 B per slot D2H -> flag + checksum written into each host "
                    "prefix (publish); value = payload GiB/s, median of 5 calls; drain_hook_verify_value: "
                    "subspace_crc32_host_slot_list over the same slots as shuffled host-address records, read "
                    "zero-copy over PCIe"}


# ------------------------------------------------------------------------------ workloads
class Workload:
    """One rank's share of a headline workload on its GPU: buffers, one step, the
    bit-exactness check. world/rank may differ from the job's (rank 0's solo leg)."""

    def __init__(self, name, ctx, dev, world, rank):
        import torch
        from subspace_amd import gpu, shard, synth
        self.name, self.ctx, self.world, self.rank = name, ctx, world, rank
        self.bufs, self.outs = [], []
        if name == "B":  # ROTATE distinct 256 MiB batches per rank (message ids r, r + world, ...)
            self.nmsg = MSGS
            for k in range(ROTATE):
                b = torch.empty(MSGS * MSG_BYTES, dtype=torch.uint8, device=dev)
                gpu.fill_uniform(b, MSG_BYTES, MSG_BYTES, MSGS, seed=synth.SEED_B, first_id=rank + k * MSGS * world,
                                 id_stride=world)
                self.bufs.append(b)
                self.outs.append(torch.empty(MSGS, dtype=torch.int32, device=dev))
            self.step_bytes = MSGS * MSG_BYTES
            self.total_bytes = self.step_bytes * world  # weak scaling: every rank its own batch
        elif name == "C":  # this rank's contiguous, byte-balanced range (one ragged call per step)
            lengths = synth.ragged_lengths(synth.SEED_C, GOLD["C"]["count"])
            self.bounds = shard.ragged_ranges(lengths, world)
            lo, hi = int(self.bounds[rank]), int(self.bounds[rank + 1])
            local = lengths[lo:hi]
            offs, arena = synth.packed_offsets(local, 64)
            self.nmsg = hi - lo
            b = torch.empty(int(arena) + 64, dtype=torch.uint8, device=dev)
            self.d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
            self.d_len = torch.from_numpy(local.astype(np.int64)).to(dev)
            if self.nmsg:
                gpu.fill_ragged(b, self.d_off, self.d_len, seed=synth.SEED_C, first_id=lo)
            self.bufs.append(b)
            self.outs.append(torch.empty(max(self.nmsg, 1), dtype=torch.int32, device=dev))
            self.step_bytes = int(local.sum())
            self.total_bytes = int(lengths.sum())
        else:  # E: this rank's round-robin shard of the 8 Mi-message batch, one buffer
            self.nmsg = shard.shard_count(E_COUNT, rank, world)
            b = torch.empty(self.nmsg * MSG_BYTES, dtype=torch.uint8, device=dev)
            gpu.fill_uniform(b, MSG_BYTES, MSG_BYTES, self.nmsg, seed=synth.SEED_E, first_id=rank, id_stride=world)
            self.bufs.append(b)
            self.outs.append(torch.empty(self.nmsg, dtype=torch.int32, device=dev))
            self.step_bytes = self.nmsg * MSG_BYTES
            self.total_bytes = E_COUNT * MSG_BYTES
        self.nbuf = len(self.bufs)

    def step(self, i, streams):
        # batch i % nbuf always runs on stream i % len(streams): nbuf is a multiple of the
        # stream count, so a batch's buffers are only ever used in order on one stream
        k = i % self.nbuf
        if self.name == "C":
            if self.nmsg:
                self.ctx.crc32_ragged(self.bufs[0], self.d_off, self.d_len, self.outs[0], stream=streams[0])
            return
        self.ctx.crc32_uniform(self.bufs[k], MSG_BYTES, MSG_BYTES, self.nmsg, self.outs[k],
                               stream=streams[i % len(streams)])

    def check(self, dist):
        """(bit-exact vs the fixture on rank 0, gather timing). Collective when world > 1: the
        4-byte CRCs of every rank are all_gathered (RCCL over xGMI) and put in global order on
        the device; HIP events on the current stream time exactly that (`gather_ms`, the device
        gather: the collective plus the on-device interleave, mean of 5 after an untimed first
        call; at world 1 one device copy). The
        D2H copy and the host hash check are timed apart (`d2h_check_ms`). B: each rank's
        batch 0 is a distinct id set, so at world 1 it is exactly config B."""
        import torch
        from subspace_amd import shard
        if self.name == "B":
            if self.world > 1:
                return None, None
            return digest(self.outs[0].cpu().numpy().view(np.uint32)) == GOLD["B"]["sha256_le_u32"], None
        def gather():
            if self.name == "C":
                return shard.gather_ragged_crcs_device(self.outs[0][:self.nmsg], self.bounds, self.world, dist)
            return shard.gather_crcs_device(self.outs[0], E_COUNT, self.world, dist)

        # one untimed gather first: its buffers' allocations and the collective's first-call
        # setup are host work the device would wait on inside the events (~20 ms at world 1)
        gather()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        reps = 5
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        ev[0].record()
        for _ in range(reps):
            full = gather()
        ev[1].record()
        torch.cuda.synchronize()
        gather_ms = ev[0].elapsed_time(ev[1]) / reps
        tc = time.perf_counter()
        ok = digest(full.cpu().numpy().view(np.uint32)) == GOLD[self.name]["sha256_le_u32"] if self.rank == 0 else None
        return ok, {"gather_ms": round(gather_ms, 4), "d2h_check_ms": round((time.perf_counter() - tc) * 1e3, 3),
                    "gather_bytes": int(full.numel()) * 4}

    def free(self):
        self.bufs, self.outs = [], []


class RoctxRegion:
    """roctxProfilerResume/Pause (librocprofiler-sdk-roctx) around the timed region, for
    `rocprofv3 --selected-regions`; a no-op unless --roctx-region."""

    def __init__(self, on: bool):
        self.lib = None
        if on:
            import ctypes
            self.lib = ctypes.CDLL("/opt/rocm/lib/librocprofiler-sdk-roctx.so")

    def resume(self):
        if self.lib:
            self.lib.roctxProfilerResume(0)

    def pause(self):
        if self.lib:
            self.lib.roctxProfilerPause(0)


SETTLE_CAP_S = 20.0


def launch_rate_steady(blocks, window_s=1.0, tol=0.003):
    """True when the last window_s seconds of (seconds, launches) blocks have a steady launch
    rate: the newer half's mean time per launch is not below the older half's by more than tol
    (still speeding up = not steady)."""
    win = []
    for blk in reversed(blocks):
        win.append(blk)
        if sum(x for x, _ in win) >= window_s:
            break
    total = sum(x for x, _ in win)
    if total < window_s:
        return False
    newer, acc = [], 0.0
    for blk in win:
        if acc >= total / 2:
            break
        acc += blk[0]
        newer.append(blk)
    older = win[len(newer):]
    if not older:
        return False
    per = lambda b: sum(x for x, _ in b) / sum(n for _, n in b)  # noqa: E731
    return per(newer) >= per(older) * (1.0 - tol)


def settle_steps(step, sync, settle, warmup, settle_s, block=50, cap_s=None):
    """Untimed settle launches before a timed region: at least `settle` - `warmup` of them and
    at least `settle_s` seconds of them, and, up to SETTLE_CAP_S, until the launch rate is
    steady (launch_rate_steady: the mean time per launch of the last 0.5 s within 0.3 % of the
    0.5 s before). VRAM freed to the driver (by this or an earlier process, e.g. a test run's
    118 GB config-C buffer) is wiped in the background for several seconds, and every HBM-bound
    kernel runs 2-4 % slower meanwhile (profiles/DESIGN_r01-r03.md 6, tools/s_launches.py,
    r03s4-r03s6). `step(i)` launches one step, `sync()` waits for it; the clock is read after
    every `block` back-to-back launches. The headline, the N > 1 solo leg and the CPU dry run's
    solo leg all settle by this rule. Returns (launches run, seconds spent)."""
    n, t0 = 0, time.perf_counter()
    cap = SETTLE_CAP_S if cap_s is None else cap_s
    blocks = []  # (seconds, launches) per block of back-to-back launches
    while (n < max(0, settle - warmup) or time.perf_counter() - t0 < settle_s or
           (settle_s > 0 and not launch_rate_steady(blocks) and time.perf_counter() - t0 < cap)):
        t_blk = time.perf_counter()
        for _ in range(block):
            step(n)
            n += 1
        sync()
        blocks.append((time.perf_counter() - t_blk, block))
    return n, time.perf_counter() - t0


def run_timed(wl, steps, warmup, settle, streams, world, dist, event_every=0, region_marks=None, settle_s=0.0):
    """W untimed warm-up steps (after the settle launches of settle_steps), then EXACTLY
    `steps` steps between barrier + synchronize on both sides. Returns (max-over-ranks seconds,
    HIP-event span of the region / steps in ms, sampled per-launch ms or None, settle launches
    run, this rank's own seconds)."""
    import torch
    stream = streams[0]
    n_settle, _ = settle_steps(lambda i: wl.step(i, streams), torch.cuda.synchronize, settle, warmup, settle_s)
    for i in range(warmup):
        wl.step(i, streams)
    torch.cuda.synchronize()
    ev = {i: (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for i in range(0, steps, event_every)} if event_every > 0 else {}
    region = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    if region_marks:
        region_marks.resume()
    t0 = time.perf_counter()
    region[0].record(stream)
    for s2 in streams[1:]:
        s2.wait_stream(stream)  # every stream starts after the region's first event
    for i in range(steps):
        e = ev.get(i)
        if e:
            e[0].record(stream)
        wl.step(i, streams)
        if e:
            e[1].record(stream)
    for s2 in streams[1:]:
        stream.wait_stream(s2)  # ... and the last event after every stream's last launch
    region[1].record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = own = time.perf_counter() - t0
    if region_marks:
        region_marks.pause()
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=stream.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    avg_ms = region[0].elapsed_time(region[1]) / steps
    sampled = float(np.mean([a.elapsed_time(b) for a, b in ev.values()])) if ev else None
    return elapsed, avg_ms, sampled, n_settle + warmup, own


def read_ceiling(wl, launches=400):
    """The measured streaming-read ceiling of config B's access shape at its launch size
    (SURVEY.md 8d): gpu.stream_read (testutil.hip: the CRC kernel's loads -- lane <-> 128-B
    line, the same sweep front, one tile in flight per wave -- with an XOR fold instead of the
    CRC) over the same rotated batches, back to back after ~60 ms of them."""
    import torch
    from subspace_amd import gpu
    sink = torch.empty(256 * 512, dtype=torch.int32, device=wl.bufs[0].device)
    for i in range(1400):
        gpu.stream_read(wl.bufs[i % wl.nbuf], sink)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(launches):
        gpu.stream_read(wl.bufs[i % wl.nbuf], sink)
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / launches * 1e3
    return {"GBps": round(wl.step_bytes / (us * 1e-6) / 1e9, 1), "us_per_launch": round(us, 2), "launches": launches,
            "kernel": "stream_read_kernel (testutil.hip): the CRC kernel's load shape and sweep, one tile in "
                      "flight, no CRC"}


# ------------------------------------------------------------------------------ secondary configs
def time_calls(fn, iters, warm_ms=60.0):
    """ms per call: one HIP event pair around `iters` back-to-back calls (after ~warm_ms of
    back-to-back warm-up calls: a stop-and-go warm-up leaves short calls in the GPU's
    power-management ramp, profiles/DESIGN_r01-r03.md 4.0), / iters -- the headline's timing rule."""
    import torch
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    fn()
    b.record()
    torch.cuda.synchronize()
    for _ in range(max(2, min(4000, int(warm_ms / max(a.elapsed_time(b), 1e-3))))):
        fn()
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def config_traffic(name):
    """(HBM bytes per call, source) of a secondary configuration from the committed PMC summary
    (profiles/traffic_configs.json, tools/pmc_configs.sh + tools/summarize_configs_traffic.py:
    separate rocprofv3 --pmc passes, not measured in this run), or (None, None)."""
    f = ROOT / "profiles" / "traffic_configs.json"
    try:
        tj = json.loads(f.read_text())
        c = tj["configs"][name]
        return c["hbm_bytes_per_call"], (f"profiles/traffic_configs.json ({c.get('source', tj.get('source', '?'))}; "
                                         f"PMC FETCH_SIZE x2 + "
                                         f"WRITE_SIZE per call, ratio {c['ratio']} of the algorithmic bytes; not "
                                         f"measured in this run)")
    except (OSError, ValueError, KeyError):
        return None, None


def config_line(nbytes, ms, bitexact, kernel, extra=None, name=None):
    gbs = nbytes / (ms * 1e-3) / 1e9
    traffic, tsrc = config_traffic(name) if name else (None, None)
    line = {"value": round(nbytes / (ms * 1e-3) / 2**30, 1), "unit": "GiB/s", "bytes": int(nbytes),
            "ms_per_call": round(ms, 4), "pct_of_hbm_peak": round(100 * gbs / HBM_PEAK_GBS, 2),
            "bitexact_vs_golden": bitexact,
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
                         "kernel": kernel,
                         "launch_ms_source": "HIP event span of back-to-back calls / calls (the whole C-ABI call: "
                                             "prep kernels + CRC kernel + combine)"}}
    if extra:
        line.update(extra)
    return line


def secondary_configs(ctx, dev, names, iters) -> dict:
    """Configs C, C unaligned, D (ragged API), D (uniform API: long-message kernel) and S
    (slot publish / verify) through the production C ABI, each checked bit-exact."""
    import torch
    from subspace_amd import gpu, slots, synth
    res = {}

    def u64t(a):
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)

    def one_config(name):
        if name in ("C", "Cu"):
            lengths = synth.ragged_lengths(synth.SEED_C, GOLD["C"]["count"])
            offsets, total = synth.packed_offsets(lengths, 1 if name == "Cu" else 64)
            buf = torch.empty(total + 64, dtype=torch.uint8, device=dev)
            d_off, d_len = u64t(offsets), u64t(lengths)
            gpu.fill_ragged(buf, d_off, d_len, seed=synth.SEED_C)
            out = torch.empty(len(lengths), dtype=torch.int32, device=dev)
            ms = time_calls(lambda: ctx.crc32_ragged(buf, d_off, d_len, out), iters)
            ok = digest(out.cpu().numpy().view(np.uint32)) == GOLD["C"]["sha256_le_u32"]
            res[name] = config_line(int(lengths.sum()), ms, ok, "subspace_crc32_batch (ragged kernel)", name=name, extra={
                "workload": "C: 1 Mi messages, 64 B - 1 MiB log-uniform, " +
                            ("packed unaligned" if name == "Cu" else "64-B aligned offsets"),
                "messages": len(lengths)})
            del buf, d_off, d_len, out
        elif name in ("D", "Du"):
            n, L = GOLD["D"]["count"], 64 << 20
            buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
            gpu.fill_uniform(buf, L, L, n, seed=synth.SEED_D)
            out = torch.empty(n, dtype=torch.int32, device=dev)
            if name == "D":
                d_off = u64t(np.arange(n, dtype=np.uint64) * np.uint64(L))
                d_len = u64t(np.full(n, L, dtype=np.uint64))
                ms = time_calls(lambda: ctx.crc32_ragged(buf, d_off, d_len, out), iters)
                kern = "subspace_crc32_batch (ragged kernel)"
            else:
                ms = time_calls(lambda: ctx.crc32_uniform(buf, L, L, n, out), iters)
                kern = "subspace_crc32_batch_uniform (long-message kernel)"
            ok = digest(out.cpu().numpy().view(np.uint32)) == GOLD["D"]["sha256_le_u32"]
            res[name] = config_line(n * L, ms, ok, kern, {"workload": "D: 256 x 64 MiB", "messages": n}, name=name)
            del buf, out
        elif name == "S":
            res.update(slot_configs(ctx, dev, iters))
        elif name == "Usmall":
            res[name] = small_uniform_config(ctx, dev)
        elif name == "S_short":
            res[name] = short_slots_config(ctx, dev)
        elif name == "S_mixed":
            res[name] = short_slots_config(ctx, dev, mixed=True)
        elif name == "S_large":
            res.update(large_slots_config(ctx, dev))

    # No torch.cuda.empty_cache() between configs: VRAM given back to the driver is wiped in the
    # background for seconds (every HBM-bound kernel ~2-4 % slower meanwhile: config S after
    # config C's 118 GB free measured 67-68 % instead of 69-71 %, r03s4-r03s6), so the configs
    # reuse the caching allocator's blocks instead
    for name in names:
        try:
            one_config(name)
        except Exception as e:  # a secondary config must never cost the headline line
            res[name] = {"error": f"{type(e).__name__}: {e}"[:300]}
    return res


def small_uniform_config(ctx, dev) -> dict:
    """Informational (no BASELINE config): 1 Mi messages of 256 B, stride 256, through
    subspace_crc32_batch_uniform -- the small-message kernel packed two lanes per message
    (crc_small.hip G = 2), 4 rotated batches; 256 sampled CRCs checked against the host
    drop-in (SubspaceCRC32, include/subspace/checksum.h)."""
    import torch
    from subspace_amd import checksum, gpu
    n, L, nb = 1 << 20, 256, 4
    bufs = [torch.empty(n * L, dtype=torch.uint8, device=dev) for _ in range(nb)]
    for k, b in enumerate(bufs):
        gpu.fill_uniform(b, L, L, n, seed=0x5EED0256 + k)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    i = [0]

    def call():
        ctx.crc32_uniform(bufs[i[0] % nb], L, L, n, out)
        i[0] += 1
    ms = time_calls(call, 400)
    ctx.crc32_uniform(bufs[0], L, L, n, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    host = bufs[0].cpu().numpy()
    idx = np.random.default_rng(1).choice(n, 256, replace=False)
    ok = all(checksum.subspace_crc32(0xFFFFFFFF, host[j * L:(j + 1) * L]) == int(got[j]) for j in idx)
    line = config_line(n * L, ms, ok, "subspace_crc32_batch_uniform: crc32_small_kernel<512, false, false, 2> "
                       "(G = 2 lanes per message, the uniform FAST loop)", name="Usmall", extra={
                           "workload": "Usmall (informational): 1 Mi x 256 B messages, stride 256, 4 batches rotated",
                           "messages_per_s": round(n / (ms * 1e-3), 1),
                           "check": "256 sampled CRCs equal the host drop-in's SubspaceCRC32"})
    del bufs, out
    return line


def short_slots_config(ctx, dev, mixed=False) -> dict:
    """Informational (no BASELINE config): a channel of 65,536 4 KiB slots (stride 4,160)
    carrying 256-B messages (S_short) or messages of 1 .. 4,096 B, uniformly random (S_mixed),
    published by the fused strided kernel, then drained as shuffled device slot lists
    (max_message_size 4096) through subspace_crc32_slots -- the small kernel's waves pack their
    windows by message size (crc_small.hip REPACK: 2^c lanes per message); 4 rotated copies.
    Bytes: span 0 + payload per slot. Check: every slot verifies (publish and verify are
    different kernels)."""
    import torch
    from subspace_amd import gpu, slots
    n, area, L, cs, ms_, nbuf = MSGS, MSG_BYTES, 256, 4, 0, 4
    ps, stride = slots.compute_prefix_size(cs, ms_), slots.slot_stride(area, cs, ms_)
    rng = np.random.default_rng(0x5EED0258 if mixed else 0x5EED0257)
    sizes = rng.integers(1, area + 1, n).astype(np.uint64) if mixed else np.full(n, L, dtype=np.uint64)
    host = rng.integers(0, 256, stride * n, dtype=np.uint8)
    host.reshape(n, stride)[:, :ps] = slots.make_prefixes(n, sizes, checksum_size=cs, metadata_size=ms_, seed=7)
    bufs = [torch.from_numpy(host).to(dev) for _ in range(nbuf)]
    d_sizes = torch.from_numpy(sizes.view(np.int64)).to(dev)
    for b in bufs:
        ctx.crc32_slots_strided(b, stride, n, sizes=d_sizes, checksum_size=cs, metadata_size=ms_,
                                mode=gpu.SLOT_CALCULATE)
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

    def call():
        ctx.crc32_slots(recs[i[0] % nbuf], max_message_size=area, checksum_size=cs, metadata_size=ms_,
                        mode=gpu.SLOT_VERIFY, status=status, error_count=errs)
        i[0] += 1
    ms = time_calls(call, 400)
    torch.cuda.synchronize()
    ok = int(errs.item()) == 0 and bool((status == 0).all().item())
    name = "S_mixed" if mixed else "S_short"
    what = "messages of 1 .. 4,096 B (uniformly random)" if mixed else "256-B messages"
    line = config_line(int(sizes.sum()) + 44 * n, ms, ok, "subspace_crc32_slots: crc32_small_kernel<512, true, "
                       "false, 32> (REPACK: 2^c lanes per message by size)", name=name, extra={
                           "workload": f"{name} (informational): 65,536 slots of 4 KiB (stride 4,160) carrying {what}, "
                                       "shuffled device slot lists, verify, 4 copies rotated",
                           "slots_per_s": round(n / (ms * 1e-3), 1),
                           "check": "every slot verifies (published by the fused strided kernel)"})
    del bufs, recs, status
    return line


def large_slots_config(ctx, dev, nbuf=4) -> dict:
    """S_large: the reference's own checksum channel shape,
    LatencyTest.PublisherLatencyPayloadChecksum (client/latency_test.cc:731-745): 32 KiB slots
    (stride 32,832) carrying payloads of rand() % 32,767 + 1 bytes, checksums on -- 65,536 slots,
    drained as shuffled device slot lists (max_message_size 32,768) through subspace_crc32_slots,
    verify and publish, 4 rotated channel copies (8.6 GB). Bytes: span 0 + payload per slot. Read
    ceiling: the tile-list probe (testutil.hip tile_list_read_kernel) over the same messages' 8 KiB
    tiles in list order, the ragged kernel's loads without the CRC. Checks: verify passes every
    slot of a channel published by the other path (subspace_crc32_slots_strided: the arena
    pipeline); a publish over a copy with checksums and flags cleared leaves 64 sampled slots with
    the host drop-in's CalculateCRC32Checksum<3> and the flag."""
    import torch
    from subspace_amd import checksum, gpu, slots
    n, area, cs, ms_ = MSGS, 32768, 4, 0
    ps, stride = slots.compute_prefix_size(cs, ms_), slots.slot_stride(area, cs, ms_)
    rng = np.random.default_rng(0x5EED0259)
    sizes = rng.integers(1, area, n).astype(np.uint64)  # rand() % (kMaxPayloadSize - 1) + 1
    d_sizes = torch.from_numpy(sizes.view(np.int64)).to(dev)
    d_pre = torch.from_numpy(slots.make_prefixes(n, sizes, checksum_size=cs, metadata_size=ms_, seed=9)).to(dev)
    d_offs = torch.from_numpy((np.arange(n, dtype=np.uint64) * np.uint64(stride) + np.uint64(ps)).view(np.int64)).to(dev)
    bufs = []
    for k in range(nbuf):
        b = torch.empty(n * stride, dtype=torch.uint8, device=dev)
        b.view(n, stride)[:, :ps] = d_pre
        gpu.fill_ragged(b, d_offs, d_sizes, seed=0x5EED0259 + k)
        ctx.crc32_slots_strided(b, stride, n, sizes=d_sizes, checksum_size=cs, metadata_size=ms_,
                                mode=gpu.SLOT_CALCULATE)
        bufs.append(b)
    order = rng.permutation(n).astype(np.uint64)
    so = sizes[order.astype(np.int64)]
    nt = (so + np.uint64(8191)) // np.uint64(8192)
    recs, tiles = [], []
    for b in bufs:
        b0 = np.uint64(b.data_ptr())
        pay = b0 + order * np.uint64(stride) + np.uint64(ps)
        r = np.stack([b0 + order * np.uint64(stride), pay, so], axis=1)
        recs.append(torch.from_numpy(np.ascontiguousarray(r).view(np.int64)).to(dev))
        first = np.repeat(np.cumsum(nt) - nt, nt.astype(np.int64))
        t = np.arange(int(nt.sum()), dtype=np.uint64) - first.astype(np.uint64)  # tile index in its message
        msg_len = np.repeat(so, nt.astype(np.int64))
        tl = np.stack([np.repeat(pay, nt.astype(np.int64)) + t * np.uint64(8192),
                       np.minimum(np.uint64(8192), msg_len - t * np.uint64(8192))], axis=1)
        tiles.append(torch.from_numpy(np.ascontiguousarray(tl).view(np.int64)).to(dev))
    nbytes = int(sizes.sum()) + 44 * n
    sink = torch.empty(256 * 512, dtype=torch.int32, device=dev)
    j = [0]

    def probe():
        gpu.tile_list_read(tiles[j[0] % nbuf], sink)
        j[0] += 1
    pms = time_calls(probe, 100)
    ceiling = {"GBps": round(nbytes / (pms * 1e-3) / 1e9, 1), "us_per_launch": round(pms * 1e3, 2),
               "tiles": int(nt.sum()),
               "kernel": "tile_list_read_kernel (testutil.hip): the ragged kernel's buffer loads over the same "
                         "messages' 8 KiB tiles in list order, no CRC"}
    status = torch.empty(n, dtype=torch.int32, device=dev)
    errs = torch.zeros(1, dtype=torch.int32, device=dev)
    res = {}
    for mode, key in ((gpu.SLOT_VERIFY, "S_large_verify"), (gpu.SLOT_CALCULATE, "S_large_publish")):
        i = [0]

        def call():
            ctx.crc32_slots(recs[i[0] % nbuf], max_message_size=area, checksum_size=cs, metadata_size=ms_, mode=mode,
                            status=status, error_count=errs if mode == gpu.SLOT_VERIFY else None)
            i[0] += 1
        ms = time_calls(call, 100)
        torch.cuda.synchronize()
        if mode == gpu.SLOT_VERIFY:
            ok = int(errs.item()) == 0 and bool((status == 0).all().item())
            check = "every slot passes (channel published by subspace_crc32_slots_strided)"
        else:
            v = bufs[0].view(n, stride)
            v[:, 48:48 + cs] = 0
            v[:, 32] &= 0xFB
            ctx.crc32_slots(recs[0], max_message_size=area, checksum_size=cs, metadata_size=ms_, mode=mode,
                            status=status)
            torch.cuda.synchronize()
            ok = bool((status == 0).all().item())
            for k in rng.choice(n, 64, replace=False):
                row = v[int(k)].cpu().numpy()
                L = int(sizes[k])
                want = checksum.calculate_crc32_checksum(
                    checksum.get_message_checksum_data(row[:ps], row[ps:ps + L], L, cs, ms_))
                ok = ok and bytes(row[48:52]) == want and bool(row[32] & 4)
            check = "64 sampled slots of copy 0 (flag + checksum cleared before the call) hold the host drop-in's " \
                    "CalculateCRC32Checksum<3> and the flag"
        res[key] = config_line(nbytes, ms, ok, "subspace_crc32_slots, max_message_size 32,768: ragged pipeline "
                               "(absolute addresses) + slot finish", name=key, extra={
                                   "workload": "S_large: the reference's checksum latency channel "
                                               "(client/latency_test.cc:731-745): 65,536 slots of 32 KiB (stride "
                                               "32,832), payloads 1 .. 32,767 B uniformly random, shuffled device slot "
                                               "lists, 4 copies rotated, " +
                                               ("verify" if mode == gpu.SLOT_VERIFY else "publish"),
                                   "slots_per_s": round(n / (ms * 1e-3), 1), "check": check})
        res[key]["roofline"]["read_ceiling"] = ceiling
        res[key]["roofline"]["frac_of_read_ceiling"] = round(pms / ms, 4)
    del bufs, recs, tiles, sink, status
    return res


def slot_leg_check(mode, buf, n, stride, ps, size, cs, ms_, status, errs, rng):
    """A slot leg's bit-exactness: a publish (CALCULATE) leaves 64 sampled slots of `buf` with the
    flag set and the host drop-in's CalculateCRC32Checksum<3> over GetMessageChecksumData
    (include/subspace/checksum.h; the channel's prefixes start without valid checksums); a
    verify passes every slot. Returns (ok, what was checked)."""
    from subspace_amd import checksum, gpu
    if mode == gpu.SLOT_VERIFY:
        return int(errs.item()) == 0 and bool((status == 0).all().item()), "verify passes every slot"
    chan = buf.cpu().numpy()
    ok = True
    for k in rng.choice(n, 64, replace=False):
        pre = chan[k * stride:k * stride + ps]
        pay = chan[k * stride + ps:k * stride + ps + size]
        want = checksum.calculate_crc32_checksum(checksum.get_message_checksum_data(pre, pay, size, cs, ms_))
        ok = ok and bytes(pre[48:52]) == want and bool(pre[32] & 4)
    return ok, "64 sampled slots hold the flag and the host drop-in's CalculateCRC32Checksum<3>"


def slot_configs(ctx, dev, iters) -> dict:
    """Config S: config B in the reference's slot layout on the device (65,536 slots of
    PrefixSize 64 + 4 KiB payload, stride 4,160, 4 rotated channel buffers), the full 3-span
    checksum. Publish (CALCULATE) must leave every prefix equal to the host drop-in's
    CalculateCRC32Checksum<3> over GetMessageChecksumData (64 sampled slots); verify
    (VERIFY) must pass every slot."""
    import torch
    from subspace_amd import checksum, gpu, slots
    n, size, cs, ms_, nbuf = MSGS, MSG_BYTES, 4, 0, 4
    ps, stride = slots.compute_prefix_size(cs, ms_), slots.slot_stride(size, cs, ms_)
    rng = np.random.default_rng(0x5EED0005)
    host = rng.integers(0, 256, stride * n, dtype=np.uint8)
    host.reshape(n, stride)[:, :ps] = slots.make_prefixes(n, np.full(n, size, dtype=np.uint64), checksum_size=cs,
                                                          metadata_size=ms_, seed=5)
    bufs = [torch.from_numpy(host).to(dev) for _ in range(nbuf)]
    status = torch.empty(n, dtype=torch.int32, device=dev)
    errs = torch.zeros(1, dtype=torch.int32, device=dev)
    nbytes = n * (size + 44)  # checksummed bytes: span 0 (44 B) + payload
    res = {}
    for mode, key in ((gpu.SLOT_CALCULATE, "S_publish"), (gpu.SLOT_VERIFY, "S_verify")):
        i = [0]

        def call():
            b = bufs[i[0] % nbuf]
            i[0] += 1
            ctx.crc32_slots_strided(b, stride, n, message_size=size, checksum_size=cs, metadata_size=ms_, mode=mode,
                                    status=status if mode == gpu.SLOT_VERIFY else None,
                                    error_count=errs if mode == gpu.SLOT_VERIFY else None)
        ms = time_calls(call, 400)
        torch.cuda.synchronize()
        ok, check = slot_leg_check(mode, bufs[0], n, stride, ps, size, cs, ms_, status, errs, rng)
        res[key] = config_line(nbytes, ms, ok, "subspace_crc32_slots_strided", name=key, extra={
            "workload": "S: 65,536 slots (prefix 64 B + 4 KiB payload, stride 4,160), 3-span checksum, " +
                        ("publish: flag + checksum stored" if mode == gpu.SLOT_CALCULATE else
                         "verify: per-slot status + mismatch count"),
            "check": check})
    # S_list: the same channels drained as device slot lists in shuffled order (a subscriber's
    # read order over several wrap-arounds), one list per channel copy, rotated like S (round 4
    # timed one copy only: 273 MB, most of it served from the 256 MB MALL -- 51.0 against 66.7
    # us per call for the round-4 kernel, r05a): subspace_crc32_slots, publish (flag + checksum
    # of every slot cleared on the device first, so the sampled check sees this leg's stores)
    # then verify
    order = rng.permutation(n).astype(np.uint64)

    def list_recs(b):
        b0 = np.uint64(b.data_ptr())
        r = np.stack([b0 + order * np.uint64(stride), b0 + order * np.uint64(stride) + np.uint64(ps),
                      np.full(n, size, dtype=np.uint64)], axis=1)
        return torch.from_numpy(np.ascontiguousarray(r).view(np.int64)).to(dev)

    d_recs = [list_recs(b) for b in bufs]
    for b in bufs:
        pre = b.view(n, stride)
        pre[:, 48:52].zero_()                # the stored checksum
        pre[:, 32].bitwise_and_(0xFB)        # kMessageHasChecksum (flags, offset 32)
    torch.cuda.synchronize()
    list_kernel = "subspace_crc32_slots: subspace_amd::crc32_small_kernel<512, true, false, 32> (one launch, " \
                  "slots finished in it; crc_small.hip)"
    # the slot-list access shape's own read ceiling: the kernel's FAST-loop loads over the same
    # rotated shuffled lists, no CRC (gpu.slot_list_read mode 4)
    sink = torch.empty(256 * 512, dtype=torch.int32, device=dev)
    j = [0]

    def probe():
        gpu.slot_list_read(d_recs[j[0] % nbuf], n, sink, mode=4)
        j[0] += 1
    pms = time_calls(probe, 400)
    ceiling = {"GBps": round(nbytes / (pms * 1e-3) / 1e9, 1), "us_per_launch": round(pms * 1e3, 2),
               "kernel": "slot_list_read_kernel<4> (testutil.hip): the small kernel's FAST-loop loads and first-window "
                         "prefix words over the same rotated shuffled lists, no CRC"}
    for mode, key in ((gpu.SLOT_CALCULATE, "S_list_publish"), (gpu.SLOT_VERIFY, "S_list_verify")):
        i = [0]
        errs.zero_()

        def call():
            r = d_recs[i[0] % nbuf]
            i[0] += 1
            ctx.crc32_slots(r, max_message_size=size, checksum_size=cs, metadata_size=ms_, mode=mode, status=status,
                            error_count=errs if mode == gpu.SLOT_VERIFY else None)
        ms = time_calls(call, 400)
        torch.cuda.synchronize()
        if mode == gpu.SLOT_CALCULATE:
            ok = bool((status == 0).all().item())
            chan = bufs[0].cpu().numpy()
            for k in rng.choice(n, 64, replace=False):
                pre = chan[k * stride:k * stride + ps]
                pay = chan[k * stride + ps:k * stride + ps + size]
                want = checksum.calculate_crc32_checksum(checksum.get_message_checksum_data(pre, pay, size, cs, ms_))
                ok = ok and bytes(pre[48:52]) == want and bool(pre[32] & 4)
            check = "64 sampled slots of copy 0 (flag + checksum cleared before the leg) hold the host drop-in's " \
                    "CalculateCRC32Checksum<3> and the flag"
        else:
            ok = int(errs.item()) == 0 and bool((status == 0).all().item())
            check = "every slot passes"
        res[key] = config_line(nbytes, ms, ok, list_kernel, name=key, extra={
            "workload": "S_list: config S's 65,536 slots as device slot lists (subspace_crc_slot records) in shuffled "
                        "order, one per channel copy, 4 copies rotated, " +
                        ("publish" if mode == gpu.SLOT_CALCULATE else "verify"),
            "check": check})
        res[key]["roofline"]["read_ceiling"] = ceiling
        res[key]["roofline"]["frac_of_read_ceiling"] = round(pms / ms, 4)
    del bufs, d_recs, sink
    # S_meta: 16 B of user metadata per slot (SetMetadataSize, client/options.h:375-391):
    # ComputePrefixSize(4, 16) = 128, stride 4,224; spans 44 + 16 + 4,096 B
    cs, ms_ = 4, 16
    ps, stride = slots.compute_prefix_size(cs, ms_), slots.slot_stride(size, cs, ms_)
    host = rng.integers(0, 256, stride * n, dtype=np.uint8)
    host.reshape(n, stride)[:, :ps] = slots.make_prefixes(n, np.full(n, size, dtype=np.uint64), checksum_size=cs,
                                                          metadata_size=ms_, seed=6)
    bufs = [torch.from_numpy(host).to(dev) for _ in range(nbuf)]
    nbytes = n * (size + 44 + ms_)
    for mode, key in ((gpu.SLOT_CALCULATE, "S_meta_publish"), (gpu.SLOT_VERIFY, "S_meta_verify")):
        i = [0]

        def call():
            b = bufs[i[0] % nbuf]
            i[0] += 1
            ctx.crc32_slots_strided(b, stride, n, message_size=size, checksum_size=cs, metadata_size=ms_, mode=mode,
                                    status=status if mode == gpu.SLOT_VERIFY else None,
                                    error_count=errs if mode == gpu.SLOT_VERIFY else None)
        errs.zero_()
        ms = time_calls(call, 200)
        torch.cuda.synchronize()
        ok, check = slot_leg_check(mode, bufs[0], n, stride, ps, size, cs, ms_, status, errs, rng)
        res[key] = config_line(nbytes, ms, ok, "subspace_crc32_slots_strided", name=key, extra={
            "workload": "S_meta: 65,536 slots (prefix 128 B with 16 B metadata + 4 KiB payload, stride 4,224), "
                        "3-span checksum, " + ("publish" if mode == gpu.SLOT_CALCULATE else "verify"),
            "check": check})
    del bufs
    return res


# ------------------------------------------------------------------------------ CPU dry run
def dry_run_cpu(args, world, rank) -> int:
    """The multi-rank path on the CPU (gloo): same spawn, shard, barrier/max timing and
    gather code as the GPU run; each rank checksums its shard with the library's host
    SubspaceCRC32 (libsubspace_crc.so), and rank 0 checks the gathered list against the
    fixture. E -> config B's 65,536 messages round-robin ("B" fixture); C -> the first
    2,048 messages of config C in byte-balanced contiguous ranges ("C_2k"); B -> every rank
    the 4,096-message "B_small" batch (weak)."""
    import torch
    import torch.distributed as dist
    from subspace_amd import checksum, shard, synth
    if world > 1:
        dist.init_process_group("gloo")
        if dist.get_world_size() != args.gpus:
            die(f"ranks joined {dist.get_world_size()} != --gpus {args.gpus}")
    wl = args.workload
    if wl == "E":
        key, count = "B", GOLD["B"]["count"]
        ids = shard.shard_ids(count, rank, world)
        data = synth.host_uniform(GOLD["B"]["seed"], ids, MSG_BYTES)
        msgs = [data[j] for j in range(len(ids))]
    elif wl == "C":
        key, count = "C_2k", GOLD["C_2k"]["count"]
        lengths = synth.ragged_lengths(synth.SEED_C, count)
        bounds = shard.ragged_ranges(lengths, world)
        lo, hi = int(bounds[rank]), int(bounds[rank + 1])
        offs, arena = synth.packed_offsets(lengths[lo:hi], 64)
        data = synth.host_ragged(synth.SEED_C, np.arange(lo, hi), lengths[lo:hi], offs, arena)
        msgs = [data[int(o):int(o) + int(n)] for o, n in zip(offs, lengths[lo:hi])]
    else:
        key, count = "B_small", GOLD["B_small"]["count"]
        data = synth.host_uniform(GOLD["B_small"]["seed"], np.arange(count, dtype=np.uint64), MSG_BYTES)
        msgs = [data[j] for j in range(count)]
    local = np.zeros(max(len(msgs), 1), dtype=np.uint32)
    step_bytes = sum(int(m.nbytes) for m in msgs)

    def step():
        for j, m in enumerate(msgs):
            local[j] = checksum.subspace_crc32(0xFFFFFFFF, m)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    elapsed = own = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # N > 1: rank 0 alone over the whole workload (the N = 1 configuration), settled by the
    # headline's rule (settle_steps; on the CPU at most 2 s of it), for the efficiency -- the
    # GPU run's solo leg, rehearsed
    solo = None
    if world > 1 and not args.no_solo:
        dist.barrier()
        if rank == 0:
            if wl == "E":
                alld = synth.host_uniform(GOLD["B"]["seed"], np.arange(count, dtype=np.uint64), MSG_BYTES)
                allm = [alld[j] for j in range(count)]
            elif wl == "C":
                offs1, arena1 = synth.packed_offsets(lengths, 64)
                alld = synth.host_ragged(synth.SEED_C, np.arange(count), lengths, offs1, arena1)
                allm = [alld[int(o):int(o) + int(n)] for o, n in zip(offs1, lengths)]
            else:
                allm = msgs
            all_out = np.zeros(len(allm), dtype=np.uint32)

            def solo_step(_i):
                for j, m in enumerate(allm):
                    all_out[j] = checksum.subspace_crc32(0xFFFFFFFF, m)

            settle_s = min(args.settle_s, 2.0) if args.settle > 0 else 0.0
            n1, t1 = settle_steps(solo_step, lambda: None, min(args.settle, 2), 0, settle_s, block=1,
                                  cap_s=2 * settle_s)
            ts = time.perf_counter()
            for i in range(args.steps):
                solo_step(i)
            el1 = time.perf_counter() - ts
            sb = sum(int(m.nbytes) for m in allm)
            solo = {"value": round(sb * args.steps / el1 / 2**30, 3), "steps": args.steps,
                    "settle_launches": n1, "settle_s": round(t1, 3),
                    "bitexact_vs_golden": digest(all_out) == GOLD[key]["sha256_le_u32"] if wl != "B" else None}
        dist.barrier()
    tl = torch.from_numpy(local[:len(msgs)].view(np.int32).copy())
    tg = time.perf_counter()
    # the same gather helpers as the GPU run (here on CPU tensors over gloo)
    if wl == "C":
        full = shard.gather_ragged_crcs_device(tl, bounds, world, dist if world > 1 else None).numpy().view(np.uint32)
    elif wl == "E":
        full = shard.gather_crcs_device(tl, count, world, dist if world > 1 else None).numpy().view(np.uint32)
    else:
        full = local[:len(msgs)]
    gather_ms = (time.perf_counter() - tg) * 1e3
    me = {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "0")), "device": "cpu", "pid": os.getpid(),
          "step_ms": round(own / args.steps * 1e3, 4)}
    everyone = [me]
    if world > 1:
        everyone = [None] * world
        dist.all_gather_object(everyone, me)
    if rank == 0:
        total = (step_bytes * world if wl == "B" else GOLD[key]["total_bytes"]) * args.steps
        value = total / elapsed / 2**30
        print(json.dumps({
            "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak" if wl == "B" else "strong", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (host twin of the device generator)",
            "dry_run_cpu": True, "device": "cpu: host SubspaceCRC32 (libsubspace_crc.so) per rank, gloo",
            "config": {"workload": f"dry run of {wl} over fixture {key} ({count} messages)",
                       "parallelism": f"{'round-robin' if wl == 'E' else 'byte-balanced contiguous' if wl == 'C' else 'replicated'} "
                                      f"shards x{world}, gloo all_gather of CRCs",
                       "gather_ms": round(gather_ms, 3)},
            "per_gpu_value": round(value / world, 3),
            "bitexact_vs_golden": digest(full) == GOLD[key]["sha256_le_u32"] if full is not None else None,
            "ranks": everyone,
            "rank_step_ms": {"min": min(r["step_ms"] for r in everyone), "max": max(r["step_ms"] for r in everyone)},
            "rccl_world": dist.get_world_size() if world > 1 else 1,
            "backend": dist.get_backend() if world > 1 else None,
            "single_gpu": solo,
            "efficiency": round(value / (world * solo["value"]), 4) if solo else None,
        }), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


# ------------------------------------------------------------------------------ main
def main():
    apply_rank_env()  # before torch and before any HIP call, in every launch form
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(spawn_ranks(args))  # this process never touches a GPU
    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        die(f"--gpus {args.gpus} but WORLD_SIZE {world}: launch with --nproc-per-node equal to --gpus")
    if args.print_rank_env:  # tests: what a rank runs with, before anything else happens
        # one write(2) of the whole line: ranks share the parent's stdout pipe, and print() under
        # PYTHONUNBUFFERED issues the record and its newline as two writes, which two ranks can
        # interleave into one line (the round-5 CPU-gate flake: JSONDecodeError "Extra data")
        sys.stdout.flush()
        rec = json.dumps({"rank": rank, "env": {k: os.environ.get(k) for k in RANK_ENV_REPORTED}}) + "\n"
        os.write(sys.stdout.fileno(), rec.encode())
        sys.exit(0)
    if args.workload is None:
        args.workload = "B" if world == 1 else "E"
    if args.dry_run_cpu:
        sys.exit(dry_run_cpu(args, world, rank))

    import torch
    import torch.distributed as dist
    from subspace_amd import gpu
    gpu_index = 0 if args.rehearse_one_gpu else local
    if torch.cuda.device_count() <= gpu_index:
        die(f"LOCAL_RANK {local} but only {torch.cuda.device_count()} visible GPU(s)")
    # a launcher (torch.distributed.run) sets WORLD_SIZE: then the process group exists even at
    # one rank, so the RCCL path (init, barriers, the max-over-ranks reduction, the gather)
    # runs exactly as at N ranks; a plain `python bench.py` (the driver's N = 1) has none
    dist_on = world > 1 or world_env is not None
    if dist_on:
        torch.cuda.set_device(gpu_index)
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu_index))
        if dist.get_world_size() != args.gpus:
            die(f"the process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    dev = torch.device("cuda", gpu_index)
    torch.cuda.set_device(dev)
    ctx = gpu.CrcContext(gpu_index)
    stream = torch.cuda.current_stream()

    wl = Workload(args.workload, ctx, dev, world, rank)
    torch.cuda.synchronize()
    if wl.nbuf % args.streams:  # workloads C and E have one buffer: their steps stay on one stream
        args.streams = 1
    streams = [stream] + [torch.cuda.Stream() for _ in range(args.streams - 1)]
    for s2 in streams[1:]:
        s2.wait_stream(stream)
    pg = dist if dist_on else None
    elapsed, avg_kern_ms, sampled_ms, settle, own_s = run_timed(wl, args.steps, args.warmup, args.settle, streams,
                                                                world, pg, args.event_every,
                                                                RoctxRegion(args.roctx_region and rank == 0),
                                                                args.settle_s if args.settle > 0 else 0.0)
    settle = max(0, settle - args.warmup)
    bitexact, gather = wl.check(pg)
    gather_ms = gather["gather_ms"] if gather else None
    ceiling = None
    if args.workload == "B" and world == 1:
        try:
            ceiling = read_ceiling(wl)
        except Exception as e:  # an extra leg must never cost the headline line
            ceiling = {"error": f"{type(e).__name__}: {e}"[:300]}
    # every rank's identity and timing, so the line shows that N distinct GPUs ran
    props = torch.cuda.get_device_properties(gpu_index)
    me = {"rank": rank, "local_rank": local, "device": torch.cuda.current_device(),
          "pci": f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}",
          "uuid": str(getattr(props, "uuid", "")), "step_ms": round(own_s / args.steps * 1e3, 4),
          "launch_ms_event": round(avg_kern_ms, 4)}
    if dist_on:
        everyone = [None] * world
        dist.all_gather_object(everyone, me)
    else:
        everyone = [me]
    step_bytes, total_step_bytes, nmsg = wl.step_bytes, wl.total_bytes, wl.nmsg
    bounds = getattr(wl, "bounds", None)

    # ---- N > 1: the same workload alone on rank 0's GPU (the N = 1 configuration), for the
    #      per-GPU efficiency; the other ranks wait at the barrier
    solo = None
    if world > 1 and not args.no_solo:
        if rank == 0:
            wl.free()  # (no empty_cache: a driver free's background wipe would slow the solo leg)
            try:
                one = Workload(args.workload, ctx, dev, 1, 0)
                torch.cuda.synchronize()
                solo_steps = max(1, min(args.steps, 200 if args.workload == "B" else 20))
                # the headline's settle rule: the buffers were just allocated
                # and filled, and the N-rank region's frees may still be wiped in the background
                el1, avg1, _, n1, _ = run_timed(one, solo_steps, min(args.warmup, 3), args.settle, [stream], 1, None,
                                                settle_s=args.settle_s if args.settle > 0 else 0.0)
                ok1, _ = one.check(None)
                solo = {"value": round(one.total_bytes * solo_steps / el1 / 2**30, 2), "steps": solo_steps,
                        "ms_per_step": round(el1 / solo_steps * 1e3, 4), "bitexact_vs_golden": ok1,
                        "settle_launches": max(0, n1 - min(args.warmup, 3)),
                        "settle_rule": f">= {args.settle} launches and >= {args.settle_s if args.settle > 0 else 0} s, "
                                       "then a steady launch rate (the headline's)",
                        "what": f"workload {args.workload} at N = 1 (the whole batch) on rank 0's GPU, timed after "
                                "the N-rank region while the other ranks wait"}
                one.free()
            except Exception as e:  # the efficiency leg must never cost the N-rank line
                solo = {"error": f"{type(e).__name__}: {e}"[:300]}
                torch.cuda.empty_cache()
        dist.barrier()
    wl.free()  # (kept in the caching allocator: see secondary_configs)

    # ---- N = 1 extras (rank 0 only): secondary configs, end-to-end, CPU baseline
    def optional(fn):  # an extra leg must never cost the headline line
        try:
            return fn()
        except Exception as e:
            torch.cuda.empty_cache()
            return {"error": f"{type(e).__name__}: {e}"[:300]}

    configs = None
    cfg_names = args.configs if args.configs is not None else ("C,Cu,D,Du,S,Usmall,S_short,S_mixed,S_large" if args.workload == "B"
                                                               else "none")
    if world == 1 and cfg_names != "none":
        configs = optional(lambda: secondary_configs(ctx, dev, [c for c in cfg_names.split(",") if c],
                                                     args.config_iters))
    e2e = None
    if world == 1 and not args.no_e2e and args.workload == "B":
        e2e = optional(lambda: end_to_end(ctx, gpu))
    cpu = None
    if world == 1 and not args.no_cpu_baseline and args.workload == "B":
        def cpu_leg():
            wl_b = Workload("B", ctx, dev, 1, 0)
            samples = cpu_samples(dev, wl_b.bufs)
            wl_b.free()
            torch.cuda.empty_cache()
            return cpu_baseline(samples, args.cpu_runs)
        cpu = optional(cpu_leg)

    traffic, traffic_source = None, None
    # PMC-measured HBM bytes per config-B launch (tools/summarize_profile.py), read from the
    # committed profile: PMC passes are separate rocprofv3 runs, not part of this process; other
    # workloads' launches are a different size, so no figure for them
    tfile = ROOT / "profiles" / "traffic_uniform4k.json"
    if tfile.exists() and args.workload == "B":
        try:
            tj = json.loads(tfile.read_text())
            traffic = tj.get("hbm_bytes_per_launch")
            traffic_source = (f"profiles/traffic_uniform4k.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, "
                              f"{tj.get('source', '?')}; not measured in this run)")
        except (OSError, ValueError):
            traffic = None

    if rank == 0:
        total_bytes = total_step_bytes * args.steps
        if args.workload == "B":
            workload = {"workload": "B: 65,536 x 4 KiB payloads per GPU per step, one CRC32 (IEEE, "
                                    "client/checksum.cc default build) each", "messages_per_gpu": nmsg,
                        "message_bytes": MSG_BYTES, "batches_rotated": ROTATE,
                        "parallelism": f"independent message shards x{world}", "streams": args.streams}
            scaling = "weak"
        elif args.workload == "C":
            workload = {"workload": "C: 1 Mi messages, 64 B - 1 MiB log-uniform (117.8 GB), one CRC32 each, "
                                    "contiguous shards balanced by bytes", "messages_total": int(bounds[-1]),
                        "messages_rank0": nmsg, "bytes_total": total_step_bytes,
                        "parallelism": f"contiguous byte-balanced shards x{world}, RCCL all_gather of CRCs "
                                       "(timed separately)",
                        "gather": gather,
                        "value_incl_gather": round(total_bytes / (elapsed + args.steps * gather_ms * 1e-3) / 2**30, 2)
                        if gather_ms is not None else None}
            scaling = "strong"
        else:
            workload = {"workload": "E: 8 Mi x 4 KiB payloads per step, round-robin over the GPUs, one CRC32 each",
                        "messages_total": E_COUNT, "messages_per_gpu": nmsg, "message_bytes": MSG_BYTES,
                        "parallelism": f"round-robin message shards x{world}, RCCL all_gather of CRCs "
                                       "(timed separately)",
                        "gather": gather,
                        # the same rate with one device gather of every step's CRCs added per step
                        "value_incl_gather": round(total_bytes / (elapsed + args.steps * gather_ms * 1e-3) / 2**30, 2)
                        if gather_ms is not None else None}
            scaling = "strong"
        value = total_bytes / elapsed / 2**30
        achieved = step_bytes / (avg_kern_ms * 1e-3) / 1e9
        kernel = {"B": "subspace_amd::crc32_uniform4k_kernel<512, false, false>",
                  "E": "subspace_amd::crc32_uniform4k_kernel<512, false, false>",
                  "C": "subspace_amd::crc32_ragged_kernel<512> + prep (whole call)"}[args.workload]
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
            "per_gpu_value": round(value / world, 2),
            "bitexact_vs_golden": bitexact,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_source,
                         "kernel": kernel,
                         "avg_launch_ms": round(avg_kern_ms, 4),
                         "launch_ms_source": f"HIP event span of rank 0's timed region / K ({args.streams} stream(s), "
                                             "consecutive launches overlap when 2)",
                         "sampled_launch_ms": round(sampled_ms, 4) if sampled_ms else None},
        }
        if ceiling is not None:
            line["roofline"]["read_ceiling"] = ceiling
            if "GBps" in ceiling:
                line["roofline"]["frac_of_read_ceiling"] = round(achieved / ceiling["GBps"], 4)
        steps_ms = [r["step_ms"] for r in everyone]
        line["ranks"] = everyone
        line["rank_step_ms"] = {"min": min(steps_ms), "max": max(steps_ms)}
        line["distinct_gpus"] = len({r["pci"] + r["uuid"] for r in everyone})
        if dist_on:
            line["rccl_world"] = dist.get_world_size()
            line["backend"] = dist.get_backend()
        if solo is not None:
            line["single_gpu"] = solo
            line["efficiency"] = round(value / (world * solo["value"]), 4) if "value" in solo else None
        line["configs"] = configs
        line["cpu_baseline"] = cpu
        line["e2e_pcie"] = e2e
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
