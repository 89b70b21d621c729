"""Full-size BASELINE configs through the C ABI, bit-exact against the committed fixtures.

These run FIRST in a `pytest -m gpu` session (tests/conftest.py orders them ahead of every
other test), each independent of the others, so that a failure elsewhere under `-x` can
never leave a BASELINE config unexercised. The fixture hashes in tests/golden/configs.json
are SHA-256 digests of the whole CRC list computed by the oracle (oracle/crc32_oracle.c,
the restatement of client/checksum.cc:125-130), with sampled messages re-checked against
zlib (tests/golden/make_golden.py).

  B  65,536 x 4 KiB                       uniform 4 KiB kernel
  C  1 Mi messages, 64 B - 1 MiB ragged   ragged kernel (117.8 GB)
  D  256 x 64 MiB                         ragged API and long-message kernel (uniform API)
  E  8 Mi x 4 KiB, round-robin over 8     uniform kernel, shard by shard
  S  65,536 slots, reference layout       fused slot publish + verify (stride 4,160)
"""
import hashlib
import json
from pathlib import Path

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from subspace_amd import gpu, slots, synth  # noqa: E402

pytestmark = [pytest.mark.gpu, pytest.mark.config]
CONFIGS = json.loads((Path(__file__).parent / "golden" / "configs.json").read_text())
DEV = "cuda"


def u64_tensor(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(DEV)


def digest(crcs: np.ndarray) -> str:
    return hashlib.sha256(np.asarray(crcs, dtype="<u4").tobytes()).hexdigest()


def test_config_B_full(gpu_ctx):
    cfg = CONFIGS["B"]
    n = cfg["count"]
    buf = torch.empty(n * 4096, dtype=torch.uint8, device=DEV)
    gpu.fill_uniform(buf, 4096, 4096, n, seed=cfg["seed"])
    out = torch.full((n,), 0xDEAD, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_uniform(buf, 4096, 4096, n, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    assert [int(x) for x in got[:16]] == cfg["first"]
    assert digest(got) == cfg["sha256_le_u32"]


def _ragged(ctx, lengths, seed, align=64):
    offsets, total = synth.packed_offsets(lengths, align)
    buf = torch.empty(int(total) + 64, dtype=torch.uint8, device=DEV)
    d_off, d_len = u64_tensor(offsets), u64_tensor(lengths)
    gpu.fill_ragged(buf, d_off, d_len, seed=seed)
    out = torch.full((len(lengths),), 0xDEAD, dtype=torch.int32, device=DEV)
    ctx.crc32_ragged(buf, d_off, d_len, out)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def test_config_C_full(gpu_ctx):
    cfg = CONFIGS["C"]
    lengths = synth.ragged_lengths(cfg["seed"], cfg["count"])
    free, _ = torch.cuda.mem_get_info()
    need = int(lengths.sum()) + 64 * len(lengths) + (1 << 30)
    if free < need:
        pytest.skip(f"needs {need / 2**30:.0f} GiB free device memory")
    assert digest(_ragged(gpu_ctx, lengths, cfg["seed"])) == cfg["sha256_le_u32"]


def test_config_C_full_unaligned(gpu_ctx):
    """Config C packed back to back with no alignment (every head and tail masked)."""
    cfg = CONFIGS["C"]
    lengths = synth.ragged_lengths(cfg["seed"], cfg["count"])
    free, _ = torch.cuda.mem_get_info()
    if free < int(lengths.sum()) + (1 << 30):
        pytest.skip("not enough free device memory")
    assert digest(_ragged(gpu_ctx, lengths, cfg["seed"], align=1)) == cfg["sha256_le_u32"]


def test_config_D_full(gpu_ctx):
    cfg = CONFIGS["D"]
    got = _ragged(gpu_ctx, np.full(cfg["count"], 64 << 20, dtype=np.uint64), cfg["seed"])
    assert digest(got) == cfg["sha256_le_u32"]


def test_config_D_full_uniform_api(gpu_ctx):
    cfg = CONFIGS["D"]
    n, L = cfg["count"], 64 << 20
    buf = torch.empty(n * L, dtype=torch.uint8, device=DEV)
    gpu.fill_uniform(buf, L, L, n, seed=cfg["seed"])
    out = torch.full((n,), 0xDEAD, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_uniform(buf, L, L, n, out)
    torch.cuda.synchronize()
    assert digest(out.cpu().numpy().view(np.uint32)) == cfg["sha256_le_u32"]


def test_config_E_sharded_full(gpu_ctx):
    """8 Mi x 4 KiB, generated and checksummed shard by shard (message i on shard i mod 8,
    as the 8-GPU run does), gathered and compared with the fixture hash."""
    cfg = CONFIGS["E"]
    n, G = cfg["count"], 8
    full = np.zeros(n, dtype=np.uint32)
    per = n // G
    buf = torch.empty(per * 4096, dtype=torch.uint8, device=DEV)
    out = torch.empty(per, dtype=torch.int32, device=DEV)
    for r in range(G):
        gpu.fill_uniform(buf, 4096, 4096, per, seed=cfg["seed"], first_id=r, id_stride=G)
        gpu_ctx.crc32_uniform(buf, 4096, 4096, per, out)
        torch.cuda.synchronize()
        full[r::G] = out.cpu().numpy().view(np.uint32)
    assert digest(full) == cfg["sha256_le_u32"]


def test_config_S_slots_publish_verify_full(gpu_ctx, oracle):
    """Config B in the reference channel layout (65,536 slots, PrefixSize 64 + 4 KiB, stride
    4,160): device publish must leave the buffer byte-identical to the oracle's publisher
    restatement (client/publisher.cc:664-675, common/channel.h:527-549); device verify passes
    every slot, then flags exactly the corrupted ones (client/client.cc:1346-1356)."""
    count, cs, ms = 65536, 4, 0
    ps = slots.compute_prefix_size(cs, ms)
    stride = slots.slot_stride(4096, cs, ms)
    sizes = np.full(count, 4096, dtype=np.uint64)
    rng = np.random.default_rng(0x5107)
    host = rng.integers(0, 256, stride * count, dtype=np.uint8)
    host.reshape(count, stride)[:, :ps] = slots.make_prefixes(count, sizes, seed=0x5108)
    dev = torch.from_numpy(host).to(DEV)
    status = torch.full((count,), 7, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_slots_strided(dev, stride, count, message_size=4096, mode=gpu.SLOT_CALCULATE, status=status)
    torch.cuda.synchronize()
    po = np.arange(count, dtype=np.uint64) * np.uint64(stride)
    oracle.publish_slots(host, po, po + np.uint64(ps), sizes, cs, ms)
    assert int(status.abs().sum().item()) == 0
    got = dev.cpu().numpy()
    bad = np.nonzero(got != host)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"

    err = torch.full((1,), 9, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_slots_strided(dev, stride, count, message_size=4096, mode=gpu.SLOT_VERIFY, status=status,
                                error_count=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 0 and int(status.abs().sum().item()) == 0
    # corrupt: a payload bit, a span-0 prefix field, the stored checksum; clear one flag
    victims = {3: ps + 4095, 40000: 8, 65535: 48}
    for slot, off in victims.items():
        dev[slot * stride + off] ^= 0x10
    flags_off = 777 * stride + 32
    dev[flags_off] = int(dev[flags_off].item()) & ~slots.MESSAGE_HAS_CHECKSUM
    gpu_ctx.crc32_slots_strided(dev, stride, count, message_size=4096, mode=gpu.SLOT_VERIFY, status=status,
                                error_count=err)
    torch.cuda.synchronize()
    st = status.cpu().numpy()
    assert int(err.item()) == len(victims)
    assert sorted(np.nonzero(st == 1)[0].tolist()) == sorted(victims)
    assert np.nonzero(st == 2)[0].tolist() == [777]  # not checksummed by its publisher: skipped
