"""GPU parity on the CRC-32C polynomial (a -msse4.2 reference build's SubspaceCRC32,
client/checksum.cc:56-76): a context created with SUBSPACE_CRC_POLY_CASTAGNOLI runs the
same kernels with Castagnoli tables and operators; every result is checked bit for bit
against the oracle's CRC-32C restatement (pinned by tests/golden/crc32c_kat.json)."""
import json
from pathlib import Path

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from subspace_amd import gpu, slots, synth  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"
M32 = 0xFFFFFFFF
KAT = json.loads((Path(__file__).parent / "golden" / "crc32c_kat.json").read_text())["kats"]


def test_known_answers_on_device(gpu_ctx_c):
    for k in KAT:
        data = bytes.fromhex(k["data_hex"])
        buf = torch.frombuffer(bytearray(data + bytes(16)), dtype=torch.uint8).to(DEV)
        out = torch.zeros(1, dtype=torch.int32, device=DEV)
        gpu_ctx_c.crc32_ragged(buf, torch.zeros(1, dtype=torch.int64, device=DEV),
                               torch.full((1,), len(data), dtype=torch.int64, device=DEV), out, finalize=True)
        torch.cuda.synchronize()
        assert int(out.item()) & M32 == k["checksum"], k["name"]


@pytest.mark.parametrize("count", [1, 7, 4097])
def test_uniform4k(gpu_ctx_c, oracle, count):
    buf = torch.empty(count * 4096, dtype=torch.uint8, device=DEV)
    gpu.fill_uniform(buf, 4096, 4096, count, seed=0xC32C)
    out = torch.empty(count, dtype=torch.int32, device=DEV)
    gpu_ctx_c.crc32_uniform(buf, 4096, 4096, count, out)
    torch.cuda.synchronize()
    want = oracle.synth_crc_batch(0xC32C, np.full(count, 4096, dtype=np.uint64), castagnoli=True)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


@pytest.mark.parametrize("align,lead", [(64, 0), (1, 5)])
def test_ragged(gpu_ctx_c, oracle, align, lead):
    rng = np.random.default_rng(align + lead)
    lengths = rng.integers(0, 50000, 1500).astype(np.uint64)
    lengths[::13] = rng.integers(0, 200, len(lengths[::13]))
    lengths[-2:] = [(3 << 20) + 7, 8192 * 5]
    offsets, total = synth.packed_offsets(lengths, align)
    offsets = offsets + np.uint64(lead)
    buf = torch.empty(int(total) + lead + 64, dtype=torch.uint8, device=DEV)
    d_off = torch.from_numpy(offsets.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lengths.view(np.int64)).to(DEV)
    gpu.fill_ragged(buf, d_off, d_len, seed=0xC32D)
    out = torch.empty(len(lengths), dtype=torch.int32, device=DEV)
    gpu_ctx_c.crc32_ragged(buf, d_off, d_len, out, init=0x12345678)
    torch.cuda.synchronize()
    want = oracle.synth_crc_batch(0xC32D, lengths, init=0x12345678, castagnoli=True)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


def test_slots_publish_and_verify(gpu_ctx_c, oracle):
    count, cs, ms = 3000, 4, 16
    ps = slots.compute_prefix_size(cs, ms)
    stride = slots.slot_stride(4096, cs, ms)
    rng = np.random.default_rng(3)
    sizes = np.full(count, 4096, dtype=np.uint64)
    host = rng.integers(0, 256, stride * count, dtype=np.uint8)
    host.reshape(count, stride)[:, :ps] = slots.make_prefixes(count, sizes, checksum_size=cs, metadata_size=ms,
                                                              seed=4)
    want = host.copy()
    po = np.arange(count, dtype=np.uint64) * np.uint64(stride)
    oracle.publish_slots(want, po, po + np.uint64(ps), sizes, cs, ms, castagnoli=True)
    dev = torch.from_numpy(host).to(DEV)
    gpu_ctx_c.crc32_slots_strided(dev, stride, count, message_size=4096, checksum_size=cs, metadata_size=ms,
                                  mode=gpu.SLOT_CALCULATE)
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), want)
    dev[17 * stride + ps + 100] ^= 1
    status = torch.zeros(count, dtype=torch.int32, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    gpu_ctx_c.crc32_slots_strided(dev, stride, count, message_size=4096, checksum_size=cs, metadata_size=ms,
                                  mode=gpu.SLOT_VERIFY, status=status, error_count=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 1 and np.nonzero(status.cpu().numpy())[0].tolist() == [17]


def test_bad_polynomial_rejected():
    with pytest.raises(gpu.CrcError):
        gpu.CrcContext(0, poly=0x04C11DB7)  # non-reflected form: no x^0 term in bit 31
