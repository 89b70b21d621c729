"""The uniform kernel's PROBE instantiation (tools/wave_timeline.py): same results as the
product kernel, and one well-formed timestamp record per wave."""
import ctypes

import numpy as np
import pytest

from subspace_amd import _lib

pytestmark = pytest.mark.gpu

N, SIZE = 65536, 4096


def _probe_lib(gpu_ctx):
    lib = _lib.load()
    return lib


def _check_records(rec, ntiles):
    t = rec[:, :4]
    assert (t > 0).all()
    entry, barrier, loop_end, exit_ = t.T
    landed = rec[:, 7]
    assert (entry <= rec[:, 4]).all() and (rec[:, 4] <= barrier).all()
    assert (barrier <= landed).all() and (landed <= loop_end).all() and (loop_end <= exit_).all()
    nk = rec[:, 5] >> 32
    assert int(nk.sum()) == ntiles  # every tile is some wave's, once
    assert set(np.unique(rec[:, 5] & 0xF)) <= set(range(8))  # XCC_ID
    # 100 MHz clock: a 256 MiB launch spans tens of microseconds, not seconds
    assert 0 < (exit_.max() - entry.min()) < 100_000


def test_probe_uniform_matches_product(gpu_ctx):
    import torch
    from subspace_amd import gpu
    lib = _probe_lib(gpu_ctx)
    waves = int(_lib.load_dev().subspace_crc_testutil_probe_waves(gpu_ctx._h, N))
    buf = torch.empty(N * SIZE, dtype=torch.uint8, device="cuda")
    gpu.fill_uniform(buf, SIZE, SIZE, N, seed=0x5EED000B)
    ref = torch.empty(N, dtype=torch.int32, device="cuda")
    out = torch.empty_like(ref)
    gpu_ctx.crc32_uniform(buf, SIZE, SIZE, N, ref)
    rec = torch.zeros((waves, 8), dtype=torch.int64, device="cuda")
    _lib.load_dev().subspace_crc_testutil_probe(gpu_ctx._h, ctypes.c_void_p(rec.data_ptr()))
    try:
        gpu_ctx.crc32_uniform(buf, SIZE, SIZE, N, out)
    finally:
        _lib.load_dev().subspace_crc_testutil_probe(gpu_ctx._h, None)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    r = rec.cpu().numpy()
    _check_records(r, N // 2)
    assert ((r[:, 6] >> 32) == 0).all()  # no slot finishing in the plain kernel
    hw = r[:, 6] & 0xFFFFFFFF  # HW_ID: waves w and w + 4 of a workgroup share a SIMD
    simd = (hw >> 4) & 3
    assert (simd.reshape(-1, 8)[:, :4] == simd.reshape(-1, 8)[:, 4:]).all()


def test_probe_slots_matches_product(gpu_ctx):
    import torch
    from subspace_amd import gpu, slots
    lib = _probe_lib(gpu_ctx)
    n = 4099  # odd: the last tile has one slot
    waves = int(_lib.load_dev().subspace_crc_testutil_probe_waves(gpu_ctx._h, n))
    ps, stride = slots.compute_prefix_size(4, 0), slots.slot_stride(SIZE, 4, 0)
    host = np.random.default_rng(11).integers(0, 256, stride * n, dtype=np.uint8)
    host.reshape(n, stride)[:, :ps] = slots.make_prefixes(n, np.full(n, SIZE, dtype=np.uint64), checksum_size=4,
                                                          metadata_size=0, seed=11)
    a = torch.from_numpy(host.copy()).cuda()
    b = torch.from_numpy(host.copy()).cuda()
    gpu_ctx.crc32_slots_strided(a, stride, n, message_size=SIZE, mode=gpu.SLOT_CALCULATE)
    rec = torch.zeros((waves, 8), dtype=torch.int64, device="cuda")
    _lib.load_dev().subspace_crc_testutil_probe(gpu_ctx._h, ctypes.c_void_p(rec.data_ptr()))
    try:
        gpu_ctx.crc32_slots_strided(b, stride, n, message_size=SIZE, mode=gpu.SLOT_CALCULATE)
    finally:
        _lib.load_dev().subspace_crc_testutil_probe(gpu_ctx._h, None)
    torch.cuda.synchronize()
    assert torch.equal(a, b)  # identical prefixes written
    r = rec.cpu().numpy()
    _check_records(r, (n + 1) // 2)
    # waves 0-3 of each workgroup finish the slots, between their loop end and their exit
    # (the record keeps the clock's low 32 bits)
    fin = (r[:, 6] >> 32).reshape(-1, 8)
    lo = lambda x: (x & 0xFFFFFFFF).reshape(-1, 8)  # noqa: E731
    assert (fin[:, 4:] == 0).all()
    assert ((fin[:, :4] - lo(r[:, 2])[:, :4]) % (1 << 32) <= (lo(r[:, 3])[:, :4] - lo(r[:, 2])[:, :4]) % (1 << 32)).all()
