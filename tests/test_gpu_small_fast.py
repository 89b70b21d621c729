"""GPU parity of the small-message kernel's FAST loop (crc_small.hip): a wave whose
window holds only whole 4 KiB payloads on 16-B boundaries runs the uniform kernel's loop and a
lean flush. Bit-exact against the oracle for publish and verify (with payload bit flips): every
wave FAST at counts around the tile, wave and ring-window edges and past one 32-tile window per
wave (more workgroups); FAST and general waves in one launch (one non-conforming message -- 4,095
bytes, a 16-B misaligned start, an oversize one -- turns only its own wave general); strided
slots with per-slot sizes (the max_len bound in the FAST test)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from subspace_amd import _lib, gpu, slots  # noqa: E402
from test_gpu_small import oracle_arena, run_slot_list  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"
SIZE = 4096


def fast_list(count, seed, cs=4, ms=0, spoil=()):
    """`count` slots of whole 4 KiB payloads at 64-B aligned starts, shuffled records; `spoil` =
    [(slot, kind)] with kind 'short' (4,095 B), 'mis' (start + 7) or 'over' (5,000 B, beyond the
    bound)."""
    rng = np.random.default_rng(seed)
    ps = slots.compute_prefix_size(cs, ms)
    sizes = np.full(count, SIZE, dtype=np.uint64)
    mis = np.zeros(count, dtype=np.uint64)
    for i, kind in spoil:
        if kind == "short":
            sizes[i] = SIZE - 1
        elif kind == "mis":
            mis[i] = 7
        else:
            sizes[i] = 5000
    room = (sizes + np.uint64(15 + 63)) & ~np.uint64(63)
    pay_off = np.concatenate([[0], np.cumsum(room)[:-1]]).astype(np.uint64) + mis
    pay_host = rng.integers(0, 256, int(room.sum()) + 64, dtype=np.uint8)
    pre_host = slots.make_prefixes(count, sizes, checksum_size=cs, metadata_size=ms, seed=seed + 1).reshape(-1).copy()
    return pre_host, pay_host, pay_off, sizes, rng.permutation(count), ps


def general_waves(ctx, lib, run):
    """Runs `run()` (one slot call) with the kernel's experiment hook on and returns (waves with
    tiles, of which general -- not FAST) from its per-wave records (crc_small.hip: lane 7 stores
    nk << 32 | fast << 48)."""
    waves = int(_lib.load_dev().subspace_crc_testutil_probe_waves(ctx._h, 1 << 22))
    rb = torch.zeros(waves * 8, dtype=torch.int64, device=DEV)
    assert _lib.load_dev().subspace_crc_testutil_probe(ctx._h, rb.data_ptr()) == 0
    try:
        run()
    finally:
        _lib.load_dev().subspace_crc_testutil_probe(ctx._h, None)
    r = rb.cpu().numpy().view(np.uint64).reshape(waves, 8)
    nk = (r[:, 7] >> np.uint64(32)) & np.uint64(0xFFFF)
    fast = (r[:, 7] >> np.uint64(48)) & np.uint64(1)
    live = (nk > 0) & (r[:, 0] > 0)
    return int(live.sum()), int((live & (fast == 0)).sum())


def publish_verify(ctx, oracle, count, seed, cs=4, ms=0, spoil=(), lib=None, general=0):
    pre, pay, pay_off, sizes, order, ps = fast_list(count, seed, cs, ms, spoil)
    got_pre, st, _ = run_slot_list(ctx, pre, pay, pay_off, sizes, order, ps, cs, ms, SIZE, gpu.SLOT_CALCULATE)
    arena, po, yo = oracle_arena(pre, pay, pay_off, count, ps)
    oracle.publish_slots(arena, po, yo, sizes, cs, ms)
    bad = np.nonzero(got_pre != arena[:len(pre)])[0]
    assert len(bad) == 0, f"{len(bad)} prefix bytes differ, first slots {np.unique(bad // ps)[:8]}"
    assert (st == 0).all()
    rng = np.random.default_rng(seed + 2)
    pay2 = pay.copy()
    flips = np.nonzero(rng.random(count) < 0.05)[0]
    for i in flips:
        pay2[int(pay_off[i]) + int(rng.integers(0, int(sizes[i])))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    _, st, err = run_slot_list(ctx, got_pre, pay2, pay_off, sizes, order, ps, cs, ms, SIZE, gpu.SLOT_VERIFY)
    arena2, po, yo = oracle_arena(got_pre, pay2, pay_off, count, ps)
    want = oracle.verify_slots(arena2, po, yo, sizes, cs, ms)
    assert np.array_equal(st, want)
    assert err == int((want == 1).sum())
    if lib is not None:  # the path the test means to cover: `general` waves off the FAST loop
        live, gen = general_waves(ctx, lib, lambda: run_slot_list(ctx, got_pre, pay2, pay_off, sizes, order, ps, cs,
                                                                   ms, SIZE, gpu.SLOT_VERIFY))
        assert live > 0 and gen == general, (live, gen)
    return st


@pytest.mark.parametrize("count", [1, 2, 3, 63, 64, 65, 4095, 4097, 65_536, 65_537])
def test_fast_every_wave(gpu_ctx, oracle, lib, count):
    """Every wave FAST: odd counts (a last tile with one message), one message per wave, full
    32-tile windows (65,536 slots on 256 CUs) and one slot past them."""
    publish_verify(gpu_ctx, oracle, count, 0xFA57 + count, lib=lib)


def test_fast_past_one_window(gpu_ctx, oracle, lib):
    """More slots than 32 tiles per wave on one workgroup per CU: the host adds workgroups, every
    wave still FAST."""
    publish_verify(gpu_ctx, oracle, 150_001, 0xFA58, lib=lib)


@pytest.mark.parametrize("kind", ["short", "mis", "over"])
def test_fast_and_general_waves_in_one_launch(gpu_ctx, oracle, lib, kind):
    """One non-conforming message among 8,191 conforming ones: its workgroup's 8 waves take the
    workgroup repack (REPACK2, round 6: the FAST decision is the workgroup's, its waves share the
    packed tiles), every other workgroup stays FAST; every slot bit-exact (an oversize one:
    computed whole, correct). 8,191 slots on 256 workgroups: 2 tiles per wave, 8 live waves per
    workgroup."""
    publish_verify(gpu_ctx, oracle, 8191, 0xFA59, spoil=[(4000, kind)], lib=lib, general=8)


def test_fast_metadata_span(gpu_ctx, oracle, lib):
    """A 16-B metadata span (prefix 128 B): the same FAST loop, the spans hashed in the prologue."""
    publish_verify(gpu_ctx, oracle, 5000, 0xFA5A, cs=4, ms=16, lib=lib)


def test_fast_strided_per_slot_sizes(gpu_ctx, oracle):
    """subspace_crc32_slots_strided with per-slot sizes, every size 4,096 but one past the slot's
    payload area (OVERSIZE, nothing read) and one of 4,095: the fused small kernel, max_len in the
    FAST test."""
    n, cs, ms = 3000, 4, 0
    ps, stride = slots.compute_prefix_size(cs, ms), slots.slot_stride(SIZE, cs, ms)
    rng = np.random.default_rng(0xFA5B)
    sizes = np.full(n, SIZE, dtype=np.uint64)
    sizes[17], sizes[2000] = SIZE + 64 + 1, SIZE - 1
    host = rng.integers(0, 256, stride * n, dtype=np.uint8)
    host.reshape(n, stride)[:, :ps] = slots.make_prefixes(n, np.minimum(sizes, SIZE), checksum_size=cs,
                                                          metadata_size=ms, seed=3)
    buf = torch.from_numpy(host.copy()).to(DEV)
    d_sizes = torch.from_numpy(sizes.view(np.int64)).to(DEV)
    status = torch.full((n,), 7, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_slots_strided(buf, stride, n, sizes=d_sizes, checksum_size=cs, metadata_size=ms,
                                mode=gpu.SLOT_CALCULATE, status=status)
    torch.cuda.synchronize()
    gpu_ctx.check()
    got = buf.cpu().numpy()
    st = status.cpu().numpy().view(np.uint32)
    want = host.copy()
    live = np.array([i for i in range(n) if i != 17])
    oracle.publish_slots(want, live.astype(np.uint64) * np.uint64(stride),
                         live.astype(np.uint64) * np.uint64(stride) + np.uint64(ps), sizes[live], cs, ms)
    assert st[17] == gpu.SLOT_OVERSIZE and (np.delete(st, 17) == 0).all()
    assert np.array_equal(got, want)
