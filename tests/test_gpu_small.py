"""GPU parity of the small-message kernel (crc_small.hip) through the C ABI, against the
CPU oracle, bit-exact for every message: slot lists (subspace_crc32_slots with
max_message_size <= 4096 -- the subscriber drain's device form), uniform batches of
messages up to 4 KiB, and messages longer than a half-tile (extended length > 4096: a
broken max_message_size bound, a 4 KiB payload off a 16-B boundary), which a wave computes
whole in its flush.
Covers the half-tile edges (lengths 0, 1, 15-17, 127-129, 4080, 4081, 4096, every start
offset & 15), odd counts, init / finalize, several flush windows per wave, the packed forms
(G = 1 ... 16 lanes per message for short messages and short slots), and agreement with the
ragged path on the same records (testutil "small_path" 0).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from subspace_amd import _lib, gpu, slots  # noqa: E402
from test_gpu_parity import M32, expected_uniform, run_uniform  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("length", [1, 15, 16, 17, 127, 128, 129, 1000, 2049, 4080, 4081])
@pytest.mark.parametrize("extra", [0, 3, 13])
def test_uniform_small_lengths(gpu_ctx, oracle, length, extra):
    """Uniform batches of messages < 4 KiB: 16-B aligned strides, and strides that give every
    message its own start offset & 15 (the head mask and the seed Z_mis^{-1}(init))."""
    stride = ((length + 15) & ~15) + extra
    count = 301
    got = run_uniform(gpu_ctx, count, length=length, stride=stride, seed=0x5A11 + length)
    assert np.array_equal(got, expected_uniform(oracle, count, length, 0x5A11 + length))


@pytest.mark.parametrize("length,count", [(128, 300_001), (256, 200_001), (512, 150_001), (1024, 100_001),
                                          (2048, 100_001), (64, 9_999)])
def test_uniform_small_exact_sizes(gpu_ctx, oracle, length, count):
    """Messages of exactly G lines on 16-B boundaries (the packed FAST loop: no masks, codes or
    padding), over several ring windows per wave, with a nonzero init and the final XOR; 64 B:
    the one-lane form's 16-step chain."""
    got = run_uniform(gpu_ctx, count, length=length, stride=length, seed=0x5A15 + length, init=0x9E3779B9,
                      finalize=True)
    want = expected_uniform(oracle, count, length, 0x5A15 + length, init=0x9E3779B9, finalize=True)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, first {bad[:5]}"


@pytest.mark.parametrize("init,finalize", [(0, False), (0x12345678, False), (0xDEADBEEF, True)])
def test_uniform_small_init_finalize(gpu_ctx, oracle, init, finalize):
    got = run_uniform(gpu_ctx, 999, length=777, stride=781, seed=0x5A12, init=init, finalize=finalize)
    assert np.array_equal(got, expected_uniform(oracle, 999, 777, 0x5A12, init=init, finalize=finalize))


def test_uniform_small_flush_windows(gpu_ctx, oracle):
    """600,001 messages of 200 B: ~147 tiles per wave, i.e. three 64-tile flush windows and a
    partial one, and an odd last tile."""
    count = 600_001
    got = run_uniform(gpu_ctx, count, length=200, stride=208, seed=0x5A13)
    want = expected_uniform(oracle, count, 200, 0x5A13)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, first {bad[:5]}"


def build_slot_list(count, seed, cs, ms, max_size, misaligned=0.0, oversize=0.0, over_max=20000):
    """Prefixes in one allocation, payloads in another, records in shuffled order. Payload
    starts are 64-B aligned except a `misaligned` fraction (offset & 15 random); an `oversize`
    fraction of the sizes exceed max_size (up to over_max)."""
    rng = np.random.default_rng(seed)
    ps = slots.compute_prefix_size(cs, ms)
    sizes = rng.integers(0, max_size + 1, count).astype(np.uint64)
    edge = [0, 1, 15, 16, 17, max_size][:count]
    sizes[:len(edge)] = edge
    over = rng.random(count) < oversize
    sizes[over] = rng.integers(max_size + 1, over_max + 1, int(over.sum()))
    mis = np.where(rng.random(count) < misaligned, rng.integers(1, 16, count), 0).astype(np.uint64)
    if count > 6:
        mis[6] = 15  # a full-size message off a 16-B boundary (a long message)
        sizes[6] = max_size
    room = (sizes + np.uint64(15) + np.uint64(63)) & ~np.uint64(63)
    pay_off = np.concatenate([[0], np.cumsum(room)[:-1]]).astype(np.uint64) + mis
    pay_host = rng.integers(0, 256, int(room.sum()) + 64, dtype=np.uint8)
    pre_host = slots.make_prefixes(count, sizes, checksum_size=cs, metadata_size=ms, seed=seed + 1).reshape(-1).copy()
    order = rng.permutation(count)
    return pre_host, pay_host, pay_off, sizes, order, ps


def run_slot_list(ctx, pre_host, pay_host, pay_off, sizes, order, ps, cs, ms, max_size, mode, small=True, lib=None):
    d_pre = torch.from_numpy(pre_host.copy()).to(DEV)
    d_pay = torch.from_numpy(pay_host).to(DEV)
    rec = slots.slot_records(d_pre.data_ptr() + order.astype(np.uint64) * np.uint64(ps),
                             d_pay.data_ptr() + pay_off[order], sizes[order])
    d_rec = torch.from_numpy(rec.view(np.int64)).to(DEV)
    n = len(sizes)
    status = torch.full((n,), 7, dtype=torch.int32, device=DEV)
    err = torch.full((1,), 12345, dtype=torch.int32, device=DEV)
    if lib is not None:
        assert _lib.load_dev().subspace_crc_testutil_set(ctx._h, b"small_path", int(small)) == 0
    try:
        ctx.crc32_slots(d_rec, max_message_size=max_size, checksum_size=cs, metadata_size=ms, mode=mode,
                        status=status, error_count=err if mode == gpu.SLOT_VERIFY else None)
        torch.cuda.synchronize()
        ctx.check()
    finally:
        if lib is not None:
            _lib.load_dev().subspace_crc_testutil_set(ctx._h, b"small_path", 1)
    st = np.empty(n, dtype=np.uint32)
    st[order] = status.cpu().numpy().view(np.uint32)  # back to slot order
    assert np.array_equal(d_pay.cpu().numpy(), pay_host)  # payloads are never written
    return d_pre.cpu().numpy(), st, int(err.item())


def oracle_arena(pre_host, pay_host, pay_off, count, ps):
    arena = np.concatenate([pre_host, pay_host])
    return arena, np.arange(count, dtype=np.uint64) * np.uint64(ps), pay_off + np.uint64(len(pre_host))


@pytest.mark.parametrize("count,cs,ms,misaligned,oversize", [
    (3001, 4, 0, 0.0, 0.0),      # the drain of a 4 KiB channel
    (3001, 4, 16, 0.3, 0.0),     # metadata span, payloads off 16-B boundaries (some longer than a half-tile)
    (999, 20, 32, 0.5, 0.02),    # a broken max_message_size bound: multi-chunk long messages
    (1, 4, 0, 1.0, 0.0),         # one slot
    (1001, 4, 100, 0.2, 0.01),   # metadata over 64 B: the small kernel + the slot-finish kernel
    (1001, 80, 0, 0.2, 0.0),     # a checksum area over 64 B: the same
])
def test_slot_list_small_publish_verify(gpu_ctx, oracle, count, cs, ms, misaligned, oversize):
    pre, pay, pay_off, sizes, order, ps = build_slot_list(count, count + cs + ms, cs, ms, 4096, misaligned, oversize)
    got_pre, st, _ = run_slot_list(gpu_ctx, pre, pay, pay_off, sizes, order, ps, cs, ms, 4096, gpu.SLOT_CALCULATE)
    arena, po, yo = oracle_arena(pre, pay, pay_off, count, ps)
    oracle.publish_slots(arena, po, yo, sizes, cs, ms)
    assert (st == 0).all()
    bad = np.nonzero(got_pre != arena[:len(pre)])[0]
    assert len(bad) == 0, f"{len(bad)} prefix bytes differ, first slots {np.unique(bad // ps)[:8]}"

    # verify the published channel after payload bit flips in a tenth of the slots
    rng = np.random.default_rng(count)
    pay2 = pay.copy()
    for i in np.nonzero(rng.random(count) < 0.1)[0]:
        if sizes[i]:
            pay2[int(pay_off[i]) + int(rng.integers(0, int(sizes[i])))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    _, st, err = run_slot_list(gpu_ctx, got_pre, pay2, pay_off, sizes, order, ps, cs, ms, 4096, gpu.SLOT_VERIFY)
    arena2, po, yo = oracle_arena(got_pre, pay2, pay_off, count, ps)
    want = oracle.verify_slots(arena2, po, yo, sizes, cs, ms)
    assert np.array_equal(st, want)
    assert err == int((want == 1).sum())


@pytest.mark.parametrize("count,max_size,cs,ms,misaligned,oversize", [
    (20_001, 64, 4, 0, 0.0, 0.0),     # one lane per slot (G = 1)
    (20_001, 100, 4, 16, 0.2, 0.02),  # G = 1, payloads off 16-B boundaries past their line: long path
    (50_001, 256, 4, 0, 0.1, 0.0),    # G = 2
    (9_999, 700, 8, 5, 0.3, 0.01),    # G = 8
    (9_999, 2000, 4, 0, 0.2, 0.0),    # G = 16
    (300_001, 200, 4, 0, 0.0, 0.0),   # G = 2, several ring windows (2 tiles each) per wave
])
def test_slot_list_packed(gpu_ctx, oracle, count, max_size, cs, ms, misaligned, oversize):
    """Slot lists of short slots: max_message_size picks G = the lanes per slot (crc_small.hip:
    64 / G slots per tile), bit-exact publish and verify against the oracle for every slot,
    including ones longer than the bound or off a 16-B boundary past their G lines (computed
    whole by the flush)."""
    pre, pay, pay_off, sizes, order, ps = build_slot_list(count, count + max_size, cs, ms, max_size, misaligned,
                                                          oversize, over_max=max_size * 3 + 50)
    got_pre, st, _ = run_slot_list(gpu_ctx, pre, pay, pay_off, sizes, order, ps, cs, ms, max_size, gpu.SLOT_CALCULATE)
    arena, po, yo = oracle_arena(pre, pay, pay_off, count, ps)
    oracle.publish_slots(arena, po, yo, sizes, cs, ms)
    assert (st == 0).all()
    bad = np.nonzero(got_pre != arena[:len(pre)])[0]
    assert len(bad) == 0, f"{len(bad)} prefix bytes differ, first slots {np.unique(bad // ps)[:8]}"
    rng = np.random.default_rng(count + 1)
    pay2 = pay.copy()
    for i in np.nonzero(rng.random(count) < 0.1)[0]:
        if sizes[i]:
            pay2[int(pay_off[i]) + int(rng.integers(0, int(sizes[i])))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    _, st, err = run_slot_list(gpu_ctx, got_pre, pay2, pay_off, sizes, order, ps, cs, ms, max_size, gpu.SLOT_VERIFY)
    arena2, po, yo = oracle_arena(got_pre, pay2, pay_off, count, ps)
    want = oracle.verify_slots(arena2, po, yo, sizes, cs, ms)
    assert np.array_equal(st, want)
    assert err == int((want == 1).sum())


@pytest.mark.parametrize("gen_max,count,spoil,cs,ms", [(100, 20_001, 0, 4, 0), (300, 50_001, 0, 4, 0),
                                                      (1500, 9_999, 0, 4, 0), (2000, 30_001, 0, 4, 0),
                                                      (700, 30_001, 3000, 4, 0), (500, 20_001, 0, 8, 16),
                                                      (500, 20_001, 0, 4, 100)])
def test_slot_list_repack(gpu_ctx, oracle, lib, gen_max, count, spoil, cs, ms):
    """A channel of 4 KiB slots (max_message_size 4096) carrying shorter messages: every wave
    that is not FAST packs its window (crc_small.hip REPACK: 2^c lanes per message by size, the
    uniform or the sorted layout); `spoil` puts one 3,000-B message in every 50th window (one
    32-lane group among short ones: the sorted layout); a metadata span (fused), and metadata
    over 64 B (the small kernel + the slot-finish kernel). Publish and verify bit-exact against
    the oracle (payload starts off 16-B boundaries included)."""
    pre, pay, pay_off, sizes, order, ps = build_slot_list(count, count + gen_max, cs, ms, gen_max, 0.2, 0.0)
    if spoil:  # (payload room: build_slot_list sized it for gen_max, so give the slot a fresh area)
        extra = []
        for i in range(0, count, 64 * 50):
            off = len(pay) + len(extra) * (spoil + 64)
            extra.append(i)
            pay_off[i] = off
            sizes[i] = spoil
        pay = np.concatenate([pay, np.random.default_rng(7).integers(0, 256, len(extra) * (spoil + 64) + 64,
                                                                      dtype=np.uint8)])
        pre = slots.make_prefixes(count, sizes, checksum_size=cs, metadata_size=ms, seed=count + gen_max + 1)
        pre = pre.reshape(-1).copy()
    got_pre, st, _ = run_slot_list(gpu_ctx, pre, pay, pay_off, sizes, order, ps, cs, ms, 4096, gpu.SLOT_CALCULATE)
    arena, po, yo = oracle_arena(pre, pay, pay_off, count, ps)
    oracle.publish_slots(arena, po, yo, sizes, cs, ms)
    assert (st == 0).all()
    bad = np.nonzero(got_pre != arena[:len(pre)])[0]
    assert len(bad) == 0, f"{len(bad)} prefix bytes differ, first slots {np.unique(bad // ps)[:8]}"
    rng = np.random.default_rng(count + 3)
    pay2 = pay.copy()
    for i in np.nonzero(rng.random(count) < 0.1)[0]:
        if sizes[i]:
            pay2[int(pay_off[i]) + int(rng.integers(0, int(sizes[i])))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    _, st, err = run_slot_list(gpu_ctx, got_pre, pay2, pay_off, sizes, order, ps, cs, ms, 4096, gpu.SLOT_VERIFY)
    arena2, po, yo = oracle_arena(got_pre, pay2, pay_off, count, ps)
    want = oracle.verify_slots(arena2, po, yo, sizes, cs, ms)
    assert np.array_equal(st, want)
    assert err == int((want == 1).sum())
    if ms <= 64:  # the fused kernel: which waves repacked, from its per-wave records
        r = wave_records(gpu_ctx, lib, lambda: run_slot_list(gpu_ctx, got_pre, pay2, pay_off, sizes, order, ps, cs,
                                                              ms, 4096, gpu.SLOT_VERIFY))
        live = (r[:, 0] > 0) & (((r[:, 7] >> np.uint64(32)) & np.uint64(0xFFFF)) > 0)
        rp = ((r[:, 7] >> np.uint64(49)) & np.uint64(1)) == 1
        assert int((live & ~rp).sum()) == 0 and int((live & rp).sum()) > 0


def wave_records(ctx, lib, run):
    """The fused slot kernel's per-wave experiment records (crc_small.hip PROBE: lane 7 = nk << 32
    | fast << 48 | repack << 49 | packed tiles << 52) for one call `run()`."""
    waves = int(_lib.load_dev().subspace_crc_testutil_probe_waves(ctx._h, 1 << 22))
    rb = torch.zeros(waves * 8, dtype=torch.int64, device=DEV)
    assert _lib.load_dev().subspace_crc_testutil_probe(ctx._h, rb.data_ptr()) == 0
    try:
        run()
    finally:
        _lib.load_dev().subspace_crc_testutil_probe(ctx._h, None)
    return rb.cpu().numpy().view(np.uint64).reshape(waves, 8)


def test_slot_list_small_matches_ragged(gpu_ctx, lib):
    """The same records through the small-message kernel and through the ragged pipeline."""
    count, cs, ms = 4000, 8, 5
    pre, pay, pay_off, sizes, order, ps = build_slot_list(count, 4242, cs, ms, 4096, 0.2, 0.01)
    a, _, _ = run_slot_list(gpu_ctx, pre, pay, pay_off, sizes, order, ps, cs, ms, 4096, gpu.SLOT_CALCULATE,
                            small=True, lib=lib)
    b, _, _ = run_slot_list(gpu_ctx, pre, pay, pay_off, sizes, order, ps, cs, ms, 4096, gpu.SLOT_CALCULATE,
                            small=False, lib=lib)
    assert np.array_equal(a, b)


def test_slot_list_all_long_then_none(gpu_ctx, oracle):
    """Every message longer than the bound (all computed whole by the flushes), then a call
    with none, on the same context."""
    count, cs, ms = 300, 4, 0
    pre, pay, pay_off, sizes, order, ps = build_slot_list(count, 77, cs, ms, 4096, 0.5, 1.0, over_max=40000)
    got_pre, st, _ = run_slot_list(gpu_ctx, pre, pay, pay_off, sizes, order, ps, cs, ms, 4096, gpu.SLOT_CALCULATE)
    arena, po, yo = oracle_arena(pre, pay, pay_off, count, ps)
    oracle.publish_slots(arena, po, yo, sizes, cs, ms)
    assert np.array_equal(got_pre, arena[:len(pre)])
    pre, pay, pay_off, sizes, order, ps = build_slot_list(2001, 78, cs, ms, 4096)
    got_pre, st, _ = run_slot_list(gpu_ctx, pre, pay, pay_off, sizes, order, ps, cs, ms, 4096, gpu.SLOT_CALCULATE)
    arena, po, yo = oracle_arena(pre, pay, pay_off, 2001, ps)
    oracle.publish_slots(arena, po, yo, sizes, cs, ms)
    assert np.array_equal(got_pre, arena[:len(pre)])


def test_small_paths_graph_capture(gpu_ctx, oracle):
    """The fused small-slot kernel (no context workspace: a counter word of the ring) and a
    small uniform batch (offsets materialised once beforehand) captured into a HIP graph and
    replayed; a payload byte flipped between replays must flip exactly that slot's status and
    the mismatch count (the captured counter word is back at 0 after every replay)."""
    count, cs, ms = 2001, 4, 16
    pre, pay, pay_off, sizes, order, ps = build_slot_list(count, 99, cs, ms, 4096)
    got_pre, _, _ = run_slot_list(gpu_ctx, pre, pay, pay_off, sizes, order, ps, cs, ms, 4096, gpu.SLOT_CALCULATE)
    d_pre = torch.from_numpy(got_pre.copy()).to(DEV)
    d_pay = torch.from_numpy(pay.copy()).to(DEV)
    rec = slots.slot_records(d_pre.data_ptr() + order.astype(np.uint64) * np.uint64(ps),
                             d_pay.data_ptr() + pay_off[order], sizes[order])
    d_rec = torch.from_numpy(rec.view(np.int64)).to(DEV)
    status = torch.full((count,), 7, dtype=torch.int32, device=DEV)
    err = torch.full((1,), 12345, dtype=torch.int32, device=DEV)
    n, L, stride = 999, 777, 781
    ubuf = torch.empty(stride * (n - 1) + L, dtype=torch.uint8, device=DEV)
    gpu.fill_uniform(ubuf, stride, L, n, seed=0x5A14)
    uout = torch.zeros(n, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_uniform(ubuf, stride, L, n, uout)  # allocates the materialised offsets
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            gpu_ctx.crc32_slots(d_rec, max_message_size=4096, checksum_size=cs, metadata_size=ms,
                                mode=gpu.SLOT_VERIFY, status=status, error_count=err)
            gpu_ctx.crc32_uniform(ubuf, stride, L, n, uout)
    torch.cuda.synchronize()
    want_u = expected_uniform(oracle, n, L, 0x5A14)
    victim = int(np.nonzero(sizes > 0)[0][3])  # a slot with a payload (slot order)
    pos = int(order.tolist().index(victim))    # its record
    for flipped in (False, True, False):
        if flipped:
            d_pay[int(pay_off[victim])] ^= 0x40
        elif d_pay[int(pay_off[victim])].item() != pay[int(pay_off[victim])]:
            d_pay[int(pay_off[victim])] ^= 0x40
        uout.zero_()
        err.fill_(12345)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        st = status.cpu().numpy().view(np.uint32)
        assert int(err.item()) == (1 if flipped else 0)
        assert st[pos] == (1 if flipped else 0) and int((st != 0).sum()) == (1 if flipped else 0)
        assert np.array_equal(uout.cpu().numpy().view(np.uint32), want_u)
    gpu_ctx.check()
