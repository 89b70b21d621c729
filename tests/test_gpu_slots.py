"""GPU parity of the message-slot checksums (subspace_crc32_slots / _slots_strided).

A channel buffer is built on the host (prefix fields as a publisher fills them, random
metadata and padding, random payloads), copied to the device, published (CALCULATE) by
the HIP path and by the oracle's publisher restatement on the host copy; the two buffers
must be byte-identical (only the flag and the checksum word change). VERIFY statuses
after targeted corruptions must equal the oracle's subscriber restatement.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from subspace_amd import gpu, slots  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"


def build_channel(count, slot_size, cs, ms, sizes, seed):
    ps = slots.compute_prefix_size(cs, ms)
    stride = slots.slot_stride(slot_size, cs, ms)
    rng = np.random.default_rng(seed)
    host = rng.integers(0, 256, stride * count, dtype=np.uint8)
    host.reshape(count, stride)[:, :ps] = slots.make_prefixes(count, sizes, checksum_size=cs, metadata_size=ms,
                                                              seed=seed + 1)
    return host, ps, stride


def offsets(count, stride, ps):
    po = np.arange(count, dtype=np.uint64) * np.uint64(stride)
    return po, po + np.uint64(ps)


def publish_strided(ctx, host, stride, count, cs, ms, sizes=None, message_size=0):
    dev = torch.from_numpy(host).to(DEV)
    status = torch.full((count,), 7, dtype=torch.int32, device=DEV)
    d_sizes = None if sizes is None else torch.from_numpy(np.asarray(sizes, dtype=np.int64)).to(DEV)
    ctx.crc32_slots_strided(dev, stride, count, message_size=message_size, sizes=d_sizes, checksum_size=cs,
                            metadata_size=ms, mode=gpu.SLOT_CALCULATE, status=status)
    torch.cuda.synchronize()
    return dev, status.cpu().numpy()


@pytest.mark.parametrize("cs,ms", [(4, 0), (4, 16), (20, 32), (8, 5), (5, 7), (6, 64), (7, 61), (4, 65), (30, 1)])
def test_publish_uniform_4k(gpu_ctx, oracle, cs, ms):
    """Contiguous 4 KiB slots, publish byte-identical to the oracle. metadata_size <= 64 goes
    through the fused slot kernel (span 1 folded in by the finishing waves, at every byte
    alignment of 48 + checksum_size); 65 through the payload kernel + slot finish kernel."""
    count = 1500
    sizes = np.full(count, 4096, dtype=np.uint64)
    host, ps, stride = build_channel(count, 4096, cs, ms, sizes, seed=cs * 100 + ms)
    dev, status = publish_strided(gpu_ctx, host, stride, count, cs, ms, message_size=4096)
    po, yo = offsets(count, stride, ps)
    oracle.publish_slots(host, po, yo, sizes, cs, ms)
    assert (status == 0).all()
    got = dev.cpu().numpy()
    bad = np.nonzero(got != host)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]} (stride {stride})"


@pytest.mark.parametrize("slot_size,cs,ms", [(256, 4, 16), (5000, 20, 32), (70000, 4, 0)])
def test_publish_ragged_sizes(gpu_ctx, oracle, slot_size, cs, ms):
    count = 700
    rng = np.random.default_rng(slot_size)
    sizes = rng.integers(0, slot_size + 1, count).astype(np.uint64)
    sizes[:3] = [0, 1, slot_size]
    host, ps, stride = build_channel(count, slot_size, cs, ms, sizes, seed=slot_size + cs)
    dev, status = publish_strided(gpu_ctx, host, stride, count, cs, ms, sizes=sizes)
    po, yo = offsets(count, stride, ps)
    oracle.publish_slots(host, po, yo, sizes, cs, ms)
    assert (status == 0).all()
    assert np.array_equal(dev.cpu().numpy(), host)


def test_publish_slot_list_split_buffers(gpu_ctx, oracle):
    """subspace_crc32_slots: prefixes in one allocation, payloads in another at unaligned
    addresses, slots in shuffled order (split buffers, client_channel.h:126-129)."""
    count, cs, ms = 900, 4, 24
    ps = slots.compute_prefix_size(cs, ms)
    rng = np.random.default_rng(5)
    sizes = rng.integers(0, 20000, count).astype(np.uint64)
    pre_host = slots.make_prefixes(count, sizes, checksum_size=cs, metadata_size=ms, seed=6).reshape(-1).copy()
    gaps = rng.integers(0, 40, count).astype(np.uint64)
    pay_off = np.concatenate([[0], np.cumsum(sizes + gaps)[:-1]]).astype(np.uint64) + np.uint64(3)
    pay_host = rng.integers(0, 256, int(pay_off[-1] + sizes[-1] + 64), dtype=np.uint8)
    d_pre = torch.from_numpy(pre_host).to(DEV)
    d_pay = torch.from_numpy(pay_host).to(DEV)
    order = rng.permutation(count)
    rec = slots.slot_records(d_pre.data_ptr() + order.astype(np.uint64) * np.uint64(ps),
                             d_pay.data_ptr() + pay_off[order], sizes[order])
    d_rec = torch.from_numpy(rec.view(np.int64)).to(DEV)
    status = torch.full((count,), 7, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_slots(d_rec, max_message_size=20000, checksum_size=cs, metadata_size=ms,
                        mode=gpu.SLOT_CALCULATE, status=status)
    torch.cuda.synchronize()
    # oracle over one host arena holding both buffers
    arena = np.concatenate([pre_host, pay_host])
    oracle.publish_slots(arena, np.arange(count, dtype=np.uint64) * np.uint64(ps),
                         pay_off + np.uint64(len(pre_host)), sizes, cs, ms)
    assert (status.cpu().numpy() == 0).all()
    assert np.array_equal(d_pre.cpu().numpy(), arena[:len(pre_host)])
    assert np.array_equal(d_pay.cpu().numpy(), pay_host)  # payloads untouched


def test_verify_statuses(gpu_ctx, oracle):
    count, slot_size, cs, ms = 2000, 4096, 4, 16
    sizes = np.full(count, 4096, dtype=np.uint64)
    sizes[1::7] = np.arange(len(sizes[1::7])) % 4097
    host, ps, stride = build_channel(count, slot_size, cs, ms, sizes, seed=77)
    po, yo = offsets(count, stride, ps)
    oracle.publish_slots(host, po, yo, sizes, cs, ms)
    rng = np.random.default_rng(78)
    kinds = rng.integers(0, 8, count)
    for i, k in enumerate(kinds):
        b = int(po[i])
        n = int(sizes[i])
        if k == 1 and n:
            host[b + ps + rng.integers(0, n)] ^= np.uint8(1 << rng.integers(0, 8))  # payload bit flip
        elif k == 2:
            host[b + 48 + cs + rng.integers(0, ms)] ^= 0x10  # metadata
        elif k == 3:
            host[b + 4 + rng.integers(0, 44)] ^= 0x01  # span 0 (any field)
        elif k == 4:
            host[b + 48 + rng.integers(0, 4)] ^= 0x80  # stored checksum
        elif k == 5:
            host[b:b + 4] ^= 0xFF  # padding word: not covered
            host[b + 48 + cs + ms:b + ps] ^= 0xAA  # prefix padding: not covered
        elif k == 6:
            host[b + 32] &= 0xFB  # no kMessageHasChecksum: not checked
    want = oracle.verify_slots(host, po, yo, sizes, cs, ms)
    assert set(np.unique(want)) == {0, 1, 2}
    dev = torch.from_numpy(host).to(DEV)
    d_sizes = torch.from_numpy(sizes.view(np.int64)).to(DEV)
    status = torch.full((count,), 7, dtype=torch.int32, device=DEV)
    err = torch.full((1,), 12345, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_slots_strided(dev, stride, count, sizes=d_sizes, checksum_size=cs, metadata_size=ms,
                                mode=gpu.SLOT_VERIFY, status=status, error_count=err)
    torch.cuda.synchronize()
    got = status.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want)
    assert int(err.item()) == int((want == 1).sum())
    assert np.array_equal(dev.cpu().numpy(), host)  # verify never writes the channel


def test_verify_roundtrip_uniform_fast_path(gpu_ctx):
    """CALCULATE then VERIFY on the device: every slot passes; one flipped bit fails exactly one."""
    count, cs, ms = 65536, 4, 0
    sizes = np.full(count, 4096, dtype=np.uint64)
    host, ps, stride = build_channel(count, 4096, cs, ms, sizes, seed=9)
    dev = torch.from_numpy(host).to(DEV)
    status = torch.zeros(count, dtype=torch.int32, device=DEV)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_slots_strided(dev, stride, count, message_size=4096, mode=gpu.SLOT_CALCULATE)
    gpu_ctx.crc32_slots_strided(dev, stride, count, message_size=4096, mode=gpu.SLOT_VERIFY, status=status,
                                error_count=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 0 and int(status.abs().sum().item()) == 0
    dev[12345 * stride + ps + 777] ^= 4
    gpu_ctx.crc32_slots_strided(dev, stride, count, message_size=4096, mode=gpu.SLOT_VERIFY, status=status,
                                error_count=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 1
    assert np.nonzero(status.cpu().numpy())[0].tolist() == [12345]


def test_empty_and_errors(gpu_ctx):
    err = torch.full((1,), 9, dtype=torch.int32, device=DEV)
    buf = torch.zeros(4160, dtype=torch.uint8, device=DEV)
    gpu_ctx.crc32_slots_strided(buf, 4160, 0, message_size=4096, mode=gpu.SLOT_VERIFY, error_count=err)
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    with pytest.raises(gpu.CrcError):
        gpu_ctx.crc32_slots_strided(buf, 4160, 1, message_size=4096, mode=5)
    with pytest.raises(gpu.CrcError):
        gpu_ctx.crc32_slots_strided(buf, 4160, 1, message_size=4096, checksum_size=2)
    with pytest.raises(gpu.CrcError):
        gpu_ctx.crc32_slots_strided(buf, 4164, 2, message_size=4096)  # prefixes not 8-B aligned


# ------------------------------------------------------------ host-memory slots (end to end)
@pytest.mark.parametrize("count,cs,ms,pinned", [(1, 4, 0, False), (20001, 4, 0, True), (3000, 20, 32, False)])
def test_host_slots_publish(gpu_ctx, oracle, count, cs, ms, pinned):
    """subspace_crc32_host_slots CALCULATE over a host channel buffer (several ~32 MiB
    chunks for 20,001 slots): byte-identical to the oracle's publisher on a copy."""
    sizes = np.full(count, 4096, dtype=np.uint64)
    host, ps, stride = build_channel(count, 4096, cs, ms, sizes, seed=count + cs)
    want = host.copy()
    po, yo = offsets(count, stride, ps)
    oracle.publish_slots(want, po, yo, sizes, cs, ms)
    if pinned:
        gpu.host_register(host)
    try:
        status = np.full(count, 7, dtype=np.uint32)
        gpu_ctx.crc32_host_slots(host, stride, count, message_size=4096, checksum_size=cs, metadata_size=ms,
                                 mode=gpu.SLOT_CALCULATE, status=status)
    finally:
        if pinned:
            gpu.host_unregister(host)
    assert (status == 0).all()
    bad = np.nonzero(host != want)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"


def test_host_slots_verify_ragged_sizes(gpu_ctx, oracle):
    """VERIFY over a host buffer with per-slot sizes and corruptions: statuses and the
    mismatch count equal the oracle's subscriber; the host buffer is not modified."""
    count, slot_size, cs, ms = 12000, 5000, 4, 8
    rng = np.random.default_rng(11)
    sizes = rng.integers(0, slot_size + 1, count).astype(np.uint64)
    host, ps, stride = build_channel(count, slot_size, cs, ms, sizes, seed=12)
    po, yo = offsets(count, stride, ps)
    oracle.publish_slots(host, po, yo, sizes, cs, ms)
    for i in rng.choice(count, 300, replace=False):
        b = int(po[i])
        if sizes[i]:
            host[b + ps + rng.integers(0, int(sizes[i]))] ^= 0x20
        else:
            host[b + 48] ^= 1
    host[int(po[5]) + 32] &= 0xFB  # unflagged slot: not checked
    want = oracle.verify_slots(host, po, yo, sizes, cs, ms)
    before = host.copy()
    status = np.full(count, 7, dtype=np.uint32)
    errors = gpu_ctx.crc32_host_slots(host, stride, count, sizes=sizes, checksum_size=cs, metadata_size=ms,
                                      mode=gpu.SLOT_VERIFY, status=status)
    assert np.array_equal(status, want)
    assert errors == int((want == 1).sum()) and errors > 0
    assert np.array_equal(host, before)


def test_host_slots_errors(gpu_ctx):
    host = np.zeros(4160 * 2, dtype=np.uint8)
    assert gpu_ctx.crc32_host_slots(host, 4160, 0, message_size=4096, mode=gpu.SLOT_VERIFY) == 0
    with pytest.raises(gpu.CrcError):
        gpu_ctx.crc32_host_slots(host, 4160, 2, message_size=4097)  # does not fit the stride
    with pytest.raises(gpu.CrcError):
        gpu_ctx.crc32_host_slots(host, 4160, 2, sizes=np.array([0, 9999], dtype=np.uint64))
    with pytest.raises(ValueError):
        gpu_ctx.crc32_host_slots(host, 4160, 3, message_size=4096)  # buffer too short


def test_host_slot_list_drain(gpu_ctx, oracle):
    """subspace_crc32_host_slot_list (the subscriber drain hook): a shuffled subset of the
    slots of two registered host channel buffers, verified in place over PCIe; statuses and
    the mismatch count equal the oracle's; then CALCULATE on a subset writes the same
    prefixes as the oracle's publisher."""
    count, slot_size, cs, ms = 4000, 3000, 4, 8
    rng = np.random.default_rng(21)
    chans = []
    for k in range(2):
        sizes = rng.integers(0, slot_size + 1, count).astype(np.uint64)
        host, ps, stride = build_channel(count, slot_size, cs, ms, sizes, seed=30 + k)
        po, yo = offsets(count, stride, ps)
        oracle.publish_slots(host, po, yo, sizes, cs, ms)
        for i in rng.choice(count, 50, replace=False):
            host[int(po[i]) + 48] ^= 0x40  # corrupt stored checksums
        chans.append((host, po, yo, sizes))
    for host, *_ in chans:
        gpu.host_register(host)
    try:
        picks = [(k, int(i)) for k in range(2) for i in rng.choice(count, 1500, replace=False)]
        rng.shuffle(picks)
        rec = slots.slot_records([chans[k][0].ctypes.data + int(chans[k][1][i]) for k, i in picks],
                                 [chans[k][0].ctypes.data + int(chans[k][2][i]) for k, i in picks],
                                 [chans[k][3][i] for k, i in picks])
        status = np.full(len(picks), 7, dtype=np.uint32)
        errors = gpu_ctx.crc32_host_slot_list(rec, max_message_size=slot_size, checksum_size=cs,
                                              metadata_size=ms, mode=gpu.SLOT_VERIFY, status=status)
        want = np.concatenate([oracle.verify_slots(chans[k][0], chans[k][1][[i]], chans[k][2][[i]],
                                                   chans[k][3][[i]], cs, ms) for k, i in picks])
        assert np.array_equal(status, want)
        assert errors == int((want == 1).sum()) and errors > 0
        # publish (CALCULATE) through the mapping: same bytes as the oracle's publisher
        expect = [c[0].copy() for c in chans]
        sub = picks[:700]
        for k, i in sub:
            oracle.publish_slots(expect[k], chans[k][1][[i]], chans[k][2][[i]], chans[k][3][[i]], cs, ms)
        gpu_ctx.crc32_host_slot_list(rec[:700], max_message_size=slot_size, checksum_size=cs, metadata_size=ms,
                                     mode=gpu.SLOT_CALCULATE)
        for k in range(2):
            assert np.array_equal(chans[k][0], expect[k]), k
    finally:
        for host, *_ in chans:
            gpu.host_unregister(host)


def test_host_slot_list_unregistered_rejected(gpu_ctx):
    host = np.zeros(8192, dtype=np.uint8)
    rec = slots.slot_records([host.ctypes.data], [host.ctypes.data + 64], [100])
    with pytest.raises(gpu.CrcError):
        gpu_ctx.crc32_host_slot_list(rec, max_message_size=4096, mode=gpu.SLOT_VERIFY)


def test_drain_helper_cpp(gpu_ctx):
    """include/subspace/checksum_batch.h from C++ (tools/drain_demo): a 64-slot memfd channel
    published in one BatchChecksum::Calculate, every slot verified by the drop-in header's
    VerifyCRC32Checksum<3> on the host; a shuffled 48-slot drain with corrupted payload and
    prefix bytes, a cleared checksum flag and truncated delivered sizes verified in one call:
    per-slot results, mismatch count and checksum_error flags equal the host templates';
    after UnregisterBuffer the drain is rejected."""
    import json
    import subprocess
    from pathlib import Path
    exe = Path(__file__).resolve().parent.parent / "tools" / "drain_demo"
    assert exe.exists(), "build tools/drain_demo first (make)"
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["device"] and d["failures"] == 0
    assert d["mismatches"] == d["expected_mismatches"] >= 3 and d["unchecked"] >= 1
    assert d["unregistered_rejected"]


def _corrupt(host, po, ps, cs, sizes, seed):
    """Corruptions of test_verify_statuses (payload bit, span 0, stored checksum, uncovered
    padding, flag cleared) on a published channel; returns the kinds applied per slot."""
    rng = np.random.default_rng(seed)
    kinds = rng.integers(0, 8, len(po))
    for i, k in enumerate(kinds):
        b, n = int(po[i]), int(sizes[i])
        if k == 1 and n:
            host[b + ps + rng.integers(0, n)] ^= np.uint8(1 << rng.integers(0, 8))
        elif k == 3:
            host[b + 4 + rng.integers(0, 44)] ^= 0x01
        elif k == 4:
            host[b + 48 + rng.integers(0, 4)] ^= 0x80
        elif k == 5:
            host[b:b + 4] ^= 0xFF
            host[b + 48 + cs:b + ps] ^= 0xAA
        elif k == 6:
            host[b + 32] &= 0xFB
    return kinds


@pytest.mark.parametrize("count", [1, 2, 3, 63, 4097, 65537, 140001, 300001])
@pytest.mark.parametrize("cs", [4, 20])
def test_fused_slot_kernel_publish_and_verify(gpu_ctx, oracle, count, cs):
    """The fused slot kernel (contiguous 4 KiB slots, metadata_size 0: payload CRC, span-0
    term and flag/checksum store or status in one pass; crc_uniform.hip SLOT): publish is
    byte-identical to the oracle's publisher restatement; verify statuses and the mismatch
    count equal the oracle's subscriber restatement after corruptions. Counts cover waves
    without tiles, odd last tiles, partial and several 32-tile windows per wave."""
    ms = 0
    sizes = np.full(count, 4096, dtype=np.uint64)
    host, ps, stride = build_channel(count, 4096, cs, ms, sizes, seed=count + cs)
    dev, status = publish_strided(gpu_ctx, host, stride, count, cs, ms, message_size=4096)
    po, yo = offsets(count, stride, ps)
    oracle.publish_slots(host, po, yo, sizes, cs, ms)
    assert (status == 0).all()
    got = dev.cpu().numpy()
    bad = np.nonzero(got != host)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
    _corrupt(host, po, ps, cs, sizes, seed=count * 3 + cs)
    want = oracle.verify_slots(host, po, yo, sizes, cs, ms)
    dev = torch.from_numpy(host).to(DEV)
    st = torch.full((count,), 7, dtype=torch.int32, device=DEV)
    err = torch.full((1,), 12345, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_slots_strided(dev, stride, count, message_size=4096, checksum_size=cs, metadata_size=ms,
                                mode=gpu.SLOT_VERIFY, status=st, error_count=err)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy().view(np.uint32), want)
    assert int(err.item()) == int((want == 1).sum())
    assert np.array_equal(dev.cpu().numpy(), host)  # verify never writes the channel
    # the error count of the next call starts from zero again (no status array this time)
    err2 = torch.full((1,), 999, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_slots_strided(dev, stride, count, message_size=4096, checksum_size=cs, metadata_size=ms,
                                mode=gpu.SLOT_VERIFY, error_count=err2)
    torch.cuda.synchronize()
    assert int(err2.item()) == int((want == 1).sum())


@pytest.mark.parametrize("slot_size,cs", [(4200, 4), (8192, 4), (8192, 20)])
def test_fused_slot_kernel_wider_slots(gpu_ctx, oracle, slot_size, cs):
    """4 KiB messages in slots larger than the message (stride 4,288 / 8,256 / 8,320): the
    fused kernel reads each payload and prefix at the slot stride and never touches the
    slot bytes past the message; publish byte-identical to the oracle, verify statuses equal
    the oracle's after corruptions."""
    count, ms = 5003, 0
    sizes = np.full(count, 4096, dtype=np.uint64)
    host, ps, stride = build_channel(count, slot_size, cs, ms, sizes, seed=slot_size + cs)
    dev, status = publish_strided(gpu_ctx, host, stride, count, cs, ms, message_size=4096)
    po, yo = offsets(count, stride, ps)
    oracle.publish_slots(host, po, yo, sizes, cs, ms)
    assert (status == 0).all()
    got = dev.cpu().numpy()
    bad = np.nonzero(got != host)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]}"
    _corrupt(host, po, ps, cs, sizes, seed=slot_size * 7 + cs)
    want = oracle.verify_slots(host, po, yo, sizes, cs, ms)
    dev = torch.from_numpy(host).to(DEV)
    st = torch.full((count,), 7, dtype=torch.int32, device=DEV)
    err = torch.full((1,), 12345, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_slots_strided(dev, stride, count, message_size=4096, checksum_size=cs, metadata_size=ms,
                                mode=gpu.SLOT_VERIFY, status=st, error_count=err)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy().view(np.uint32), want)
    assert int(err.item()) == int((want == 1).sum())
    assert np.array_equal(dev.cpu().numpy(), host)


@pytest.mark.parametrize("cs,ms,off", [(4, 0, 0), (4, 0, 64), (4, 0, 192), (20, 0, 64), (4, 16, 64), (4, 16, 0),
                                        (5, 7, 64), (6, 64, 64)])
def test_fused_slot_kernel_line_offsets(gpu_ctx, oracle, cs, ms, off):
    """The fused slot kernel with the channel at a 128-B line offset `off`: the even or the
    odd slots' payloads (or both) start 64 B into a line; publish is byte-identical to the
    oracle, nothing outside the channel is written, and verify statuses equal the oracle's
    after corruptions, for prefix sizes 64 and 128 (with metadata)."""
    count = 4097
    sizes = np.full(count, 4096, dtype=np.uint64)
    host, ps, stride = build_channel(count, 4096, cs, ms, sizes, seed=off + 31 * cs + ms)
    full = torch.zeros(len(host) + 256, dtype=torch.uint8, device=DEV)
    assert full.data_ptr() % 256 == 0
    full[off:off + len(host)] = torch.from_numpy(host).to(DEV)
    status = torch.full((count,), 7, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_slots_strided(full, stride, count, message_size=4096, checksum_size=cs, metadata_size=ms,
                                mode=gpu.SLOT_CALCULATE, status=status, base_offset=off)
    torch.cuda.synchronize()
    po, yo = offsets(count, stride, ps)
    oracle.publish_slots(host, po, yo, sizes, cs, ms)
    assert (status.cpu().numpy() == 0).all()
    got = full.cpu().numpy()
    assert not got[:off].any() and not got[off + len(host):].any()  # nothing outside the channel
    bad = np.nonzero(got[off:off + len(host)] != host)[0]
    assert len(bad) == 0, f"{len(bad)} bytes differ, first at {bad[:8]} (stride {stride}, offset {off})"
    _corrupt(host, po, ps, cs, sizes, seed=off * 5 + cs + ms)
    want = oracle.verify_slots(host, po, yo, sizes, cs, ms)
    full[off:off + len(host)] = torch.from_numpy(host).to(DEV)
    err = torch.full((1,), 12345, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_slots_strided(full, stride, count, message_size=4096, checksum_size=cs, metadata_size=ms,
                                mode=gpu.SLOT_VERIFY, status=status, error_count=err, base_offset=off)
    torch.cuda.synchronize()
    assert np.array_equal(status.cpu().numpy().view(np.uint32), want)
    assert int(err.item()) == int((want == 1).sum())


def test_fused_and_two_kernel_slot_paths_agree(gpu_ctx):
    """fused_slots off (payload kernel + crc32_slot_finish_kernel) and on give the same
    channel bytes and statuses."""
    from subspace_amd import _lib
    lib = _lib.load()
    count, cs, ms = 20001, 4, 0
    sizes = np.full(count, 4096, dtype=np.uint64)
    host, ps, stride = build_channel(count, 4096, cs, ms, sizes, seed=4242)
    out = []
    for fused in (0, 1):
        assert _lib.load_dev().subspace_crc_testutil_set(gpu_ctx._h, b"fused_slots", fused) == 0
        try:
            dev, status = publish_strided(gpu_ctx, host.copy(), stride, count, cs, ms, message_size=4096)
            out.append((dev.cpu().numpy(), status))
        finally:
            _lib.load_dev().subspace_crc_testutil_set(gpu_ctx._h, b"fused_slots", 1)
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])


def test_fused_slot_verify_graph_replay(gpu_ctx):
    """The fused verify (with its self-resetting mismatch counter) captured in a hipGraph:
    every replay reports the same mismatch count."""
    count, cs, ms = 5000, 4, 0
    sizes = np.full(count, 4096, dtype=np.uint64)
    host, ps, stride = build_channel(count, 4096, cs, ms, sizes, seed=31)
    dev = torch.from_numpy(host).to(DEV)
    gpu_ctx.crc32_slots_strided(dev, stride, count, message_size=4096, mode=gpu.SLOT_CALCULATE)
    torch.cuda.synchronize()
    for i in (5, 777, 4999):
        dev[i * stride + ps + 100] ^= 1
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            gpu_ctx.crc32_slots_strided(dev, stride, count, message_size=4096, mode=gpu.SLOT_VERIFY, error_count=err)
    torch.cuda.synchronize()
    for _ in range(3):
        err.fill_(-1)
        g.replay()
        torch.cuda.synchronize()
        assert int(err.item()) == 3


@pytest.mark.parametrize("fused", [1, 0])
def test_calculate_zeroes_error_count(gpu_ctx, fused):
    """A publish (CALCULATE) has no mismatches: the error count it is given reads 0 afterwards,
    through the fused slot kernel and the two-kernel path alike (include/subspace_crc.h:
    'set to the number of SUBSPACE_CRC_SLOT_MISMATCH slots of this call')."""
    from subspace_amd import _lib
    lib = _lib.load()
    count, cs, ms = 3001, 4, 0
    sizes = np.full(count, 4096, dtype=np.uint64)
    host, ps, stride = build_channel(count, 4096, cs, ms, sizes, seed=606)
    dev = torch.from_numpy(host).to(DEV)
    err = torch.full((1,), 777, dtype=torch.int32, device=DEV)
    assert _lib.load_dev().subspace_crc_testutil_set(gpu_ctx._h, b"fused_slots", fused) == 0
    try:
        gpu_ctx.crc32_slots_strided(dev, stride, count, message_size=4096, mode=gpu.SLOT_CALCULATE, error_count=err)
        torch.cuda.synchronize()
    finally:
        _lib.load_dev().subspace_crc_testutil_set(gpu_ctx._h, b"fused_slots", 1)
    assert int(err.item()) == 0


@pytest.mark.parametrize("cs,ms", [(4, 16), (5, 7), (6, 64), (4, 65)])
def test_verify_metadata_channels(gpu_ctx, oracle, cs, ms):
    """Verify statuses and the mismatch count of channels with user metadata equal the oracle's
    after corruptions (metadata bytes included), fused (ms <= 64) and two-kernel (65) alike."""
    count = 3001
    sizes = np.full(count, 4096, dtype=np.uint64)
    host, ps, stride = build_channel(count, 4096, cs, ms, sizes, seed=cs * 1000 + ms)
    po, yo = offsets(count, stride, ps)
    oracle.publish_slots(host, po, yo, sizes, cs, ms)
    rng = np.random.default_rng(ms)
    for i in rng.choice(count, 40, replace=False):  # metadata, span 0 and payload bytes
        k = int(rng.integers(0, 3))
        at = [48 + cs + int(rng.integers(0, ms)), 4 + int(rng.integers(0, 44)), ps + int(rng.integers(0, 4096))][k]
        host[int(po[i]) + at] ^= 0x10
    want = oracle.verify_slots(host, po, yo, sizes, cs, ms)
    dev = torch.from_numpy(host).to(DEV)
    st = torch.full((count,), 7, dtype=torch.int32, device=DEV)
    err = torch.full((1,), 12345, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_slots_strided(dev, stride, count, message_size=4096, checksum_size=cs, metadata_size=ms,
                                mode=gpu.SLOT_VERIFY, status=st, error_count=err)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy().view(np.uint32), want)
    assert int(err.item()) == int((want == 1).sum()) > 0


@pytest.mark.parametrize("slot_size,cs,ms", [(1000, 4, 0), (4000, 8, 5), (1000, 4, 100), (5000, 20, 32)])
def test_strided_oversize_sizes_are_flagged(gpu_ctx, oracle, slot_size, cs, ms):
    """a per-slot size beyond the slot's payload area would run into the next slot,
    whose prefix a publish rewrites in the same (fused) launch. Such slots get
    SUBSPACE_CRC_SLOT_OVERSIZE and are left untouched, on every path: the fused small-slot
    kernel (1000 / 4000-B slots), small + finish kernels (metadata > 64 B), ragged + finish
    (5000-B slots); every other slot is published and verified as the oracle's. ADVICE r04: no
    payload kernel reads an oversize slot's bytes -- the last slot's size (2^40) points far past
    the end of the buffer, and the middle slot's (2^33) past it too."""
    count = 900
    rng = np.random.default_rng(slot_size + ms)
    area = (slot_size + 63) & ~63
    sizes = rng.integers(0, area + 1, count).astype(np.uint64)
    big = rng.random(count) < 0.1
    sizes[big] = rng.integers(area + 1, area + 3000, int(big.sum()))
    big[[count // 2, count - 1]] = True
    sizes[count // 2], sizes[count - 1] = 1 << 33, 1 << 40
    host, ps, stride = build_channel(count, slot_size, cs, ms, sizes, seed=slot_size + cs + ms)
    assert stride - ps == area
    orig = host.copy()
    dev, status = publish_strided(gpu_ctx, host, stride, count, cs, ms, sizes=sizes)
    assert np.array_equal(status == gpu.SLOT_OVERSIZE, big)
    assert (status[~big] == 0).all()
    po, yo = offsets(count, stride, ps)
    oracle.publish_slots(host, po[~big], yo[~big], sizes[~big], cs, ms)
    got = dev.cpu().numpy()
    assert np.array_equal(got, host)
    for i in np.nonzero(big)[0]:  # oversize slots: prefix untouched
        assert np.array_equal(got[i * stride:i * stride + ps], orig[i * stride:i * stride + ps])
    st = torch.full((count,), 7, dtype=torch.int32, device=DEV)
    err = torch.full((1,), 123, dtype=torch.int32, device=DEV)
    d_sizes = torch.from_numpy(sizes.view(np.int64)).to(DEV)
    gpu_ctx.crc32_slots_strided(dev, stride, count, sizes=d_sizes, checksum_size=cs, metadata_size=ms,
                                mode=gpu.SLOT_VERIFY, status=st, error_count=err)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    assert np.array_equal(st == gpu.SLOT_OVERSIZE, big) and (st[~big] == 0).all() and int(err.item()) == 0


@pytest.mark.parametrize("mode", ["publish", "verify"])
def test_large_slot_list_latency_channel_shape(gpu_ctx, oracle, mode):
    """S_large's shape at a reduced count: the reference's checksum latency
    channel (client/latency_test.cc:731-745) -- 32 KiB slots, payloads of rand() % 32,767 + 1
    bytes -- as a shuffled device slot list with max_message_size 32,768 (the ragged pipeline at
    absolute addresses + the slot finish), publish byte-identical to oracle.publish_slots and
    verify after bit flips equal to oracle.verify_slots."""
    count, area, cs, ms = 1500, 32768, 4, 0
    rng = np.random.default_rng(0x5A1A + (mode == "verify"))
    sizes = rng.integers(1, area, count).astype(np.uint64)
    sizes[:4] = [1, 8191, 8192, 32767]
    host, ps, stride = build_channel(count, area, cs, ms, sizes, seed=0x5A1B)
    po, yo = offsets(count, stride, ps)
    if mode == "verify":
        oracle.publish_slots(host, po, yo, sizes, cs, ms)
        for i in rng.choice(count, count // 3, replace=False):
            host[int(yo[i]) + int(rng.integers(0, int(sizes[i])))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    dev = torch.from_numpy(host).to(DEV)
    order = rng.permutation(count)
    base = np.uint64(dev.data_ptr())
    rec = slots.slot_records(base + po[order], base + yo[order], sizes[order])
    d_rec = torch.from_numpy(rec.view(np.int64)).to(DEV)
    status = torch.full((count,), 7, dtype=torch.int32, device=DEV)
    err = torch.full((1,), 12345, dtype=torch.int32, device=DEV)
    gmode = gpu.SLOT_CALCULATE if mode == "publish" else gpu.SLOT_VERIFY
    gpu_ctx.crc32_slots(d_rec, max_message_size=area, checksum_size=cs, metadata_size=ms, mode=gmode, status=status,
                        error_count=err if mode == "verify" else None)
    torch.cuda.synchronize()
    got = status.cpu().numpy().view(np.uint32)
    if mode == "publish":
        oracle.publish_slots(host, po, yo, sizes, cs, ms)
        assert (got == 0).all()
        assert np.array_equal(dev.cpu().numpy(), host)
    else:
        want = oracle.verify_slots(host, po[order], yo[order], sizes[order], cs, ms)
        assert np.array_equal(got, want)
        assert int(err.item()) == int((want == 1).sum()) > 0


@pytest.mark.parametrize("mode", ["publish", "verify"])
def test_large_slot_list_statuses(gpu_ctx, oracle, mode):
    """Slot lists past 4 KiB (the ragged path at absolute addresses, finished by its last
    kernel: crc_slots.hip crc32_ragged_final_slot_kernel) with a metadata span, empty payloads
    and records longer than max_message_size (a list's records carry their sizes: computed
    whole, as on the small-kernel path), and for verify every status the oracle gives:
    mismatches in the payload, metadata, span 0 and stored checksum, uncovered bytes changed,
    and slots without kMessageHasChecksum."""
    count, area, max_len, cs, ms = 1200, 32768, 20000, 4, 16
    rng = np.random.default_rng(0x5A2A + (mode == "verify"))
    sizes = rng.integers(0, max_len + 1, count).astype(np.uint64)
    sizes[rng.choice(count, 40, replace=False)] = rng.integers(max_len + 1, area + 1, 40).astype(np.uint64)
    sizes[:6] = [0, 1, 8192, max_len, max_len + 1, area]
    host, ps, stride = build_channel(count, area, cs, ms, sizes, seed=0x5A2B)
    po, yo = offsets(count, stride, ps)
    kinds = rng.integers(0, 8, count)
    if mode == "verify":
        oracle.publish_slots(host, po, yo, sizes, cs, ms)
        for i, k in enumerate(kinds):
            b, n = int(po[i]), int(sizes[i])
            if k == 1 and n:
                host[b + ps + rng.integers(0, n)] ^= np.uint8(1 << rng.integers(0, 8))
            elif k == 2:
                host[b + 48 + cs + rng.integers(0, ms)] ^= 0x10
            elif k == 3:
                host[b + 4 + rng.integers(0, 44)] ^= 0x01
            elif k == 4:
                host[b + 48 + rng.integers(0, 4)] ^= 0x80
            elif k == 5:
                host[b:b + 4] ^= 0xFF
            elif k == 6:
                host[b + 32] &= 0xFB
    before = host.copy()
    dev = torch.from_numpy(host).to(DEV)
    order = rng.permutation(count)
    base = np.uint64(dev.data_ptr())
    rec = slots.slot_records(base + po[order], base + yo[order], sizes[order])
    d_rec = torch.from_numpy(rec.view(np.int64)).to(DEV)
    status = torch.full((count,), 7, dtype=torch.int32, device=DEV)
    err = torch.full((1,), 12345, dtype=torch.int32, device=DEV)
    gmode = gpu.SLOT_CALCULATE if mode == "publish" else gpu.SLOT_VERIFY
    gpu_ctx.crc32_slots(d_rec, max_message_size=max_len, checksum_size=cs, metadata_size=ms, mode=gmode,
                        status=status, error_count=err)
    torch.cuda.synchronize()
    got = status.cpu().numpy().view(np.uint32)
    if mode == "publish":
        assert (got == 0).all() and int(err.item()) == 0
        oracle.publish_slots(before, po, yo, sizes, cs, ms)
        assert np.array_equal(dev.cpu().numpy(), before)
    else:
        want = oracle.verify_slots(host, po[order], yo[order], sizes[order], cs, ms)
        assert set(np.unique(want)) == {0, 1, 2}
        assert np.array_equal(got, want)
        assert int(err.item()) == int((want == 1).sum())
        assert np.array_equal(dev.cpu().numpy(), before)  # verify never writes the channel
