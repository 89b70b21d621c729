"""CPU models of the kernels' load addresses and tile indexing (subspace_amd/csrc/
crc_ragged.hip make_desc + load_line, crc_uniform.hip load_tile, and the sweep
front mapping): every byte any load can read lies inside the caller's messages, every
message byte is read, every tile is visited exactly once. Runs without a GPU."""
import collections
import itertools

import numpy as np
import pytest

M32 = 1 << 32


def tiles_for_length(n):
    return (n + 8191) >> 13


def ragged_loads(s, e):
    """For message [s, e): (tile j, lane, block, address or None) for every load of
    load_line. Tiles cover the extended message [s0, e), s0 = s rounded down to 16 B: tile
    j starts at ts = s0 + 8192j and holds min(8192, e - ts) bytes; loads are buffer loads
    against the range [ts, tile end rounded up to 16 B), and an offset >= the range size
    reads zeros without a memory access (None). Lane l loads the 8 blocks at 128*l + 16*b."""
    s0 = s & ~15
    nt = tiles_for_length(e - s0)
    for j in range(nt):
        ts = s0 + (j << 13)
        nrec = (min(8192, e - ts) + 15) & ~15
        for lane in range(64):
            for b in range(8):
                off = lane * 128 + 16 * b
                yield j, lane, b, (ts + off if off < nrec else None)


def ragged_line_window(s, e, j, lane):
    """The 8 blocks process() reads for (tile j, lane) -- as addresses (None = zeros)."""
    return [addr for jj, ln, b, addr in ragged_loads(s, e) if jj == j and ln == lane]


@pytest.mark.parametrize("seed", range(6))
def test_every_ragged_load_stays_in_its_message_blocks(seed):
    rng = np.random.default_rng(seed)
    for _ in range(200):
        s = int(rng.integers(0, 5000))
        n = int(rng.choice([rng.integers(1, 300), rng.integers(1, 40000),
                            8192 * int(rng.integers(1, 4)) + int(rng.integers(-20, 20))]))
        n = max(n, 1)
        e = s + n
        for j, lane, b, addr in ragged_loads(s, e):
            if addr is None:
                continue
            # a 16-B block that holds at least one message byte
            assert addr + 16 > s and addr < e, (s, e, j, lane, b, addr)


@pytest.mark.parametrize("s,n", [(0, 1), (3, 100), (17, 8192), (5, 8193), (0, 4096), (1, 65536 + 7), (15, 24577),
                                 (64, 16384 + 9), (7, 8192 * 3)])
def test_ragged_line_windows_hold_each_line(s, n):
    """Every lane's 128-B line [ts + 128l, +128) is its 8 consecutive aligned blocks, and
    every message byte of the line comes from a real load."""
    e = s + n
    s0 = s & ~15
    nt = tiles_for_length(e - s0)
    for j in range(nt):
        ts = s0 + (j << 13)
        for lane in range(64):
            win = ragged_line_window(s, e, j, lane)
            base = ts + 128 * lane
            for b, addr in enumerate(win):
                if addr is not None:
                    assert addr == base + 16 * b, (s, n, j, lane, b)
            for x in range(base, base + 128):
                if s <= x < e:
                    assert win[(x - base) // 16] is not None, (s, n, j, lane, x)


def test_ragged_loads_cover_every_message_byte():
    for s, n in [(0, 1), (3, 100), (17, 8192), (5, 8193), (0, 4096), (1, 65536 + 7), (15, 24577)]:
        e = s + n
        covered = set()
        for j, lane, b, addr in ragged_loads(s, e):
            if addr is not None:
                covered.update(range(max(addr, s), min(addr + 16, e)))
        assert covered == set(range(s, e))


def wave_descriptor_indices(total, nblocks, waves_per_block):
    """Replays crc32_ragged_kernel's descriptor indexing (fetch_desc) for every wave:
    prologue fetches k = 0, 1; loop fetches k + 2 and k + 3 per pair of tiles."""
    nw = nblocks * waves_per_block
    for w in range(nw):
        nk = (total - w + nw - 1) // nw if w < total else 0

        def tau(k):
            return (min(k, nk - 1) * nw + w) if nk else total - 1

        idx = [tau(0), tau(1)]
        k = 0
        while k < nk:
            idx.append(tau(k + 2))
            if k + 1 >= nk:
                break
            idx.append(tau(k + 3))
            k += 2
        yield w, nk, idx


@pytest.mark.parametrize("total", [1, 2, 7, 100, 2047, 2048, 2049, 5000, 100003])
def test_every_descriptor_index_is_a_real_tile(total):
    for w, nk, idx in wave_descriptor_indices(total, 256, 8):
        assert all(0 <= t < total for t in idx), (w, nk, idx[:6])


def test_tiles_are_covered_exactly_once():
    total, nw = 5003, 256 * 8
    seen = []
    for w in range(nw):
        nk = (total - w + nw - 1) // nw if w < total else 0
        seen += [k * nw + w for k in range(nk)]
    assert sorted(seen) == list(range(total))


@pytest.mark.parametrize("count,stride", [(1, 4096), (2, 4096), (3, 4160), (1000, 4096), (4097, 8192),
                                          (20001, 4096)])
@pytest.mark.parametrize("depth", [1, 2])
def test_uniform_kernel_loads_stay_in_messages(count, stride, depth):
    """Replays crc32_uniform4k_kernel's load_tile ranges (order 0, 256 x 8 waves): every
    in-range load lies inside message 2*tau + h, and every message of every tile is read."""
    ntiles = (count + 1) // 2
    nblocks, wpb = 256, 8
    nw = nblocks * wpb
    read = set()
    for b in range(nblocks):
        for wid in range(wpb):
            t0 = front_slot(b, nblocks, wid)
            nk = (ntiles - t0 + nw - 1) // nw if t0 < ntiles else 0
            # loads issued: prologue tiles 0..depth-1, then k+depth for every processed tile k
            ks = list(range(depth)) + [k + depth for k in range(nk)]
            for k in ks:
                live = k < nk
                m0 = 2 * (t0 + k * nw)
                nrec = 0 if not live else (stride + 4096 if m0 + 1 != count else 4096)
                for h in (0, 1):
                    for l in range(32):
                        for i in range(8):
                            off = h * stride + l * 128 + 16 * i
                            if off >= nrec:
                                continue
                            msg = m0 + h
                            assert msg < count and off - h * stride + 16 <= 4096
                            read.add(msg)
    assert read == set(range(count))


def front_slot(b, G, wid):
    """crc_device.h front_slot: consecutive pairs of sweep-front slots go to consecutive
    workgroups (round-robin over XCDs)."""
    return (b + G * (wid >> 1)) * 2 + (wid & 1)


@pytest.mark.parametrize("wg", [256, 512, 768, 1024])
@pytest.mark.parametrize("grid", [1, 2, 3, 255, 256])
def test_front_slot_is_a_bijection(wg, grid):
    wpb = wg // 64
    slots = [front_slot(b, grid, wid) for b in range(grid) for wid in range(wpb)]
    assert sorted(slots) == list(range(grid * wpb))


def test_front_slot_tiles_covered_exactly_once():
    grid, wpb, total = 256, 8, 70001
    nw = grid * wpb
    seen = []
    for b in range(grid):
        for wid in range(wpb):
            w = front_slot(b, grid, wid)
            nk = (total - w + nw - 1) // nw if w < total else 0
            seen += [k * nw + w for k in range(nk)]
    assert sorted(seen) == list(range(total))


def xcd_group_slot(b, G, wid, wpb):
    """crc_uniform.hip order 3: aligned groups of 16 front slots on one XCD (b % 8), groups
    rotating over the XCDs; only for 8 | G and 16 | (G/8)*wpb (else the kernel uses order 0)."""
    x, local = b & 7, (b >> 3) * wpb + wid
    return ((local >> 4) * 8 + x) * 16 + (local & 15)


@pytest.mark.parametrize("wg", [256, 512, 768, 1024])
@pytest.mark.parametrize("grid", [8, 16, 64, 128, 256])
def test_xcd_group_slot_is_a_bijection(wg, grid):
    wpb = wg // 64
    if ((grid // 8) * wpb) % 16:
        pytest.skip("the kernel falls back to order 0 for this grid")
    slots = [xcd_group_slot(b, grid, wid, wpb) for b in range(grid) for wid in range(wpb)]
    assert sorted(slots) == list(range(grid * wpb))
    # every group of 16 consecutive slots (one 128-B line of results) is on one XCD
    xcd = {xcd_group_slot(b, grid, wid, wpb): b & 7 for b in range(grid) for wid in range(wpb)}
    for g in range(grid * wpb // 16):
        assert len({xcd[16 * g + i] for i in range(16)}) == 1


def desc_kernel_stores(ntiles, capacity, lane_tiles=2, rows=1):
    """Replays crc32_ragged_desc_kernel (crc_ragged.hip, message-centric): thread m stores
    tiles tile_base[m] + j of its message for j < min(nt, kLaneTiles); then per wave, for each
    wave, the later tiles of its 64 messages in the load-balanced expansion below. Nothing is
    stored when the batch has more tiles than the capacity. Returns ({tile: (message, j)} with every store counted, tile_base)."""
    count = len(ntiles)
    tb = np.concatenate([[0], np.cumsum(ntiles, dtype=np.int64)])
    total = int(tb[count])
    stores = collections.Counter()
    owner = {}
    if total > capacity:
        return owner, stores, tb
    for w0 in range(0, count, 64):
        ms = range(w0, min(w0 + 64, count))
        for m in ms:
            for j in range(min(int(ntiles[m]), lane_tiles)):
                owner[int(tb[m]) + j] = (m, j)
                stores[int(tb[m]) + j] += 1
        # SUBSPACE_DESC_EXPAND: later tiles numbered q in message order (exclusive scan of
        # b = nt - kLaneTiles), round r of row y stores q = 64 (y + r rows) + lane, its message by a
        # 6-step binary search over the 64 scan values (lanes past the wave's messages: b = 0)
        b = [max(int(ntiles[m]) - lane_tiles, 0) for m in ms] + [0] * (64 - len(ms))
        ex = list(itertools.accumulate([0] + b[:-1]))
        W = ex[63] + b[63]
        # one row: messages starting in the round mark their first position, a max-scan over
        # the lanes carries the marks on from the previous round's last message
        long_lanes = [i for i in range(64) if b[i]]
        for y in range(rows):
            carry = long_lanes[0] + 1 if long_lanes else 0
            for q0 in range(64 * y, W, 64 * rows):
                if rows == 1:
                    marks = [0] * 64
                    for i in long_lanes:
                        if q0 <= ex[i] < q0 + 64:
                            marks[ex[i] - q0] = i + 1
                    owners = [max(carry, *marks[:lane + 1]) - 1 for lane in range(64)]
                    carry = owners[63] + 1
                for lane in range(64):
                    q = q0 + lane
                    if rows == 1:
                        o = owners[lane]
                    else:
                        o = 0
                        for st in (32, 16, 8, 4, 2, 1):
                            if ex[o + st] <= q:
                                o += st
                    if q < W:
                        m, j = w0 + o, lane_tiles + q - ex[o]
                        owner[int(tb[m]) + j] = (m, j)
                        stores[int(tb[m]) + j] += 1
    return owner, stores, tb


def descw_stores(ntiles, capacity, lane_tiles=8):
    """Replays crc_desc.h descw_wave (the wide fused tile-count scan + descriptor kernel,
    crc_combine.hip crc32_ragged_count_desc16_kernel: absolute-address batches): each lane stores
    its message's first kLaneTilesW tiles, then every message with more, one after the other, 64
    tiles per round (tile j = kLaneTilesW + lane + 64 r); no tile at or past the capacity."""
    count = len(ntiles)
    tb = np.concatenate([[0], np.cumsum(ntiles, dtype=np.int64)])
    stores = collections.Counter()
    owner = {}
    for w0 in range(0, count, 64):
        for m in range(w0, min(w0 + 64, count)):
            nt = int(ntiles[m])
            js = list(range(min(nt, lane_tiles)))
            if nt > lane_tiles:  # the wave's long messages, in lane order
                for r0 in range(lane_tiles, nt, 64):
                    js += [j for j in range(r0, min(r0 + 64, nt))]
            for j in js:
                if int(tb[m]) + j < capacity:
                    owner[int(tb[m]) + j] = (m, j)
                    stores[int(tb[m]) + j] += 1
    return owner, stores, tb


@pytest.mark.parametrize("seed", range(4))
def test_wide_fused_desc_stores_every_tile_once(seed):
    rng = np.random.default_rng(100 + seed)
    parts = []
    for _ in range(40):
        parts.append(np.zeros(int(rng.integers(0, 50)), dtype=np.int64))
        parts.append(rng.integers(1, 6, int(rng.integers(1, 200))))       # S_large: 1 .. 5 tiles
        parts.append(rng.integers(6, 200, int(rng.integers(0, 3))))       # longer messages
    ntiles = np.concatenate(parts).astype(np.int64)
    total = int(ntiles.sum())
    for capacity in (total, total + 1000, total - 7):
        owner, stores, tb = descw_stores(ntiles, capacity)
        assert sorted(owner) == list(range(min(total, capacity)))
        assert set(stores.values()) == {1}
        for tau, (m, j) in owner.items():
            assert tb[m] <= tau < tb[m + 1] and tau == tb[m] + j


@pytest.mark.parametrize("seed,rows", [(s, 1) for s in range(6)] + [(6, 3), (7, 64)])
def test_desc_kernel_stores_every_tile_once(seed, rows):
    rng = np.random.default_rng(seed)
    parts = []
    for _ in range(40):
        parts.append(np.zeros(int(rng.integers(0, 150)), dtype=np.int64))  # zero-tile runs
        parts.append(rng.integers(1, 3, int(rng.integers(1, 100))))        # one/two-tile messages
        parts.append(rng.integers(3, 300, int(rng.integers(0, 3))))        # multi-tile messages
    ntiles = np.concatenate(parts).astype(np.int64)
    total = int(ntiles.sum())
    for capacity in (total, total + 1000, total - 1):
        owner, stores, tb = desc_kernel_stores(ntiles, capacity, rows=rows)
        if capacity < total:
            assert not owner  # the search path: no descriptors
            continue
        assert sorted(owner) == list(range(total))
        assert set(stores.values()) == {1}
        for tau, (m, j) in owner.items():
            assert tb[m] <= tau < tb[m + 1] and tau == tb[m] + j


# ------------------------------------------------------------------ fused slot kernel
def slot_grid(count, num_cus=256):
    """capi.hip slots_strided_impl: 8-wave workgroups, one per CU up to the tile count, and
    more workgroups when a wave would get more than kSlotRingRounds (32) tiles."""
    tiles = (count + 1) // 2
    return max(max(1, min(num_cus, (tiles + 7) // 8)), (tiles + 8 * 32 - 1) // (8 * 32))


def slot_kernel_accesses(count, stride, prefix_size, num_cus=256, cs=4, ms=0):
    """Every access of crc32_uniform4k_kernel<512, true, false> (crc_uniform.hip, SLOT) as
    byte offsets from the first prefix (the channel buffer): payload tile loads (16 B each),
    the finishing waves' prefix loads (16 B each, both rounds, issued unconditionally), their
    flag/checksum stores (prefix words 8 and 12) and the LDS ring entries they read. Returns
    (loads, stores_by_message, ring_reads, max tiles per wave). With metadata (ms > 0) the
    finishing waves also read span 1 as dwords: the one holding byte 48 + cs and the next
    (sh + ms + 3) / 4 - 1, each index clamped to the last (18 loads, crc_uniform.hip)."""
    G = slot_grid(count, num_cus)
    ntiles = (count + 1) // 2
    nw = 8 * G
    lane = np.arange(64)
    loads, stores, ring = [], {}, []
    max_nk = 0
    nk_of = lambda t0: (ntiles - t0 + nw - 1) // nw if t0 < ntiles else 0  # noqa: E731
    for b in range(G):
        for wid in range(8):
            t0 = front_slot(b, G, wid)
            nk = nk_of(t0)
            max_nk = max(max_nk, nk)
            for k in range(nk + 1):  # the prologue's tile 0 and every prefetch, clamped
                kk = k if k < nk else (nk - 1 if nk else 0)
                for h in (0, 1):
                    msg = 2 * (t0 + kk * nw) + h if nk else 0
                    msg = msg if msg < count else msg - 1
                    base = prefix_size + msg * stride
                    loads.append(base + (lane[:32, None] * 128 + 16 * np.arange(8)[None, :]).ravel())
            if wid >= 4:
                continue
            fw, fh = (lane >> 1) & 7, lane & 1
            ft0 = np.array([front_slot(b, G, int(w)) for w in fw])
            fnk = np.array([nk_of(int(t)) for t in ft0])
            nk0 = nk_of(front_slot(b, G, 0))
            for r in (0, 1):
                ftile = 16 * r + 4 * wid + (lane >> 4)
                fmsg = 2 * (ft0 + ftile * nw) + fh
                valid = (ftile < fnk) & (fmsg < count)
                m = np.where(valid, fmsg, 0)
                loads.append((m * stride)[:, None] + 16 * np.arange(4)[None, :])  # prefix line, 4 x 16 B
                if ms and 16 * r < nk0:
                    o1 = 48 + cs
                    nwords = ((o1 & 3) + ms + 3) >> 2
                    j = np.minimum(np.arange(18), nwords - 1)
                    span1 = (m * stride)[:, None] + (o1 & ~3) + 4 * j[None, :]
                    assert (span1 % 4 == 0).all()
                    # dword loads: 4 B each, model them as 16-B-aligned blocks for the range check
                    loads.append(span1 & ~15)
                if 16 * r >= nk0:
                    continue
                ring.append(fw * 512 + 16 * ftile + 8 * fh)
                for msg in fmsg[valid]:
                    stores[int(msg)] = stores.get(int(msg), 0) + 1
    return np.concatenate([x.ravel() for x in loads]), stores, np.concatenate(ring) if ring else np.zeros(0), max_nk


@pytest.mark.parametrize("count,stride,prefix,cs,ms", [
    (1, 4160, 64, 4, 0), (2, 4160, 64, 4, 0), (3, 4160, 64, 4, 0), (63, 4160, 64, 4, 0), (4097, 4160, 64, 4, 0),
    (65536, 4160, 64, 4, 0), (65537, 4160, 64, 4, 0), (140001, 4160, 64, 4, 0), (300001, 4160, 64, 4, 0),
    (5003, 8256, 64, 4, 0), (5003, 8320, 128, 20, 0), (3001, 4224, 128, 4, 16), (3001, 4160, 64, 5, 7),
    (3001, 4224, 128, 6, 64), (3001, 4224, 128, 7, 61), (1, 4224, 128, 4, 16)])
def test_slot_kernel_accesses_stay_in_the_channel(count, stride, prefix, cs, ms):
    """Every vector load of the fused slot kernel is 16-B aligned (the buffer and stride are)
    and lies inside the channel buffer [0, count * stride); every slot's flag and checksum are
    stored exactly once, by one finishing wave; no wave has more tiles than its ring holds, and
    every ring entry read lies in the 4 KiB ring area. (the product kernel
    issues no load outside the buffer and no b128 load at a 4-B-aligned address.)"""
    assert prefix == ((48 + cs + ms + 63) & ~63)  # ComputePrefixSize
    loads, stores, ring, max_nk = slot_kernel_accesses(count, stride, prefix, cs=cs, ms=ms)
    assert (loads % 16 == 0).all()
    assert loads.min() >= 0 and loads.max() + 16 <= count * stride
    assert sorted(stores) == list(range(count)) and set(stores.values()) == {1}
    assert max_nk <= 32
    assert ring.size == 0 or (ring.min() >= 0 and ring.max() + 8 <= 8 * 512)


def test_r02s3i_prefix_variant_was_in_bounds():
    """The round-2 variant that faulted (r02s3i: three dwordx4 prefix loads per window at
    prefix + 4, + 20, + 36) read inside each slot: its addresses were in bounds, so the fault
    was not an out-of-range address -- the property it alone had is the 4-B-aligned b128 load
    (DESIGN.md 4.8). Every product b128 load is 16-B aligned (test above)."""
    stride, prefix = 4160, 64
    for msg in (0, 1, 65535):
        addrs = [msg * stride + off for off in (4, 20, 36)]
        assert all(a % 16 == 4 for a in addrs)
        assert all(msg * stride <= a and a + 16 <= msg * stride + prefix for a in addrs)


# ------------------------------------------------------------------ small-message kernel
def small_kernel_loads(starts, lengths, G, lanes=32):
    """Replays crc32_small_kernel<512, SLOT, false, lanes>'s general loop (crc_small.hip): per wave
    (order-0 front, G workgroups x 8 waves) the tiles whose lines it loads -- the prologue's tile
    0, then tiles k+1 and k+2 per loop pair, clamped records past the wave's last tile -- and per
    message (M = 64 / lanes per tile, C = 128 lanes bytes) the 16-B blocks of load_lines: line li
    of message mj loads s0 + min(128 li + 16 b, last block) for E = L + (s & 15) in [1, C] and
    L > 0, else the step table's block (None here; longer messages take long_crc). Yields
    (message or None, block address or None); returns nothing else."""
    count = len(starts)
    M, C = 64 // lanes, 128 * lanes
    ntiles = (count + M - 1) // M
    nw = 8 * G
    for b in range(G):
        for wid in range(8):
            t0 = front_slot(b, G, wid)
            nk = (ntiles - t0 + nw - 1) // nw if t0 < ntiles else 0
            ks = [0]
            k = 0
            while k + 1 < nk:
                ks += [k + 1, k + 2]
                k += 2
            for k in ks:
                for mj in range(M):
                    m = M * (t0 + k * nw) + mj
                    present = k < nk and m < count
                    kk = k if k < nk else max(nk - 1, 0)
                    mr = min(M * (t0 + kk * nw) + mj if nk else 0, count - 1)  # the record read
                    s, L = int(starts[mr]), int(lengths[mr])
                    E = L + (s & 15)
                    if not (present and L and E <= C):
                        yield None, None
                        continue
                    assert mr == m
                    lastb = (E - 1) & ~15
                    for li in range(lanes):
                        for blk in range(8):
                            yield m, (s & ~15) + min(128 * li + 16 * blk, lastb)


@pytest.mark.parametrize("seed,count,G,lanes", [(0, 1, 1, 32), (1, 2, 1, 32), (2, 3, 1, 32), (3, 999, 63, 32),
                                                (4, 5001, 256, 32), (5, 30001, 256, 32), (6, 1, 1, 1),
                                                (7, 67, 1, 1), (8, 999, 3, 2), (9, 4097, 256, 4),
                                                (10, 3001, 7, 8), (11, 2049, 256, 16)])
def test_small_kernel_loads_stay_in_messages(seed, count, G, lanes):
    """Every line load of the small-message kernel's tile loop is a 16-B-aligned block holding at
    least one byte of its own message (no load outside the caller's messages; messages at any
    offset & 15, empty ones, and ones over C, which read only the step table), and every byte of
    every message it computes is loaded -- for G = 32 lanes per message and the packed forms
    (lanes = 1 .. 16: M = 64 / lanes messages per tile, each over lanes 128-B lines)."""
    rng = np.random.default_rng(seed)
    C = 128 * lanes
    lengths = rng.integers(0, C + 1, count)
    lengths[rng.random(count) < 0.05] = rng.integers(C + 1, 2 * C + 900)
    starts = np.cumsum(np.concatenate([[0], lengths[:-1] + rng.integers(0, 40, count - 1)])) + 7
    covered = {}
    for m, addr in small_kernel_loads(starts, lengths, G, lanes):
        if m is None:
            continue
        s, e = int(starts[m]), int(starts[m] + lengths[m])
        assert addr % 16 == 0 and addr + 16 > s and addr < e, (m, s, e, addr)
        if count <= 5001:
            covered.setdefault(m, set()).update(range(max(addr, s), min(addr + 16, e)))
    if count <= 5001:
        for m in range(count):
            s, L = int(starts[m]), int(lengths[m])
            if L and L + (s & 15) <= C:
                assert covered.get(m) == set(range(s, s + L)), m


def small_kernel_repack_loads(starts, lengths, G):
    """Replays crc32_small_kernel<512, false, false, 32>'s REPACK loop (crc_small.hip; the slot
    instantiation packs per workgroup instead: small_kernel_repack2 below): a wave with
    at most 32 tiles that is not FAST packs its window's entries (entry e = the record lane e
    loaded: message 2 (t0 + (e / 2) nw) + e % 2) by size: an entry of E = L + (s & 15) in
    [1, 4096] has class c (2^c lanes, the least with 128 2^c >= E); empty, absent and longer
    entries get no lanes. Uniform layout (one class with the placed entries first, or sorting
    saves too little): entry e at lanes e 2^cmax ..; sorted layout: the entries by class, largest
    first, each class's in lane order. Packed tile j's lane i (position P = 64 j + i) loads line
    P - (its group's first position) of its entry, clamped like load_lines; positions past the
    layout (the loop's tile rnt among them) read the step table. Yields (message or None, block
    address or None) for the packing waves, ('msg', m) for each message they compute with lanes,
    then ('waves', number of them)."""
    count = len(starts)
    ntiles = (count + 1) // 2
    nw = 8 * G
    waves = 0
    for b in range(G):
        for wid in range(8):
            t0 = front_slot(b, G, wid)
            nk = (ntiles - t0 + nw - 1) // nw if t0 < ntiles else 0
            if nk == 0 or nk > 32:
                continue
            ent = [2 * (t0 + (e // 2) * nw) + e % 2 for e in range(64)]
            ent = [m if e < 2 * nk and m < count else None for e, m in enumerate(ent)]
            if all(m is None or (int(lengths[m]) == 4096 and int(starts[m]) % 16 == 0) for m in ent):
                continue  # FAST
            waves += 1
            cls = []
            for m in ent:
                E = int(lengths[m]) + (int(starts[m]) & 15) if m is not None else 0
                if m is None or lengths[m] == 0 or E > 4096:
                    cls.append(-1)
                else:
                    cls.append(max(0, (((E + 127) >> 7) - 1).bit_length()))
            placed = [e for e in range(64) if cls[e] >= 0]
            for e in placed:
                yield "msg", ent[e]
            if not placed:
                continue
            cmax = max(cls[e] for e in placed)
            lanes = sum(1 << cls[e] for e in placed)
            nu = (placed[-1] + 1) << cmax
            tu, ts = (nu + 63) >> 6, (lanes + 63) >> 6
            prefix_one = placed == list(range(len(placed))) and len({cls[e] for e in placed}) == 1
            owner = {}  # position -> (entry, line in its group)
            if prefix_one or not (ts < tu and (tu >= 4 or ts + 2 <= tu)):
                for e in placed:
                    for li in range(1 << cmax):
                        owner[(e << cmax) + li] = (e, li)
                total = nu if not prefix_one else len(placed) << cmax
            else:
                pos = 0
                for c in range(5, -1, -1):
                    for e in placed:
                        if cls[e] == c:
                            assert pos % (1 << c) == 0 and pos // 64 == (pos + (1 << c) - 1) // 64
                            for li in range(1 << c):
                                owner[pos + li] = (e, li)
                            pos += 1 << c
                total = pos
            rnt = (total + 63) >> 6
            for j in list(range(rnt)) + [rnt]:
                for i in range(64):
                    if (64 * j + i) not in owner:
                        yield None, None
                        continue
                    e, li = owner[64 * j + i]
                    m = ent[e]
                    s = int(starts[m])
                    lastb = (int(lengths[m]) + (s & 15) - 1) & ~15
                    for blk in range(8):
                        yield m, (s & ~15) + min(128 * li + 16 * blk, lastb)
    yield "waves", waves


@pytest.mark.parametrize("seed,count,G,top", [(20, 1, 1, 64), (21, 65, 1, 300), (22, 999, 63, 2048),
                                              (23, 4001, 31, 1000), (24, 20001, 256, 129), (25, 3001, 7, 4096),
                                              (26, 999, 5, 5000), (27, 2001, 40, 256)])
def test_small_kernel_repack_loads_stay_in_messages(seed, count, G, top):
    """REPACK's loads obey the same rule as the tile loop's: every block holds a byte of its own
    message and every byte of every message it computes with lanes is loaded, in the uniform and
    the sorted layout (messages up to `top` bytes: past 4 KiB they take no lanes)."""
    rng = np.random.default_rng(seed)
    lengths = rng.integers(0, top + 1, count)
    starts = np.cumsum(np.concatenate([[0], lengths[:-1] + rng.integers(0, 40, count - 1)])) + 3
    starts = starts - (starts & 15) * (rng.random(count) < 0.5)  # some 16-B aligned
    covered, waves, want = {}, 0, set()
    for m, addr in small_kernel_repack_loads(starts, lengths, G):
        if m == "waves":
            waves = addr
            continue
        if m == "msg":
            want.add(addr)
            continue
        if m is None:
            continue
        s, e = int(starts[m]), int(starts[m] + lengths[m])
        assert addr % 16 == 0 and addr + 16 > s and addr < e, (m, s, e, addr)
        covered.setdefault(m, set()).update(range(max(addr, s), min(addr + 16, e)))
    assert waves > 0 and set(covered) == want
    for m, byts in covered.items():
        assert byts == set(range(int(starts[m]), int(starts[m] + lengths[m]))), m


def small_kernel_repack2(starts, lengths, grid, rng):
    """Replays the slot kernel's REPACK2 (crc32_small_kernel<512, true, false, 32>, crc_small.hip):
    per workgroup, lane i < 32 of wave w holds message i of its window (entry q = 32 w + i,
    message 2 (t0 + (i / 2) nw) + i % 2); an entry of E = L + (s & 15) in [1, 4096] has n = ceil(E /
    128) lines, laid out back to back in lane order (r2x: the wave's lines before it). The wave's
    first Q lines are its local tiles (Q: the workgroup's least wave's lines rounded down to whole
    tiles, at least 64, or its largest wave's rounded up when that is at most 64 more): lane P of local tile j takes the entry of rank k - 1, k = the entries with
    lines starting before the tile + popcount(the tile's start marks & (2 << P) - 1), or line / n
    when the wave's entries are lanes 0, 1, ... with one line count; ranks map to lanes as the
    kernel's ds_permute does; when Q = 64 in a workgroup with FAST waves, a wave's lines 64 ..
    127, loaded on speculation before Q is known, are loads only. The other lines of every wave form the shared stream (wave after
    wave); entries with shared lines are
    ranked r = 0, 1, ... in the same order (record at r, ring entry in the offset's top byte,
    first shared position and first line), the shared tiles' start marks S_j and first entries
    (by rank) built as the kernel builds them, and shared tile j's lane i finds its entry as r =
    first_j + popcount(S_j & (2 << i) - 1) - (S_j & 1). Each line gets a random value; every tile's
    inclusive XOR scan and the scan value before the entry's first lane in the tile give the part
    its last lane XORs into the entry's ring word. Yields ('load', message, block address) for
    every load, ('line', (workgroup, q), li) for every line computed, ('ring', q, got, want) per
    entry with lines, and ('wgs', repacking workgroups) at the end."""
    count = len(starts)
    ntiles = (count + 1) // 2
    nw = 8 * grid
    assert ntiles <= 16 * nw
    wgs = 0
    for b in range(grid):
        waves = []  # per wave: [(q, message or None, E, n)] for lanes 0..31
        fast_all = True
        fast_w = []  # per wave: FAST (every live entry a whole aligned 4 KiB payload)
        for wid in range(8):
            t0 = front_slot(b, grid, wid)
            nk = (ntiles - t0 + nw - 1) // nw if t0 < ntiles else 0
            ents = []
            fw = True
            for i in range(32):
                m = 2 * (t0 + (i // 2) * nw) + i % 2
                live = i // 2 < nk and m < count
                E = int(lengths[m]) + (int(starts[m]) & 15) if live else 0
                ok = live and int(lengths[m]) != 0 and E <= 4096
                if live and not (int(lengths[m]) == 4096 and int(starts[m]) % 16 == 0):
                    fast_all = False
                    fw = False
                ents.append((32 * wid + i, m if live else None, E if ok else 0, (E + 127) >> 7 if ok else 0))
            fast_w.append(fw)
            waves.append(ents)
        if fast_all:
            continue
        wgs += 1
        vals, ring = {}, {}
        for ents in waves:
            for q, m, E, n in ents:
                ring[q] = 0
                for li in range(n):
                    vals[(q, li)] = int(rng.integers(0, 1 << 32))
        tiles = []  # (lane -> (q, m, E, n, li, first lane of the entry's part in the tile)) per tile

        def emit(lanes):
            tiles.append(lanes)
        # local tiles: every wave's first Q lines, Q = the least wave's lines rounded down to whole
        # tiles, at least 64; the counts of entries with lines past 64 (i + 1) checked against Q's
        tots = [sum(n for *_, n in ents) for ents in waves]
        tmin = min(tots)
        Q = tmin & ~63 if tmin >= 128 else 64
        tm = (max(tots) + 63) & ~63
        if tm <= Q + 64:  # at most one tile beyond Q: no shared stream
            Q = max(tm, 64)
        shared = []  # (q, m, E, n, first shared line) in stream order
        spec = []  # (message, block) loads of a speculative local tile 1 the workgroup dropped
        for ents in waves:
            r2x = [int(x) for x in np.concatenate([[0], np.cumsum([n for *_, n in ents])])[:-1]]
            tot = sum(n for *_, n in ents)
            nloc = min(tot, Q)
            withl = [i for i in range(32) if ents[i][3]]  # rank -> lane
            nset = {ents[i][3] for i in withl}
            runi = withl == list(range(len(withl))) and len(nset) <= 1
            for j in range((nloc + 63) // 64):
                lanes = {}
                for lane in range(64):
                    P = 64 * j + lane
                    if P >= nloc:
                        continue
                    if runi:
                        k = P // ents[0][3] + 1
                    else:
                        base = sum(1 for i in withl if r2x[i] < 64 * j)
                        k = base + sum(1 for i in withl if 64 * j <= r2x[i] <= P)
                    i = withl[k - 1]
                    q, m, E, n = ents[i]
                    lanes[lane] = (q, m, E, n, P - r2x[i], max(r2x[i] - 64 * j, 0))
                emit(lanes)
            if Q < 128 and any(fast_w) and tot > 64:
                # local tile 1 loaded on speculation (lines 64 .. min(tot, 128)) before Q is known
                # (a workgroup with FAST waves), then dropped
                for P in range(64, min(tot, 128)):
                    if runi:
                        k = P // ents[0][3] + 1
                    else:
                        k = sum(1 for i in withl if r2x[i] <= P)
                    i = withl[k - 1]
                    q, m, E, n = ents[i]
                    li = P - r2x[i]
                    assert 0 <= li < n
                    for blk in range(8):
                        spec.append((m, (int(starts[m]) & ~15) + min(128 * li + 16 * blk, (E - 1) & ~15)))
            cnt = sum(1 for i in range(32) if ents[i][3] and r2x[i] + ents[i][3] > Q)
            got = 0
            for i in range(32):
                q, m, E, n = ents[i]
                if n and r2x[i] + n > Q:
                    a0 = max(r2x[i], Q)
                    shared.append((q, m, E, n, a0 - r2x[i], r2x[i] + n - a0))
                    got += 1
            assert got == cnt
        # shared stream
        start = [int(x) for x in np.concatenate([[0], np.cumsum([c for *_, c in shared])])[:-1]]
        T = sum(c for *_, c in shared)
        ntl = (T + 63) >> 6
        S = [0] * max(ntl, 1)
        first = [None] * max(ntl, 1)
        for r, ((q, m, E, n, li0, c), st) in enumerate(zip(shared, start)):
            S[st >> 6] |= 1 << (st & 63)
            jb = (st + 63) >> 6
            if 64 * jb < st + c:
                assert first[jb] is None
                first[jb] = r
        for j in range(ntl):
            lanes = {}
            for i in range(64):
                P = 64 * j + i
                if P >= T:
                    continue
                r = first[j] + bin(S[j] & ((2 << i) - 1)).count("1") - (S[j] & 1)
                q, m, E, n, li0, c = shared[min(r, len(shared) - 1)]
                st = start[r]
                lanes[i] = (q, m, E, n, P - st + li0, st - 64 * j if st > 64 * j else 0)
            emit(lanes)
        for lanes in tiles:
            scan, acc = [], 0
            for i in range(64):
                if i in lanes:
                    q, m, E, n, li, mst = lanes[i]
                    assert 0 <= li < n, (q, li, n)
                    yield "line", (b, q), li
                    s0 = int(starts[m])
                    lastb = (E - 1) & ~15
                    for blk in range(8):
                        yield "load", m, (s0 & ~15) + min(128 * li + 16 * blk, lastb)
                    acc ^= vals[(q, li)]
                scan.append(acc)
            for i, (q, m, E, n, li, mst) in lanes.items():
                if li == n - 1 or i == 63:
                    ring[q] ^= scan[i] ^ (scan[mst - 1] if mst else 0)
        for m, addr in spec:
            yield "load", m, addr
        for ents in waves:
            for q, m, E, n in ents:
                if n:
                    want = 0
                    for li in range(n):
                        want ^= vals[(q, li)]
                    yield "ring", q, ring[q], want
    yield "wgs", wgs, None


@pytest.mark.parametrize("seed,count,grid,top", [(40, 1, 1, 64), (41, 511, 2, 4096), (42, 4096, 16, 4096),
                                                 (43, 4095, 16, 300), (44, 2000, 8, 5000), (45, 999, 4, 4096)])
def test_small_kernel_repack2_packs_every_line_once(seed, count, grid, top):
    """REPACK2: every line of every message with lines is computed exactly once, every load
    holds a byte of its own message and every byte is loaded, and the parts XORed into each
    entry's ring word (messages straddling packed tiles included) make the XOR of all its lines."""
    rng = np.random.default_rng(seed)
    lengths = rng.integers(0, top + 1, count)
    lengths[: min(count, 3)] = [4096, 1, 129][: min(count, 3)]
    starts = np.cumsum(np.concatenate([[0], lengths[:-1] + rng.integers(0, 40, count - 1)])) + 3
    starts = starts - (starts & 15) * (rng.random(count) < 0.5)
    lines, covered, want_cov = {}, {}, {}
    wgs = 0
    for kind, a, b, *rest in small_kernel_repack2(starts, lengths, grid, rng):
        if kind == "wgs":
            wgs = a
        elif kind == "line":
            lines[(a, b)] = lines.get((a, b), 0) + 1
        elif kind == "load":
            s, e = int(starts[a]), int(starts[a] + lengths[a])
            assert b % 16 == 0 and b + 16 > s and b < e, (a, s, e, b)
            covered.setdefault(a, set()).update(range(max(b, s), min(b + 16, e)))
        elif kind == "ring":
            assert b == rest[0], (a, b, rest[0])
    assert wgs > 0 and all(v == 1 for v in lines.values())
    for m, cov in covered.items():
        assert cov == set(range(int(starts[m]), int(starts[m] + lengths[m]))), m


@pytest.mark.parametrize("seed,count,grid,top", [(50, 4096, 16, 200), (51, 4096, 16, 4096), (52, 2048, 8, 600)])
def test_small_kernel_repack2_with_fast_waves(seed, count, grid, top):
    """REPACK2 in workgroups where waves 0 and 4 are FAST (every message a whole aligned 4 KiB
    payload) and the others are not: the FAST waves' bookkeeping comes after the prologue barrier,
    so the others' local tile 1 is loaded on speculation before Q is known (dropped when Q = 64).
    Same properties as test_small_kernel_repack2_packs_every_line_once."""
    rng = np.random.default_rng(seed)
    nw = 8 * grid
    fastm = np.zeros(count, dtype=bool)
    for m in range(count):
        t0 = (m // 2) % nw
        wid = 2 * ((t0 >> 1) // grid) + (t0 & 1)
        fastm[m] = wid % 4 == 0
    lengths = np.where(fastm, 4096, rng.integers(0, top + 1, count))
    starts, cur = [], 3
    for m in range(count):
        if fastm[m]:
            cur = (cur + 15) & ~15
        starts.append(cur)
        cur += int(lengths[m]) + int(rng.integers(0, 40))
    starts = np.array(starts, dtype=np.int64)
    lines, covered = {}, {}
    wgs = 0
    for kind, a, b, *rest in small_kernel_repack2(starts, lengths, grid, rng):
        if kind == "wgs":
            wgs = a
        elif kind == "line":
            lines[(a, b)] = lines.get((a, b), 0) + 1
        elif kind == "load":
            s, e = int(starts[a]), int(starts[a] + lengths[a])
            assert b % 16 == 0 and b + 16 > s and b < e, (a, s, e, b)
            covered.setdefault(a, set()).update(range(max(b, s), min(b + 16, e)))
        elif kind == "ring":
            assert b == rest[0], (a, b, rest[0])
    assert wgs > 0 and all(v == 1 for v in lines.values())
    for m, cov in covered.items():
        assert cov == set(range(int(starts[m]), int(starts[m] + lengths[m]))), m


def uniform_fast_reads(count, L, stride, G, grid):
    """Replays crc_small.hip's UNIFORM FAST loads (a uniform batch of L-byte messages, G lanes
    per message, C = 128 G >= L, + 15 when the stride is not 16-B aligned): for every tile the
    kernel loads, the byte ranges its lanes read -- [s0, s0 + C) from the 16-B block holding the
    message's first byte, s0 = (m * stride) & ~15, for the tile's messages when the tile's last
    message is at most usafe (u_safe), else the clamped blocks of the extended message [s0, m *
    stride + L)."""
    M, C = 64 // G, 128 * G
    upad = C - min(L, C)
    usafe = count - 1 if upad == 0 else (-1 if stride == 0 else count - 1 - -(-upad // stride))
    ntiles = -(-count // M)
    nw = 8 * grid
    for b in range(grid):
        for wid in range(8):
            t0 = front_slot(b, grid, wid)
            nk = (ntiles - t0 + nw - 1) // nw if t0 < ntiles else 0
            for k in range(nk + 2):  # (the loop loads up to two tiles past the last: clamped)
                kk = k if k < nk else max(nk - 1, 0)
                if not nk:
                    continue
                last = M * (t0 + kk * nw) + M - 1
                for j in range(M):
                    m = min(M * (t0 + kk * nw) + j, count - 1)
                    s0 = (m * stride) & ~15
                    if last <= usafe:
                        yield s0, s0 + C
                    else:
                        lastb = (L + (m * stride & 15) - 1) & ~15
                        for li in range(G):
                            for blk in range(8):
                                o = s0 + min(128 * li + 16 * blk, lastb)
                                yield o, o + 16


@pytest.mark.parametrize("count,L,stride,G,grid", [(1000, 1000, 1008, 8, 4), (5000, 16, 16, 1, 8), (301, 129, 144, 2, 3),
                                                   (70, 100, 112, 1, 2), (4097, 2000, 2000, 16, 16),
                                                   (63, 512, 512, 4, 1), (2, 17, 32, 1, 1),
                                                   (3001, 3000, 3008, 32, 12), (65, 4000, 4000, 32, 1),
                                                   (2, 2100, 2112, 32, 1), (3000, 200, 200, 2, 4),
                                                   (2000, 1000, 1000, 8, 8), (3001, 1500, 1500, 16, 8),
                                                   (999, 3000, 3000, 32, 16), (77, 100, 100, 1, 2),
                                                   (5, 4081, 4081, 32, 1), (1000, 17, 17, 1, 3)])
def test_uniform_fast_reads_stay_in_the_batch(count, L, stride, G, grid):
    """The packed uniform FAST loop reads past a message's L bytes (into the next messages) but
    never past the batch: every range it reads lies in [0, end) with end the batch's last byte
    rounded up to its 16-B block (the clamped loads' rule: whole 16-B blocks holding message
    bytes), and the unclamped C-byte reads end within the batch itself -- for 16-B strides and
    packed ones (round 6)."""
    end = (count - 1) * stride + L
    end16 = (end + 15) & ~15
    for lo, hi in uniform_fast_reads(count, L, stride, G, grid):
        assert 0 <= lo and hi <= (end if hi - lo == 128 * G else end16), (lo, hi, end)


def fast_line_blocks(s, l):
    """The FAST loop's 8 loads of lane l (one address, immediate offsets 0..112)."""
    return [s + 128 * l + 16 * b for b in range(8)]


@pytest.mark.parametrize("s", [0, 16, 64, 4160 * 7 + 64, (1 << 40) + 4096])
def test_fast_loads_equal_the_general_loads(s):
    """For a message the FAST path accepts (4,096 bytes on a 16-B boundary) its one-address,
    immediate-offset loads are exactly the general loop's clamped blocks s0 + min(128 l + 16 b,
    last block): the same bytes, every one inside the message."""
    L = 4096
    E = L + (s & 15)
    lastb = (E - 1) & ~15
    for l in range(32):
        general = [(s & ~15) + min(128 * l + 16 * b, lastb) for b in range(8)]
        assert fast_line_blocks(s, l) == general
        assert all(s <= a and a + 16 <= s + L for a in general)



# ------------------------------------------------------------------ zero-copy host slot lists
def small_grid(count, num_cus=256):
    """capi.hip small_run: one workgroup per CU, or more so no wave gets more than 32 tiles."""
    tiles = (count + 1) // 2
    return max(min(num_cus, max(1, -(-tiles // 8))), -(-tiles // (8 * 32)))


def small_slot_accesses(recs, cs, ms, num_cus=256):
    """Replays every global access of crc32_small_kernel<512, true> (crc_small.hip) for slot
    records (prefix, payload, size): the line loads of half-tile messages, the whole-wave chunk
    loads of messages longer than a half-tile (long_crc), the finish's prefix loads (7 x 8 B,
    then the metadata words), and a publish's two 4-B stores. Yields (slot, kind, address,
    width); record and table reads (device memory) are left out."""
    count = len(recs)
    G = small_grid(count, num_cus)
    ntiles, nw = (count + 1) // 2, 8 * G
    for b in range(G):
        for wid in range(8):
            t0 = front_slot(b, G, wid)
            nk = (ntiles - t0 + nw - 1) // nw if t0 < ntiles else 0
            assert nk <= 32
            for k in range(nk):
                for h in (0, 1):
                    m = 2 * (t0 + k * nw) + h
                    if m >= count:
                        continue
                    pre, s, L = recs[m]
                    E = L + (s & 15)
                    s0 = s & ~15
                    if L and E <= 4096:  # load_lines
                        lastb = (E - 1) & ~15
                        for lane in range(32):
                            for blk in range(8):
                                yield m, "line", s0 + min(128 * lane + 16 * blk, lastb), 16
                    elif E > 4096:  # long_crc: 8 KiB chunks, all 64 lanes
                        for j in range((E + 8191) >> 13):
                            ln = min(8192, E - (j << 13))
                            lastb = (ln - 1) & ~15
                            for lane in range(64):
                                for blk in range(8):
                                    yield m, "chunk", s0 + (j << 13) + min(128 * lane + 16 * blk, lastb), 16
                    for i in range(7):  # span_crc: prefix words 0..13
                        yield m, "prefix", pre + 8 * i, 8
                    if ms:
                        o1 = 48 + cs
                        sh = o1 & 3
                        for j in range((sh + ms + 3) >> 2):
                            yield m, "meta", pre + (o1 & ~3) + 4 * j, 4
                    yield m, "store", pre + 32, 4  # flags word (SetHasChecksum)
                    yield m, "store", pre + 48, 4  # checksum


@pytest.mark.parametrize("seed,count,cs,ms", [(0, 1, 4, 0), (1, 37, 4, 0), (2, 999, 4, 16), (3, 2001, 20, 33),
                                              (4, 5000, 64, 64)])
def test_host_slot_list_accesses_stay_in_registered_regions(seed, count, cs, ms):
    """VERDICT r03 item 6 (the r02s3i question): the zero-copy drain (subspace_crc32_host_slot_list
    -> subspace_crc32_slots -> crc32_small_kernel) reads and writes host memory through the
    device aliases of regions registered with subspace_crc_host_register. capi.hip admits a
    record only if [prefix, prefix + prefix_size) and [payload, payload + size) each lie inside
    one registered region; then every access the kernel makes is width-aligned (16-B line and
    chunk loads on 16-B boundaries, 8-B prefix loads, 4-B metadata words and stores -- no b128
    load at a 4-B-aligned address, the one property only the faulting r02s3i variant had) and
    stays inside the 16-B blocks that hold the record's own bytes, hence inside the pinned
    pages of its region, for payloads at every offset & 15 (a region's first byte included)
    and for sizes beyond max_message_size (whole-wave chunks)."""
    rng = np.random.default_rng(seed)
    ps = ((48 + cs + ms) + 63) & ~63
    page = 4096
    # payload regions at arbitrary byte offsets (a payload may start at a region's first byte),
    # prefixes in one 8-B aligned region, as the ABI requires
    regions, recs, owner = [], [], []
    pre_base = 7 * page + 8 * int(rng.integers(0, 32))
    regions.append((pre_base, count * ps))
    cursor = 1 << 30
    for i in range(count):
        L = int(rng.choice([rng.integers(0, 4097), 4096, rng.integers(4097, 20000)], p=[0.8, 0.15, 0.05]))
        mis = int(rng.integers(0, 16))
        start = cursor + mis
        if rng.random() < 0.3:  # the payload is its region's first byte
            regions.append((start, max(L, 1)))
            owner.append(len(regions) - 1)
        else:
            owner.append(None)
        recs.append((pre_base + i * ps, start, L))
        cursor = ((start + L + 4095) // 4096 + 1) * 4096 + int(rng.integers(0, 64))
    big = (1 << 30, cursor - (1 << 30))  # one region holding every other payload
    regions.append(big)
    order = rng.permutation(count)
    recs = [recs[i] for i in order]
    owner = [owner[i] for i in order]

    def pages(reg):
        a, n = reg
        return a - a % page, -(-(a + n) // page) * page

    for m, kind, addr, w in small_slot_accesses(recs, cs, ms):
        assert addr % w == 0, (kind, addr, w)
        pre, s, L = recs[m]
        if kind in ("line", "chunk"):
            assert addr + w > s and addr < s + L, (kind, m, addr)  # a block holding payload bytes
            reg = regions[owner[m]] if owner[m] is not None else big
        else:
            assert pre <= addr and addr + w <= pre + ps, (kind, m, addr)
            reg = regions[0]
        lo, hi = pages(reg)
        assert lo <= addr and addr + w <= hi, (kind, m, addr, reg)


# ------------------------------------------------------------------ 8-B tile descriptors
# crc_device.h kDesc8* / kD8*: tile starts < 2^37, after < 2^25
START_BITS, AFTER_BITS = 37, 25
HI_START = START_BITS - 36
MIS_SHIFT, FIRST_BIT, X_SHIFT = HI_START, 1 << (HI_START + 4), HI_START + 5
K_FIRST, K_LAST8 = 0x80000000, 1 << AFTER_BITS


def pack_desc8(tile_start, after, first, length, mis):
    """crc_ragged.hip pack_desc8 (TileDesc -> TileDesc8), restated."""
    s16 = tile_start >> 4
    x = (K_LAST8 | length) if (after == 0 or length == 0) else after
    hi = ((s16 >> 32) & ((1 << HI_START) - 1)) | (mis << MIS_SHIFT) | (FIRST_BIT if first else 0) | (x << X_SHIFT)
    return s16 & 0xFFFFFFFF, hi & 0xFFFFFFFF


def unpack_desc8(lo, hi):
    """crc_ragged.hip unpack_desc8, restated: (tile_start, after | first flag, len | mis << 16)."""
    tile_start = ((hi & ((1 << HI_START) - 1)) << 36) | (lo << 4)
    x = hi >> X_SHIFT
    last = (x & K_LAST8) != 0
    after = (0 if last else x) | (K_FIRST if hi & FIRST_BIT else 0)
    length = ((x & 0x3FFF) if last else 8192) | (((hi >> MIS_SHIFT) & 15) << 16)
    return tile_start, after, length


def wide_message(s, length):
    """crc32_ragged_count_scan_kernel's flag: a tile of message (s, length) beyond the 8-B form."""
    nt = (length + (s & 15) + 8191) >> 13 if length else 0
    return nt > 0 and ((((s & ~15) + ((nt - 1) << 13)) >> START_BITS) != 0 or ((nt - 1) >> AFTER_BITS) != 0)


def descs_of(s, length):
    """make_desc for every tile of one message: (tile_start, after, first, bytes, mis)."""
    mis = s & 15
    nt = (length + mis + 8191) >> 13
    for j in range(nt):
        rest = length + mis - (j << 13)
        yield (s & ~15) + (j << 13), nt - 1 - j, j == 0, min(rest, 8192), mis


@pytest.mark.parametrize("s,length", [(0, 1), (15, 1), (3, 8189), (3, 8190), (0, 8192), (1, 8192), (7, 3 * 8192 + 5),
                                      ((1 << 37) - 8192 - 16, 8192), ((1 << 37) - 8192 - 16 + 9, 8183),
                                      ((1 << 36) + 17, 5 << 13), (4096, (1 << 25) << 13), (0, (1 << 25) << 13)])
def test_desc8_round_trip_or_flagged(s, length):
    """Every tile of a message that the count scan does not flag round-trips through the 8-B
    form exactly; a flagged message is one whose tiles would not."""
    if wide_message(s, length):
        nt = (length + (s & 15) + 8191) >> 13
        last_start = (s & ~15) + ((nt - 1) << 13)
        assert last_start >= 1 << START_BITS or nt - 1 >= 1 << AFTER_BITS
        return
    n = 0
    for tile_start, after, first, nbytes, mis in descs_of(s, length):
        lo, hi = pack_desc8(tile_start, after, first, nbytes, mis)
        want = (tile_start, after | (K_FIRST if first else 0), nbytes | (mis << 16))
        assert unpack_desc8(lo, hi) == want
        n += 1
        if n > 64:  # long messages: the first 64 tiles and the last one
            mis = s & 15
            nt = (length + mis + 8191) >> 13
            last = ((s & ~15) + ((nt - 1) << 13), 0, nt == 1, length + mis - ((nt - 1) << 13), mis)
            assert unpack_desc8(*pack_desc8(*last)) == (last[0], last[1] | (K_FIRST if last[2] else 0),
                                                          last[3] | (last[4] << 16))
            break


def test_desc8_flag_edges():
    # the last tile start 2^37 - 16 fits; 2^37 does not
    assert not wide_message((1 << 37) - 16, 1)
    assert wide_message(1 << 37, 1)
    assert wide_message((1 << 37) - 8192, 8193)  # second tile starts at 2^37
    # 2^25 tiles: after up to 2^25 - 1 fits (a message of 2^25 tiles starting at 0 ends at 2^38:
    # its last tile start is past 2^37, so that one is flagged by the start)
    assert wide_message(0, (1 << 25) << 13)
    assert not wide_message(0, (1 << 24) << 13)
    assert wide_message(0, ((1 << 25) << 13) + 1)
    assert not wide_message(0, 0)


def desc8_incremental(so, length, j):
    """crc32_ragged_desc_kernel's later tiles (j >= kLaneTiles), built from the message's first."""
    mis = so & 15
    nt = (length + mis + 8191) >> 13
    last = nt - 1
    last_len = length + mis - (last << 13)
    t16 = (so >> 4) + (j << 9)
    x = (K_LAST8 | last_len) if j == last else last - j
    return t16 & 0xFFFFFFFF, ((t16 >> 32) & ((1 << HI_START) - 1)) | (mis << MIS_SHIFT) | (x << X_SHIFT)


@pytest.mark.parametrize("so,length", [(0, 3 * 8192), (5, 3 * 8192), (4095, 100000), ((1 << 37) - (40 << 13) + 3, 30 << 13),
                                       ((1 << 36) - 8192 * 2 - 1, 9 * 8192 + 1), (1 << 32, (1 << 20) + 7)])
def test_desc8_incremental_matches_pack(so, length):
    assert not wide_message(so, length)
    tiles = list(descs_of(so, length))
    for j in range(2, len(tiles)):
        assert desc8_incremental(so, length, j) == pack_desc8(*tiles[j]), j


def call_mismatch_count(G, counts, order):
    """Replays crc_device.h add_call_mismatches: workgroups in `order` add their counts to group
    word b % 8; a group's last adds the group total to the top word and resets its word; the last
    group writes the call's total and resets the top. Returns (writes of the total, words left)."""
    words = [0] * 9
    writes = []
    for b in order:
        g = b % 8
        ng = (G - g + 7) // 8
        old = words[1 + g]
        words[1 + g] += (1 << 32) | counts[b]
        if old >> 32 == ng - 1:
            tot = (old + counts[b]) & 0xFFFFFFFF
            words[1 + g] = 0
            o2 = words[0]
            words[0] += (1 << 32) | tot
            if o2 >> 32 == min(G, 8) - 1:
                writes.append((o2 + tot) & 0xFFFFFFFF)
                words[0] = 0
    return writes, words


@pytest.mark.parametrize("G", [1, 2, 7, 8, 9, 17, 256, 257, 1000])
def test_call_mismatch_count_is_written_once_and_resets(G):
    """The slot kernels' two-level mismatch count: whatever order the workgroups finish in,
    exactly one of them writes the call's total, and every counter word is 0 afterwards (the next
    call that takes the entry starts clean, no memset)."""
    rng = np.random.default_rng(G)
    counts = [int(x) for x in rng.integers(0, 600, G)]
    for _ in range(5):
        writes, words = call_mismatch_count(G, counts, rng.permutation(G))
        assert writes == [sum(counts)] and words == [0] * 9


@pytest.mark.parametrize("seed,count,grid,L", [(50, 4096, 16, 1024), (51, 4000, 16, 256), (52, 2047, 8, 4096),
                                               (53, 999, 4, 3000)])
def test_small_kernel_repack2_fixed_sizes(seed, count, grid, L):
    """REPACK2 on a fixed-size channel (one line count per wave: the local tiles' line / n map),
    every line once, loads in their messages, ring words complete."""
    rng = np.random.default_rng(seed)
    lengths = np.full(count, L)
    lengths[count // 2] = L - 1  # one wave not FAST when L = 4096
    starts = np.arange(count) * ((L + 15 + 63) & ~63) + 64
    lines, wgs = {}, 0
    for kind, a, b, *rest in small_kernel_repack2(starts, lengths, grid, rng):
        if kind == "wgs":
            wgs = a
        elif kind == "line":
            lines[(a, b)] = lines.get((a, b), 0) + 1
        elif kind == "load":
            s, e = int(starts[a]), int(starts[a] + lengths[a])
            assert b % 16 == 0 and b + 16 > s and b < e, (a, s, e, b)
        elif kind == "ring":
            assert b == rest[0], (a, b, rest[0])
    assert wgs > 0 and all(v == 1 for v in lines.values())
