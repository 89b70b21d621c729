"""CPU model of the kernels' CRC decomposition (the algebra, not the HIP code):
the ragged kernel's 16-B aligned tiles (head bytes masked, first line seeded with
Z_mis^{-1}(init)) with a zero-padded last tile, per-lane line-shift
operators + DPP half reduction, Z_4096 join, Z_{8192*T} shift, XOR combine and the
padding undone with Z_{2^b}^{-1}; the uniform kernel's per-line
CRCs and transposed tree. Each must equal the reference CRC (zlib) bit for bit."""
import zlib

import numpy as np
import pytest

M32 = 0xFFFFFFFF
POLY = 0xEDB88320
TABLE = []
for b in range(256):
    c = b
    for _ in range(8):
        c = (c >> 1) ^ POLY if c & 1 else c >> 1
    TABLE.append(c)


def crc_raw(c, data):
    for x in data:
        c = (c >> 8) ^ TABLE[(c ^ x) & 0xFF]
    return c


def apply(m, v):
    r = 0
    i = 0
    while v:
        if v & 1:
            r ^= m[i]
        v >>= 1
        i += 1
    return r


def mul(a, b):
    return [apply(a, col) for col in b]


Z1 = [((1 << i) >> 8) ^ TABLE[(1 << i) & 0xFF] for i in range(32)]
IDENT = [1 << i for i in range(32)]


def zbytes(n):
    r, p = IDENT, Z1
    while n:
        if n & 1:
            r = mul(p, r)
        p = mul(p, p)
        n >>= 1
    return r


def inverse(m):
    rows = [sum(((m[c] >> r) & 1) << c for c in range(32)) for r in range(32)]
    inv = [1 << r for r in range(32)]
    for c in range(32):
        p = next(i for i in range(c, 32) if (rows[i] >> c) & 1)
        rows[c], rows[p] = rows[p], rows[c]
        inv[c], inv[p] = inv[p], inv[c]
        for r in range(32):
            if r != c and (rows[r] >> c) & 1:
                rows[r] ^= rows[c]
                inv[r] ^= inv[c]
    return [sum(((inv[r] >> c) & 1) << r for r in range(32)) for c in range(32)]


ZINV_POW2 = [inverse(zbytes(1 << b)) for b in range(13)]  # the final kernel's padding inverses
ZTREE = [zbytes(128 << k) for k in range(6)]
ZTILE = [zbytes(8192 << k) for k in range(8)]
LANE_OPS = [zbytes(128 * sl) for sl in range(32)]
Z4096 = zbytes(4096)


def ragged_model(buf: bytes, s: int, L: int, init: int) -> int:
    e = s + L
    if L == 0:
        return init
    mis = s & 15
    s0 = s - mis  # the extended message [s0, e): its first mis bytes are masked to zero
    nt = (L + mis + 8191) >> 13
    out = 0
    for j in range(nt):
        ts = s0 + (j << 13)
        lines = []
        for lane in range(64):
            ls = ts + 128 * lane
            data = bytearray(128)  # bytes outside [s, e) stay zero (head mask, padded last tile)
            for i in range(128):
                if s <= ls + i < e:
                    data[i] = buf[ls + i]
            seed = 0
            if j == 0 and lane == 0:
                seed = init
                for b in range(4):  # Z_mis^{-1}(init): after the mis zero bytes the state is init
                    if (mis >> b) & 1:
                        seed = apply(ZINV_POW2[b], seed)
            lines.append(crc_raw(seed, bytes(data)))
        # per lane: Z_{128*(31 - l%32)} on its line; XOR over each half (DPP); the halves
        # joined with Z_4096; then the shift to the padded message end, Z_{8192*T}
        shifted = [apply(LANE_OPS[31 - (lane & 31)], lines[lane]) for lane in range(64)]
        red = dpp_half_xor(shifted)
        t = apply(Z4096, red[31]) ^ red[63]
        after = nt - 1 - j
        k = 0
        while after:
            if after & 1:
                t = apply(ZTILE[k], t)
            after >>= 1
            k += 1
        out ^= t
    # out = Z_p(crc_raw(init, D)), p = 8192*nt - (L + mis): undo the padding
    pad = (-(L + mis)) % 8192
    for b in range(13):
        if (pad >> b) & 1:
            out = apply(ZINV_POW2[b], out)
    return out


def uniform_model(msg: bytes, init: int) -> int:
    assert len(msg) == 4096
    lines = [crc_raw(init if i == 0 else 0, msg[128 * i:128 * i + 128]) for i in range(32)]
    # lane q holds lines 4q..4q+3: a = Z128(s0)^s1, b = Z128(s2)^s3, c = Z256(a)^b
    quads = []
    for q in range(8):
        s0, s1, s2, s3 = lines[4 * q:4 * q + 4]
        a = apply(ZTREE[0], s0) ^ s1
        b = apply(ZTREE[0], s2) ^ s3
        quads.append(apply(ZTREE[1], a) ^ b)
    cur = quads
    for k in (2, 3, 4):
        cur = [apply(ZTREE[k], cur[2 * i]) ^ cur[2 * i + 1] for i in range(len(cur) // 2)]
    return cur[0]


def ref(state, data):
    return (~zlib.crc32(bytes(data), (~state) & M32)) & M32


@pytest.mark.parametrize("init", [M32, 0, 0x12345678])
def test_uniform_decomposition(init):
    rng = np.random.default_rng(init & 0xFFFF)
    msg = rng.integers(0, 256, 4096, dtype=np.uint8).tobytes()
    assert uniform_model(msg, init) == ref(init, msg)


@pytest.mark.parametrize("s,L", [(0, 1), (0, 100), (3, 128), (5, 129), (16, 8192), (7, 8191), (1, 8193),
                                 (100, 20000), (0, 3 * 8192), (13, 2 * 8192 + 300)])
def test_ragged_decomposition(s, L):
    rng = np.random.default_rng(s * 7 + L)
    buf = rng.integers(0, 256, s + L + 64, dtype=np.uint8).tobytes()
    for init in (M32, 0xA5A5A5A5):
        assert ragged_model(buf, s, L, init) == ref(init, buf[s:s + L]), (s, L, hex(init))


def test_uniform_line_as_two_64b_chains():
    """ILP = 2 in crc32_uniform4k_kernel: a line's CRC from two independent 64-B chains,
    Z_64(crc(s, first half)) ^ crc(0, second half) == crc(s, line)."""
    z64 = zbytes(64)
    rng = np.random.default_rng(64)
    for init in (M32, 0, 0x0BADCAFE):
        line = rng.integers(0, 256, 128, dtype=np.uint8).tobytes()
        assert apply(z64, crc_raw(init, line[:64])) ^ crc_raw(0, line[64:]) == crc_raw(init, line)


def dpp_half_xor(vals):
    """crc32_uniform4k_kernel's reduction: XOR with row_shr 1, 2, 4, 8 (lanes whose source
    falls outside the 16-lane row keep their value), then row_bcast:15 into rows 1 and 3.
    Returns the 64 lane values."""
    v = list(vals)
    for n in (1, 2, 4, 8):
        v = [v[i] ^ (v[i - n] if (i % 16) >= n else 0) for i in range(64)]
    bc = [0] * 64
    for r in (1, 3):
        for i in range(16 * r, 16 * r + 16):
            bc[i] = v[16 * r - 1]
    return [v[i] ^ bc[i] for i in range(64)]


def test_uniform_per_lane_operators_and_dpp_reduction():
    """Per tile: lane l of half h applies Z_{128*(31-l)} to its line CRC; the DPP
    reduction leaves message 2*tau + h's CRC in lane 32*h + 31."""
    ops = [zbytes(128 * s) for s in range(32)]
    rng = np.random.default_rng(31)
    for init in (M32, 0x1234ABCD):
        msgs = [rng.integers(0, 256, 4096, dtype=np.uint8).tobytes() for _ in range(2)]
        lanes = []
        for h in range(2):
            for l in range(32):
                line = msgs[h][128 * l:128 * l + 128]
                lanes.append(apply(ops[31 - l], crc_raw(init if l == 0 else 0, line)))
        red = dpp_half_xor(lanes)
        assert red[31] == ref(init, msgs[0]) and red[63] == ref(init, msgs[1])


def tilecrc_index(w, k, nwb):
    """crc_device.h tilecrc_index: 64 x 64 blocks of (w, k), w-major inside a block."""
    return ((((k >> 6) * nwb + (w >> 6)) << 6 | (w & 63)) << 6) | (k & 63)


def local_index(w, k, nwb):
    """crc_device.h local_index: the same blocks, k-major inside a block."""
    return ((((k >> 6) * nwb + (w >> 6)) << 6 | (k & 63)) << 6) | (w & 63)


def _segment_combine_model(values_tau, nw):
    """Replay of crc_combine.hip on the CPU: the blocked tile-value array the main kernels write
    (tile tau = k*nw + w at tilecrc_index(w, k)), tile_segment_scan_kernel (block (a, b): 64-tile
    row segments, inclusive XOR scan per segment into local_index(w, k), segment XORs),
    segment_prefix_kernel (exclusive XOR scan of the segment XORs) and tile_prefix (crc_device.h)."""
    n = len(values_tau)
    nkmax = -(-max(n, 1) // nw)
    nwb = -(-nw // 64)
    nblk = -(-nkmax // 64) * nwb
    tilecrc = np.full(nblk * 4096, 0xDEADBEEF, dtype=np.uint32)  # never-written entries: garbage
    for t in range(n):
        tilecrc[tilecrc_index(t % nw, t // nw, nwb)] = values_tau[t]
    local = np.full(nblk * 4096, 0xDEADBEEF, dtype=np.uint32)
    segx = np.zeros(nkmax * nwb, dtype=np.uint32)
    for a in range(-(-nkmax // 64)):
        for b in range(nwb):
            blk = (a * nwb + b) * 4096
            tile = np.zeros((64, 64), dtype=np.uint32)  # t[y][x]: w = 64 b + y, k = 64 a + x
            for y in range(64):
                for x in range(64):
                    w, k = 64 * b + y, 64 * a + x
                    if w < nw and k < nkmax:
                        assert blk + 64 * y + x == tilecrc_index(w, k, nwb)
                        tile[y][x] = tilecrc[blk + 64 * y + x]
            for y in range(64):  # row k = 64 a + y
                k = 64 * a + y
                if k >= nkmax:
                    continue
                scan = np.bitwise_xor.accumulate(tile[:, y])
                for x in range(64):
                    w = 64 * b + x
                    if w < nw and k * nw + w < n:
                        assert blk + 64 * y + x == local_index(w, k, nwb)
                        local[blk + 64 * y + x] = scan[x]
                segx[k * nwb + b] = scan[63]
    excl = np.zeros_like(segx)
    excl[1:] = np.bitwise_xor.accumulate(segx)[:-1]

    def tile_prefix(t):
        k, w = t // nw, t % nw
        return int(excl[k * nwb + (w >> 6)] ^ local[local_index(w, k, nwb)])
    return tile_prefix


@pytest.mark.parametrize("nw,n", [(128, 1000), (2048, 5000), (96, 777), (64, 64), (2048, 1)])
def test_segment_prefix_decomposition_equals_full_xor_scan(nw, n):
    """P(tau) = segx[s(tau)] ^ local[tau] is the inclusive XOR prefix in tile order, for
    nw a multiple of 64 or not (the last segment of a row is then short)."""
    rng = np.random.default_rng(nw * 7 + n)
    vals = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    tp = _segment_combine_model(vals, nw)
    full = np.bitwise_xor.accumulate(vals)
    for t in list(range(min(n, 300))) + list(range(max(0, n - 300), n)):
        assert tp(t) == int(full[t])
    # a message [t0, t1) is P(t1 - 1) ^ P(t0 - 1)
    t0, t1 = n // 3, max(n // 3 + 1, 2 * n // 3)
    if t1 <= n:
        want = int(np.bitwise_xor.reduce(vals[t0:t1]))
        assert tp(t1 - 1) ^ (tp(t0 - 1) if t0 else 0) == want
