"""CPU model of the ragged kernel's load addresses (subspace_amd/csrc/crc_ragged.hip,
make_desc + load_line): every 16-B block any lane loads must overlap its own message,
so no load can leave the caller's buffer. Runs without a GPU."""
import numpy as np
import pytest


def tiles_for_length(n):
    return (n + 8191) >> 13


def loaded_blocks(s, e):
    """(lane, block, src) for every load the kernel issues for message [s, e)."""
    n = e - s
    nt = tiles_for_length(n)
    for j in range(nt):
        tile_end = e - ((nt - 1 - j) << 13)
        mis = (tile_end & 15) != 0
        safe = s & ~15
        for lane in range(64):
            line_start = tile_end - 8192 + lane * 128
            a0 = line_start & ~15
            for b in range(9):
                blk = a0 + 16 * b
                need = (b < 8 or mis) and blk + 16 > s
                yield lane, b, (blk if need else safe), need


@pytest.mark.parametrize("seed", range(6))
def test_every_load_overlaps_its_message(seed):
    rng = np.random.default_rng(seed)
    for _ in range(300):
        s = int(rng.integers(0, 5000))
        n = int(rng.choice([rng.integers(1, 300), rng.integers(1, 40000), 8192 * int(rng.integers(1, 4)) + int(rng.integers(-20, 20))]))
        n = max(n, 1)
        e = s + n
        for lane, b, src, need in loaded_blocks(s, e):
            assert src + 16 > s and src < e, (s, e, lane, b, src)
            assert src >= 0


def test_needed_blocks_cover_message():
    # the blocks marked `need` cover every message byte exactly once per line window
    for s, n in [(0, 1), (3, 100), (17, 8192), (5, 8193), (0, 4096), (1, 65536 + 7)]:
        e = s + n
        covered = set()
        for lane, b, src, need in loaded_blocks(s, e):
            if need:
                covered.update(range(max(src, s), min(src + 16, e)))
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


@pytest.mark.parametrize("count,stride", [(1, 4096), (2, 4096), (3, 4160), (1000, 4096), (4097, 8192), (65537, 4096)])
def test_uniform_kernel_lines_stay_in_messages(count, stride):
    """Replays crc32_uniform4k_kernel's line_ptr / prefetch clamping (order 0, 256 x 8 waves)."""
    ntiles = (count + 1) // 2
    nblocks, wpb = 256, 8
    nw = nblocks * wpb
    for w in range(nw):
        t0, tstep = w, nw
        nk = (ntiles - t0 + tstep - 1) // tstep if t0 < ntiles else 0
        ks = [0] if nk else []
        k = 0
        while k < nk:  # prefetch(B, k+1); process(A, k); prefetch(A, k+2); process(B, k+1)
            ks += [min(k + 1, nk - 1), min(k + 2, nk - 1)]
            k += 2
        for kk in ks:
            for h in (0, 1):
                msg = 2 * (t0 + kk * tstep) + h
                msg = msg if msg < count else msg - 1
                assert 0 <= msg < count
        if nk == 0:
            continue  # idle waves read lines of message 0 (base + l*128 for h == 0, else base)


def front_slot(b, G, wid):
    """crc_device.h front_slot: consecutive pairs of sweep-front slots go to consecutive
    workgroups (round-robin over XCDs)."""
    return (b + G * (wid >> 1)) * 2 + (wid & 1)


@pytest.mark.parametrize("wg", [256, 512, 640, 768, 1024])
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
