"""Seeded random batches through subspace_crc32_batch (the ragged pipeline: tile-count scan,
descriptors, ragged kernel, segment scans, final kernel), bit-exact against the oracle's byte
loop over the same arena: random lengths (0, tiny, around 8 KiB tiles, up to 1 MiB), random
starts (packed with gaps, any alignment, or overlapping), random init / final XOR, tight and
loose arena bounds."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
DEV = "cuda"


def lengths_for(rng, count):
    kind = rng.integers(0, 4, count)
    small = rng.integers(0, 300, count)
    tile = 8192 * rng.integers(1, 5, count) + rng.integers(-2, 3, count)
    mid = rng.integers(300, 40_000, count)
    big = rng.integers(40_000, 1 << 20, count)
    L = np.select([kind == 0, kind == 1, kind == 2], [small, tile, mid], big)
    L[rng.random(count) < 0.05] = 0
    return np.maximum(L, 0).astype(np.uint64)


@pytest.mark.parametrize("case", range(48))
def test_ragged_random_batches(gpu_ctx, oracle, case):
    rng = np.random.default_rng(0x2A66ED + case)
    count = int(rng.choice([1, 2, 7, 64, 1000, int(rng.integers(1000, 6000))]))
    L = lengths_for(rng, count)
    while int(L.sum()) > (160 << 20):
        L = L // np.uint64(2)
    layout = int(rng.integers(0, 3))
    if layout == 0:  # packed in order, random gaps and alignment
        gaps = rng.integers(0, 40, count).astype(np.uint64)
        starts = np.concatenate([[0], np.cumsum(L + gaps)[:-1]]).astype(np.uint64) + np.uint64(rng.integers(0, 16))
    elif layout == 1:  # packed, shuffled order
        perm = rng.permutation(count)
        pos = np.concatenate([[0], np.cumsum(L[perm])[:-1]]).astype(np.uint64)
        starts = np.empty(count, dtype=np.uint64)
        starts[perm] = pos
    else:  # overlapping: every start somewhere in a shared region
        region = int(max(int(L.max()) if count else 1, 1 << 16))
        starts = rng.integers(0, region, count).astype(np.uint64)
    end = int((starts + L).max()) if count else 0
    arena = rng.integers(0, 256, end + 64, dtype=np.uint8)
    init = int(rng.choice([0xFFFFFFFF, 0, int(rng.integers(0, 1 << 32))]))
    fin = bool(rng.integers(0, 2))
    buf = torch.from_numpy(arena).to(DEV)
    d_off = torch.from_numpy(starts.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(L.view(np.int64)).to(DEV)
    out = torch.full((count,), 0xDEAD, dtype=torch.int32, device=DEV)
    tight = bool(rng.integers(0, 2))
    gpu_ctx.crc32_ragged(buf, d_off, d_len, out, init=init, finalize=fin, arena_bytes=end if tight else None)
    torch.cuda.synchronize()
    gpu_ctx.check()
    got = out.cpu().numpy().view(np.uint32)
    want = oracle.crc32_batch(arena, starts, L, init=init, threads=8)
    if fin:
        want = ~want
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (case, count, layout, len(bad), bad[:5], L[bad[:5]])
