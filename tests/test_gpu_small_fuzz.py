"""Seeded random shapes through the small-message kernel's forms (crc_small.hip: packed G = 1 .. 32,
the uniform FAST loop with and without padding, the slot FAST loop, REPACK, the general loop,
long messages), bit-exact against the oracle: uniform batches of random length, stride,
alignment, count, init and final XOR; slot lists of random bounds, sizes (some past the bound),
payload alignment and span sizes, published and then verified after bit flips."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from subspace_amd import gpu  # noqa: E402
from test_gpu_parity import expected_uniform  # noqa: E402
from test_gpu_small import build_slot_list, oracle_arena, run_slot_list  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("case", range(64))
def test_uniform_random_shapes(gpu_ctx, oracle, case):
    rng = np.random.default_rng(0xF022 + case)
    L = int(rng.choice([int(rng.integers(1, 129)), int(rng.integers(129, 1025)), int(rng.integers(1025, 4097))]))
    stride = L + int(rng.choice([0, 0, 16 - (L % 16) if L % 16 else 0, int(rng.integers(1, 64))]))
    count = int(rng.choice([2, 3, 63, 64, 65, int(rng.integers(100, 5000)), int(rng.integers(5000, 60_000))]))
    count = max(2, min(count, (96 << 20) // max(stride, 1)))
    init = int(rng.choice([0, 0xFFFFFFFF, int(rng.integers(0, 1 << 32))]))
    fin = bool(rng.integers(0, 2))
    pad = int(rng.integers(0, 3)) * 16 + int(rng.integers(0, 16))  # (the allocation's end: any)
    seed = 0xF0220 + case
    buf = torch.empty(stride * (count - 1) + L + pad, dtype=torch.uint8, device=DEV)
    gpu.fill_uniform(buf, stride, L, count, seed=seed)
    out = torch.full((count,), 0xDEAD, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_uniform(buf, stride, L, count, out, init=init, finalize=fin)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    want = expected_uniform(oracle, count, L, seed, init=init, finalize=fin)
    bad = np.nonzero(got != want)[0]
    assert len(bad) == 0, (L, stride, count, init, fin, len(bad), bad[:5])


@pytest.mark.parametrize("case", range(48))
def test_slot_list_random_shapes(gpu_ctx, oracle, case):
    rng = np.random.default_rng(0x5F022 + case)
    bound = int(rng.choice([int(rng.integers(1, 200)), int(rng.integers(200, 2100)), 4096]))
    gen_max = int(rng.choice([bound, max(1, bound // int(rng.integers(2, 20)))]))  # (REPACK when small)
    count = int(rng.choice([1, 2, 65, int(rng.integers(100, 3000)), int(rng.integers(3000, 40_000))]))
    cs = int(rng.choice([4, 4, 8, 20]))
    ms = int(rng.choice([0, 0, 16, 5, 100]))
    mis = float(rng.choice([0.0, 0.0, 0.2]))
    over = float(rng.choice([0.0, 0.0, 0.01]))
    pre, pay, pay_off, sizes, order, ps = build_slot_list(count, 0x5F0220 + case, cs, ms, gen_max, mis, over,
                                                          over_max=bound + 3000)
    got_pre, st, _ = run_slot_list(gpu_ctx, pre, pay, pay_off, sizes, order, ps, cs, ms, bound, gpu.SLOT_CALCULATE)
    arena, po, yo = oracle_arena(pre, pay, pay_off, count, ps)
    oracle.publish_slots(arena, po, yo, sizes, cs, ms)
    assert (st == 0).all()
    bad = np.nonzero(got_pre != arena[:len(pre)])[0]
    assert len(bad) == 0, (bound, gen_max, count, cs, ms, np.unique(bad // ps)[:8])
    pay2 = pay.copy()
    for i in np.nonzero(rng.random(count) < 0.1)[0]:
        if sizes[i]:
            pay2[int(pay_off[i]) + int(rng.integers(0, int(sizes[i])))] ^= np.uint8(1 << int(rng.integers(0, 8)))
    _, st, err = run_slot_list(gpu_ctx, got_pre, pay2, pay_off, sizes, order, ps, cs, ms, bound, gpu.SLOT_VERIFY)
    arena2, po, yo = oracle_arena(got_pre, pay2, pay_off, count, ps)
    want = oracle.verify_slots(arena2, po, yo, sizes, cs, ms)
    assert np.array_equal(st, want), (bound, gen_max, count, cs, ms)
    assert err == int((want == 1).sum())
