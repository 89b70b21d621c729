"""Stale device state is reported, never returned as OK.

The look-back scans of the ragged path (crc_combine.hip) keep a ticket and status words in
the context that every call expects at zero. A stale ticket used to be absorbed by a bounded
spin that substituted the identity prefix: wrong CRCs and SUBSPACE_CRC_OK. Now the kernels
raise a bit in the context's fault word, the downstream kernels of that call (its generation
in the fault words) skip work that would index with an untrusted tile_base, and
subspace_crc_ctx_check returns SUBSPACE_CRC_EFAULT (then clears the fault and resets the scan
state). A later call is correct with or without a check in between.
"""
import ctypes

import numpy as np
import pytest

from subspace_amd import _lib, gpu, synth

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _ragged_batch(n, seed):
    lengths = synth.ragged_lengths(seed, n) // np.uint64(64)
    offsets, total = synth.packed_offsets(lengths, align=1)
    buf = torch.empty(total + 64, dtype=torch.uint8, device=DEV)
    d_off = torch.from_numpy(offsets.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lengths.view(np.int64)).to(DEV)
    gpu.fill_ragged(buf, d_off, d_len, seed=seed)
    return buf, d_off, d_len, lengths


@pytest.mark.parametrize("ticket", [1 << 30, 1])
def test_stale_scan_ticket_reports_efault(gpu_ctx, oracle, ticket):
    """ticket 2^30: every workgroup's ticket is beyond the grid (kFaultTicket, no wait);
    ticket 1: tickets 1.. wait for a predecessor that never publishes (kFaultLookbackSpin
    after the bounded spin, ~1 s) and the last one is beyond the grid."""
    n = 3 * 4096  # four count-scan workgroups
    buf, d_off, d_len, lengths = _ragged_batch(n, seed=0xFA17)
    want = oracle.synth_crc_batch(0xFA17, lengths)
    out = torch.empty(n, dtype=torch.int32, device=DEV)
    gpu_ctx.check()  # nothing pending
    gpu_ctx.crc32_ragged(buf, d_off, d_len, out)
    gpu_ctx.check()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    assert _lib.load_dev().subspace_crc_testutil_set(gpu_ctx._h, b"stale_ticket", ticket) == 0
    gpu_ctx.crc32_ragged(buf, d_off, d_len, out)  # asynchronous: returns OK
    with pytest.raises(gpu.CrcError) as ei:
        gpu_ctx.check()
    assert ei.value.code == gpu.EFAULT
    assert "scan" in str(ei.value)
    # the fault is cleared and the scan state reset: the next call is correct and clean
    out.fill_(0)
    gpu_ctx.crc32_ragged(buf, d_off, d_len, out)
    gpu_ctx.check()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


def test_calls_on_two_streams_are_ordered(gpu_ctx, oracle):
    """Ragged calls that share the context's workspaces, issued on two streams without any
    user synchronisation, give the right results (the second call's stream waits for the
    first's workspace use)."""
    n = 20000
    b1, o1, l1, len1 = _ragged_batch(n, seed=0x5151)
    b2, o2, l2, len2 = _ragged_batch(n, seed=0x5252)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out1 = torch.zeros(n, dtype=torch.int32, device=DEV)
    out2 = torch.zeros(n, dtype=torch.int32, device=DEV)
    for _ in range(3):
        gpu_ctx.crc32_ragged(b1, o1, l1, out1, stream=s1)
        gpu_ctx.crc32_ragged(b2, o2, l2, out2, stream=s2)
    torch.cuda.synchronize()
    gpu_ctx.check()
    assert np.array_equal(out1.cpu().numpy().view(np.uint32), oracle.synth_crc_batch(0x5151, len1))
    assert np.array_equal(out2.cpu().numpy().view(np.uint32), oracle.synth_crc_batch(0x5252, len2))


def test_fault_marks_only_its_own_call(gpu_ctx, oracle):
    """a scan fault marks the call it happened in (the fault words' generation),
    not every later one. A caller that never calls check still gets correct CRCs from the next
    call (whose kernels start from the state the faulted call's later kernels reset), and the
    fault is still reported by the next check."""
    n = 3 * 4096
    buf, d_off, d_len, lengths = _ragged_batch(n, seed=0xFA18)
    want = oracle.synth_crc_batch(0xFA18, lengths)
    out = torch.zeros(n, dtype=torch.int32, device=DEV)
    gpu_ctx.reserve(n, 4 * n)  # (the stale ticket is planted in the ragged workspace)
    gpu_ctx.check()
    assert _lib.load_dev().subspace_crc_testutil_set(gpu_ctx._h, b"stale_ticket", 1 << 30) == 0
    gpu_ctx.crc32_ragged(buf, d_off, d_len, out)  # faults: its kernels skip
    out2 = torch.zeros(n, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_ragged(buf, d_off, d_len, out2)  # no check in between
    torch.cuda.synchronize()
    assert np.array_equal(out2.cpu().numpy().view(np.uint32), want)
    with pytest.raises(gpu.CrcError) as ei:
        gpu_ctx.check()
    assert ei.value.code == gpu.EFAULT
    gpu_ctx.check()  # cleared


def test_fault_mark_does_not_outlive_a_graph_replay(gpu_ctx, oracle):
    """a captured ragged call replays the same generation every time. A scan fault
    in one replay marks that generation; the next replay's tile-count scan (ticket 0) clears the
    mark, so the replay after a faulted one computes every CRC without a check in between, and
    the fault is still reported by the next check."""
    n = 3 * 4096
    buf, d_off, d_len, lengths = _ragged_batch(n, seed=0xFA19)
    want = oracle.synth_crc_batch(0xFA19, lengths)
    out = torch.zeros(n, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_ragged(buf, d_off, d_len, out)  # workspaces allocated before the capture
    torch.cuda.synchronize()
    gpu_ctx.check()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            gpu_ctx.crc32_ragged(buf, d_off, d_len, out, stream=s)
    torch.cuda.synchronize()
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    gpu_ctx.check()
    assert _lib.load_dev().subspace_crc_testutil_set(gpu_ctx._h, b"stale_ticket", 1 << 30) == 0
    g.replay()  # faults: its kernels skip
    torch.cuda.synchronize()
    out.zero_()
    torch.cuda.synchronize()
    g.replay()  # the same generation, no check in between
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
    with pytest.raises(gpu.CrcError) as ei:
        gpu_ctx.check()
    assert ei.value.code == gpu.EFAULT
    gpu_ctx.check()  # cleared
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    gpu_ctx.check()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


def _fault_words(ctx):
    w = (ctypes.c_uint32 * 2)()
    assert _lib.load_dev().subspace_crc_testutil_fault_words(ctx._h, w, None) == 0
    return int(w[0]), int(w[1])


def test_check_clears_the_fault_bits_but_keeps_the_generation_mark(gpu_ctx, oracle):
    """subspace_crc_ctx_check clears word 0 (the kFault* bits) only. Word 1, the
    generation of the call whose scan faulted, stays: a graph replay of that generation still
    running on another stream (replays record no workspace event, so the check cannot wait for
    them) must keep skipping its tile_base-indexed work. A later non-graph call takes a new
    generation and runs normally."""
    n = 3 * 4096
    buf, d_off, d_len, lengths = _ragged_batch(n, seed=0xFA1A)
    want = oracle.synth_crc_batch(0xFA1A, lengths)
    out = torch.zeros(n, dtype=torch.int32, device=DEV)
    gpu_ctx.crc32_ragged(buf, d_off, d_len, out)
    gpu_ctx.check()
    assert _fault_words(gpu_ctx)[0] == 0
    assert _lib.load_dev().subspace_crc_testutil_set(gpu_ctx._h, b"stale_ticket", 1 << 30) == 0
    gpu_ctx.crc32_ragged(buf, d_off, d_len, out)  # faults
    gen = int(_lib.load_dev().subspace_crc_testutil_call_gen(gpu_ctx._h))
    torch.cuda.synchronize()
    bits, mark = _fault_words(gpu_ctx)
    assert bits != 0 and mark == gen
    with pytest.raises(gpu.CrcError) as ei:
        gpu_ctx.check()
    assert ei.value.code == gpu.EFAULT
    bits, mark = _fault_words(gpu_ctx)
    assert bits == 0 and mark == gen  # the mark outlives the check
    out.zero_()
    gpu_ctx.crc32_ragged(buf, d_off, d_len, out)  # a new generation: not skipped
    assert int(_lib.load_dev().subspace_crc_testutil_call_gen(gpu_ctx._h)) != gen
    gpu_ctx.check()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
