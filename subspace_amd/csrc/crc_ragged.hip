// Ragged-batch kernels: one CRC32 per message for arbitrary offsets, lengths and
// alignment (BASELINE configs C and D; any subspace_crc32_batch call).
//
// Decomposition (DESIGN.md "Ragged kernel"):
//  * Message m = bytes [s, e), L = e - s, mis = s & 15. It is read as the EXTENDED message
//    [s0, e), s0 = s - mis (the 16-B block holding s), whose first mis bytes are masked to
//    zero, cut into nt = ceil((L + mis)/8192) tiles: tile j covers [s0 + 8192j, +8192), and
//    only the last tile can be short (len = L + mis - 8192(nt-1) bytes). Lane l of a tile
//    owns the 128-B line [s0 + 8192j + 128l, +128): 64 consecutive lines per wave load
//    instruction, exactly like the uniform kernel, and every line is whole aligned 16-B
//    blocks -- no realignment, whatever the message's alignment and length.
//  * Head: line 0 of tile 0 starts from seed[mis] = Z_mis^{-1}(init) (host-computed), so
//    after its mis zero bytes the state is exactly init:
//      crc_raw(Z_mis^{-1}(init), 0^mis || D) = crc_raw(init, D);
//    every other line starts from 0 (zero data from state 0 stays 0).
//  * Tail: the last tile is read as if zero-padded to 8 KiB (bytes at and past e masked),
//    so the tiles compute
//      crc_raw(init, D || 0^p) = Z_p(crc_raw(init, D)),   p = 8192*nt - (L + mis) < 8192,
//    and the final kernel undoes the padding with p's binary decomposition over the
//    inverse operators Z_{2^b}^{-1} (b = 0..12; Z_n is invertible since P has an x^0 term)
//    before the final XOR.
//  * Waves stream the global tile list in sweep order (tau = k*nw + w), one tile of
//    loads in flight ahead. Per-tile 8-B descriptors (tile start, tiles after, first-tile
//    flag, bytes in the last tile and mis; 16 B for batches with a tile start at or beyond 2^37
//    bytes or with 2^25 tiles after a tile: kDesc8StartBits / kDesc8AfterBits, crc_device.h) are
//    precomputed by crc32_ragged_desc_kernel (or the fused count + descriptor kernel).
//  * Per tile, lane l of half h applies its own line-shift operator Z_{128*(31-l)} (the
//    uniform kernel's conflict-free [nibble][value][lane] tables) and a DPP reduction
//    leaves the two half-tile values in lanes 31 and 63. They are parked, one tile per
//    lane, in registers (lane k&63 keeps tile k); every 64 tiles each lane finishes its own tile,
//      tile value = Z_{8192*T}( Z_4096(half0) ^ half1 )     (T = tiles after it)
//    with a per-lane binary decomposition of T over nibble operators -- one wave pass
//    shifts 64 tiles -- and stores them to tilecrc, wave-major ([w][k]: one wave's 64
//    values are 256 contiguous bytes). A message's padded CRC is the XOR of its tiles'
//    values, i.e. the difference of two entries of the inclusive XOR prefix of the values
//    in tile order tau (crc_combine.hip: tile_segment_scan_kernel, segment_prefix_kernel;
//    crc32_ragged_final_kernel). No atomics: huge messages (config D: 8192 tiles each, all
//    in flight at once) would otherwise serialise every tile on one output word.
//    (Batches whose tiles overflow the workspace -- overlapping messages -- fall back to
//    atomicXor into pre-zeroed words.)
//  * Loads never touch a 16-B block that holds no byte of the message.
#include "crc_desc.h"

namespace subspace_amd {

__device__ inline u64 find_msg(const u64* __restrict__ tile_base, u64 count, u64 tau) {
  // last m with tile_base[m] <= tau (skips zero-tile messages, whose base equals the next one's)
  u64 lo = 0, hi = count;  // invariant: tile_base[lo] <= tau < tile_base[hi]
  while (hi - lo > 1) {
    const u64 mid = (lo + hi) >> 1;
    if (tile_base[mid] <= tau) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Tiles of message (s, L): its extended length L + (s & 15) in 8 KiB tiles (0 if L = 0).
__device__ __forceinline__ u64 ext_tiles(u64 s, u64 len) { return len ? (len + (s & 15) + 8191) >> 13 : 0; }

__device__ inline TileDesc make_desc(const u64* __restrict__ offsets, u32 ostride, const u64* __restrict__ lengths,
                                     u32 lstride, const u64* __restrict__ tile_base, u64 m, u64 tau) {
  const u64 nt = tile_base[m + 1] - tile_base[m];
  const u64 j = tau - tile_base[m];
  const u64 s = offsets[m * ostride];
  const u64 L = lengths[m * lstride];
  const u32 mis = (u32)(s & 15);
  const u64 rest = L + mis - (j << 13);  // extended bytes from the tile start on
  TileDesc d;
  d.tile_start = (s & ~(u64)15) + (j << 13);
  d.after = (u32)(nt - 1 - j) | (j == 0 ? kFirstTile : 0u);
  d.len = (rest < 8192 ? (u32)rest : 8192u) | (mis << 16);
  // Defence in depth: a tile that is not one of the message's own (only possible with an
  // inconsistent tile_base, which the fault checks below already exclude) reads nothing: an
  // empty buffer range loads zeros without touching memory.
  if (j >= nt || j >= ext_tiles(s, L)) {
    d.tile_start = s & ~(u64)15;
    d.len = mis << 16;
  }
  return d;
}


// Per tile (up to `capacity`): its descriptor, 8 B unless the tile-count scan flagged the batch
// wide (overflow[1]). Sets overflow[0] if the batch has more tiles (then nothing is written:
// the main kernel searches). Message-centric: thread m of column x reads its message's tile
// range and (offset, length) with coalesced loads -- no search -- and the wave writes its 64
// messages' descriptors (crc_desc.h desc8_wave; 16-B ones one long message after the other);
// workgroup rows y share the later tiles of long messages (the host adds rows when a batch
// has few, long messages: config D). (Batches with a known arena below 2^37 bytes take the
// fused tile-count scan + descriptor kernel instead, crc_combine.hip.)
__global__ __launch_bounds__(256) void crc32_ragged_desc_kernel(const u64* __restrict__ offsets, u32 ostride,
                                                                const u64* __restrict__ lengths, u32 lstride,
                                                                const u64* __restrict__ tile_base, u64 count,
                                                                u64 capacity, TileDesc* __restrict__ desc,
                                                                u32* __restrict__ overflow, u64* scan_status,
                                                                u64 scan_words, u32* scan_ticket, FaultRef fault) {
  if (blockIdx.y == 0) reset_scan_state(scan_status, scan_words, scan_ticket);  // the tile-count scan is done
  if (scan_faulted(fault)) return;
  const u64 total = tile_base[count];
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) overflow[0] = total > capacity ? 1u : 0u;
  if (total > capacity) return;  // the search path: no descriptors
  const bool wide = overflow[1] != 0u;
  TileDesc8* const desc8 = reinterpret_cast<TileDesc8*>(desc);
  const u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  u64 t0 = 0, nt = 0, so = 0, L = 0;
  if (m < count) {
    t0 = tile_base[m];
    nt = tile_base[m + 1] - t0;
    so = offsets[m * ostride];
    L = lengths[m * lstride];
  }
  // tile j of the message at so with length tL, first tile tt0 and tnt tiles (16-B form)
  auto put = [&](u64 tso, u64 tL, u64 tt0, u64 tnt, u64 j) {
    const u32 mis = (u32)(tso & 15);
    const u64 rest = tL + mis - (j << 13);
    TileDesc d;
    d.tile_start = (tso & ~(u64)15) + (j << 13);
    d.after = (u32)(tnt - 1 - j) | (j == 0 ? kFirstTile : 0u);
    d.len = (rest < 8192 ? (u32)rest : 8192u) | (mis << 16);
    desc[tt0 + j] = d;
  };
  const u32 lane = threadIdx.x & 63u;
  const u32 y = rfl(blockIdx.y), ystep = 64u * rfl(gridDim.y);  // in SGPRs, read once
  if (!wide) {
    __shared__ u32 sxa[4][kDesc8WaveWords][64];
    desc8_wave(desc8, capacity, t0, nt, so, L, y, ystep, sxa[threadIdx.x >> 6], blockIdx.y == 0);
    return;
  }
  if (blockIdx.y == 0) {
#pragma unroll
    for (u32 j = 0; j < kLaneTiles; j++)
      if (j < nt) put(so, L, t0, nt, j);
  }
  // wide batches (16-B descriptors): one long message after the other, 64 tiles per store
  u64 big = __ballot(nt > kLaneTiles);
  while (big) {
    const int src = __ffsll((unsigned long long)big) - 1;
    big &= big - 1;
    const u64 bt0 = __shfl(t0, src, 64), bnt = __shfl(nt, src, 64);
    const u64 bso = __shfl(so, src, 64), bL = __shfl(L, src, 64);
    for (u64 j = kLaneTiles + 64ull * y + lane; j < bnt; j += ystep) put(bso, bL, bt0, bnt, j);
  }
}

// ------------------------------------------------------------------ main kernel

// MODE: kDescSearch (no descriptors: every tile located by binary search), kDesc16, kDesc8.
constexpr int kDescSearch = 0, kDesc16 = 1, kDesc8 = 2;
template <int WG, int MODE>
__device__ __forceinline__ void ragged_body(const uint8_t* __restrict__ base, const u64* __restrict__ offsets,
                                            u32 ostride, const u64* __restrict__ lengths, u32 lstride,
                                            const u64* __restrict__ tile_base, u64 count,
                                            const TileDesc* __restrict__ desc, const u32* __restrict__ gtab,
                                            const u32* __restrict__ gops, const HeadSeeds& seeds,
                                            u32* __restrict__ out, u32* __restrict__ tilecrc, u32 nwb,
                                            u32 sbase) {
  const int lane = threadIdx.x & 63;
  const u32 wid = rfl(threadIdx.x >> 6);
  const u32 lc0 = sbase + ((u32)(lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  const u32 z64 = sbase + kLdsOps + 4u * (u32)kRagZ64Words + 4u * (u32)(lane & 3);  // Z_64 copy lane & 3
  const u32 lop = sbase + kLdsOps + 4u * (u32)(31 - (lane & 31));  // this lane's line-shift operator
  const u64 total = tile_base[count];
  const u64 w = front_slot(blockIdx.x, gridDim.x, wid);  // sweep front slot (crc_device.h)
  const u64 nw = (u64)gridDim.x * (WG / 64);
  const u64 nk = w < total ? (total - w + nw - 1) / nw : 0;  // tiles tau = k*nw + w, k < nk
  if (total == 0) return;  // every message empty: all waves of all blocks leave before any load
  // An opaque zero in a VGPR: descriptor loads indexed with it are vector loads, so they
  // retire in order with the line loads (vmcnt) instead of coupling with LDS (lgkmcnt).
  u32 vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));

  // Descriptor of tile k as raw dwords (a vector load; kDescSearch: built by search, with
  // the message id for the atomic path). Past the wave's last tile it is clamped to that
  // tile; a wave without tiles uses the batch's last tile, so every load the kernel issues
  // stays inside a real message.
  constexpr bool DESC = MODE != kDescSearch;
  auto fetch_desc = [&](u64 k, u32x4& d, u32& dm) {
    const u64 tau = nk ? (k < nk ? k : nk - 1) * nw + w : total - 1;
    if (MODE == kDesc8) {
      const u32x2 v = *reinterpret_cast<const u32x2*>(reinterpret_cast<const TileDesc8*>(desc) + tau + vzero);
      d = u32x4{v[0], v[1], 0u, 0u};
      dm = 0;
    } else if (MODE == kDesc16) {
      d = *reinterpret_cast<const u32x4*>(desc + tau + vzero);
      dm = 0;
    } else {
      const u64 m = find_msg(tile_base, count, tau);
      const TileDesc t = make_desc(offsets, ostride, lengths, lstride, tile_base, m, tau);
      d = u32x4{(u32)t.tile_start, (u32)(t.tile_start >> 32), t.after, t.len};
      dm = (u32)m;
    }
  };
  auto unpack = [&](const u32x4& d) {
    if constexpr (MODE == kDesc8) return unpack_desc8(rfl(d[0]), rfl(d[1]));
    TileDesc t;
    t.tile_start = rfl64(d[0], d[1]);
    t.after = rfl(d[2]);
    t.len = rfl(d[3]);
    return t;
  };
  // Issue the loads of tile d: buffer loads against a scalar resource spanning exactly the
  // 16-B blocks that hold the tile's bytes, [tile start, tile end rounded up to 16). Lane l
  // loads the 8 blocks from 128*l; blocks past the range (past the message end) read as
  // zeros without touching memory, so every lane issues every load (no divergent branch
  // around loads). `live` false (a prefetch past the wave's last tile) gives an empty range.
  auto load_line = [&](const TileDesc& d, u32x4 (&L)[8], bool live) {
    const u32 nrec = live ? (((d.len & 0xFFFFu) + 15u) & ~15u) : 0u;
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base + d.tile_start), (short)0,
                                                     (int)nrec, kBufferRsrcFlags);
    const u32 vo = (u32)lane * 128u;
#pragma unroll
    for (int b = 0; b < 8; b++) L[b] = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 16u * b, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };

  // Half-tile values parked one tile per lane (slot k & 63), finished every 64 tiles.
  u32 H0 = 0, H1 = 0, AF = 0, MG = 0;  // half 0, half 1, after | kFirstTile, message (DESC false)

  auto process = [&](const u32x4 (&cur)[8], const TileDesc& dcur, u32 dm, u64 k) {
    const bool first = (dcur.after & kFirstTile) != 0;  // wave-uniform, like everything below
    const u32 len = dcur.len & 0xFFFFu, mis = dcur.len >> 16;
    u32x4 d[8];
#pragma unroll
    for (int b = 0; b < 8; b++) d[b] = cur[b];
    // Head: the first tile's first mis bytes precede the message (lane 0's first block).
    // Tail: a short tile whose end is not 16-B aligned also holds bytes past the message in
    // its last loaded block. Each lane keeps only its line's message bytes.
    const bool head = first && mis != 0u, tail = len < 8192u && (len & 15u) != 0u;
    if (head || tail) {
      const int v0 = (int)len - 128 * lane;
      const u32 hi = v0 <= 0 ? 0u : (v0 >= 128 ? 128u : (u32)v0);
      const u32 lo = (head && lane == 0) ? mis : 0u;
      keep_bytes(d, lo, hi);
    }
    const u32 crc = line_crc32_2chain(d, (first && lane == 0) ? seeds.v[mis] : 0u, lc0, lc1, z64);

    // line l of half h -> Z_{128*(31-l)}(line): 8 conflict-free nibble lookups; then XOR
    // over each half with DPP (lane 31: lines 0..31, lane 63: lines 32..63)
    u32 v = lane_shift(lop, crc);
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    const u32 h0 = (u32)__builtin_amdgcn_readlane((int)v, 31), h1 = (u32)__builtin_amdgcn_readlane((int)v, 63);
    const bool mine = lane == (int)(k & 63);  // one compare, selects of wave-uniform values
    H0 = mine ? h0 : H0;
    H1 = mine ? h1 : H1;
    AF = mine ? dcur.after : AF;
    if (!DESC) MG = mine ? dm : MG;
  };

  // Finish and store the parked tiles kf .. kf+nt-1 (lane i holds tile kf + i).
  auto flush = [&](u64 kf, u32 nt) {
    const bool valid = (u32)lane < nt;
    u32 c = opmul(sbase, kRagOpZ4096, H0) ^ H1;  // the tile's 8 KiB from its two halves
    u32 rem = valid ? (AF & ~kFirstTile) : 0u;   // shift to the (padded) message end: Z_{8192 * after}
    int bit = 0;
    for (; bit < kNumTileOps && __any(rem != 0u); bit++) {
      const u32 cm = opmul(sbase, kRagOpZTile + bit, c);
      c = (rem & 1u) ? cm : c;
      rem >>= 1;
    }
    for (; bit < 31 && __any(rem != 0u); bit++) {  // messages of 16 GiB and more
      const u32 cm = opmul_global(gops + kRagHighOps + 128 * (bit - kNumTileOps), c);
      c = (rem & 1u) ? cm : c;
      rem >>= 1;
    }
    if (valid) {
      if (DESC) tilecrc[tilecrc_index(w, kf + (u64)lane, nwb)] = c;  // blocked: contiguous per flush
      else atomicXor(&out[MG], c);
    }
  };

  // Prologue: table loads, then descriptors 0 and 1 and tile 0's line loads, then the LDS
  // stores and the barrier (tile 0's latency hides behind the fill).
  LdsFill<WG, kRagLdsOpWords / 128> fill;
  fill.load(gtab, gops);
  u32x4 dA, dB;
  u32 mA, mB;
  fetch_desc(0, dA, mA);
  fetch_desc(1, dB, mB);
  TileDesc dcur = unpack(dA);
  u32 mcur = mA;
  u32x4 A[8], B[8];
  load_line(dcur, A, nk != 0);
  fill.store(sbase);
  __syncthreads();
  if (nk == 0) return;

  // Ping-pong line buffers, loop unrolled by two, descriptors two tiles ahead. The body
  // has no early exit (a break between the halves would give the loop head a predecessor
  // with fewer loads in flight, and hipcc's waitcnt merge would drain the prefetch there);
  // an odd last tile, already loaded, follows the loop. The parked tiles are finished
  // whenever all 64 slots are full -- right after the next tile's loads are issued, so the
  // stores retire during that tile's compute instead of stalling the next drain
  // (crc_long.hip) -- and once more at the end.
  u64 k = 0;
  for (; k + 1 < nk; k += 2) {
    issue_prio_hi();                  // (crc_device.h)
    drain_before_issue();             // at most one tile of loads in flight (crc_uniform.hip)
    const TileDesc d1 = unpack(dB);   // tile k+1
    const u32 m1 = mB;
    fetch_desc(k + 2, dA, mA);        // tile k+2 (clamped)
    load_line(d1, B, true);
    issue_prio_lo();
    if (k && (k & 63) == 0) flush(k - 64, 64u);
    process(A, dcur, mcur, k);
    issue_prio_hi();
    drain_before_issue();
    const TileDesc d2 = unpack(dA);   // tile k+2 (clamped)
    const u32 m2 = mA;
    fetch_desc(k + 3, dB, mB);        // tile k+3 (clamped)
    load_line(d2, A, k + 2 < nk);
    issue_prio_lo();
    process(B, d1, m1, k + 1);
    dcur = d2;
    mcur = m2;
  }
  if (k < nk) {
    if (k && (k & 63) == 0) flush(k - 64, 64u);
    process(A, dcur, mcur, k);
  }
  const u64 kf = (nk - 1) & ~(u64)63;  // the last window (1..64 tiles), not flushed yet
  flush(kf, (u32)(nk - kf));
}

template <int WG>
__global__ __launch_bounds__(WG) void crc32_ragged_kernel(const uint8_t* __restrict__ base,
                                                          const u64* __restrict__ offsets, u32 ostride,
                                                          const u64* __restrict__ lengths, u32 lstride,
                                                          const u64* __restrict__ tile_base, u64 count,
                                                          const TileDesc* __restrict__ desc,
                                                          const u32* __restrict__ overflow,
                                                          const u32* __restrict__ gtab, const u32* __restrict__ gops,
                                                          HeadSeeds seeds, u32* __restrict__ out,
                                                          u32* __restrict__ tilecrc, u32 nwb, u64* scan_status,
                                                          u64 scan_words, u32* scan_ticket, FaultRef fault) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  const u32 sbase = (u32)(uintptr_t)smem;
  // the tile-count scan's state (when the fused count + descriptor kernel ran, no other kernel
  // of the call follows that scan)
  reset_scan_state(scan_status, scan_words, scan_ticket);
  if (scan_faulted(fault)) return;  // workgroup-uniform, before any barrier
  // Precomputed descriptors (8 B, or 16 B for a wide batch) unless the batch had more tiles
  // than the workspace holds (overlapping messages) or the fused kernel met a message past the
  // 8-B range; then every tile is located by binary search.
  if (overflow[0] != 0u || overflow[2] != 0u)
    ragged_body<WG, kDescSearch>(base, offsets, ostride, lengths, lstride, tile_base, count, desc, gtab, gops, seeds,
                                 out, tilecrc, nwb, sbase);
  else if (overflow[1] != 0u)
    ragged_body<WG, kDesc16>(base, offsets, ostride, lengths, lstride, tile_base, count, desc, gtab, gops, seeds, out,
                             tilecrc, nwb, sbase);
  else
    ragged_body<WG, kDesc8>(base, offsets, ostride, lengths, lstride, tile_base, count, desc, gtab, gops, seeds, out,
                            tilecrc, nwb, sbase);
}

template __global__ void crc32_ragged_kernel<512>(const uint8_t*, const u64*, u32, const u64*, u32, const u64*, u64,
                                                  const TileDesc*, const u32*, const u32*, const u32*, HeadSeeds,
                                                  u32*, u32*, u32, u64*, u64, u32*, FaultRef);

// Per message with tiles: its padded CRC = XOR of its tiles' values = P(t1 - 1) ^ P(t0 - 1)
// (P = inclusive XOR prefix of the tile values in tile order, crc_combine.hip), or the XOR
// the overflow path accumulated in out[m]; then the padding undone -- Z_p^{-1} for
// p = -(L + mis) mod 8192, as p's bits over the inverse operators Z_{2^b}^{-1} -- and the
// final XOR applied.
__global__ void crc32_ragged_final_kernel(const u64* __restrict__ tile_base, const u64* __restrict__ offsets,
                                          u32 ostride, const u64* __restrict__ lengths, u32 lstride, u64 count,
                                          const u32* __restrict__ local, const u32* __restrict__ segx, u32 nw, u32 nwb,
                                          u32* __restrict__ overflow, const u32* __restrict__ gops,
                                          u32 final_xor, u32* __restrict__ out, u64* scan_status, u64 scan_words,
                                          u32* scan_ticket, FaultRef fault) {
  reset_scan_state(scan_status, scan_words, scan_ticket);  // the segment scan is done
  // the wide flag (overflow[1], set by the tile-count scan) and the fused kernel's out-of-range
  // flag (overflow[2]): zero again for the next call (a call that faulted before this point
  // leaves them set: the next call then takes 16-B descriptors or the search, correct either way)
  if (blockIdx.x == 0 && threadIdx.x == 0) overflow[1] = overflow[2] = 0u;
  if (scan_faulted(fault)) return;
  // the padding inverses staged in LDS, per 1,024-message workgroup: the 45 nibble inverses
  // and Z_4096^{-1} (23 KiB; from global memory, up to 104 dependent lookups per message took
  // 61 us for config C, r01bu). Four steps of 8 lookups undo any padding (the 13 bit inverses:
  // 13 steps, every one taken by some lane of a wave)
  __shared__ u32 inv[(kNumNibInvOps + 1) * 128];
  for (u32 i = threadIdx.x; i < kNumNibInvOps * 128u; i += blockDim.x) inv[i] = gops[kRagNibInvOps + i];
  for (u32 i = threadIdx.x; i < 128u; i += blockDim.x) inv[kNumNibInvOps * 128 + i] = gops[kRagInvOps + 128 * 12 + i];
  __syncthreads();
  auto undo = [&](u32 slot, u32 x) {
    const u32* op = inv + 128 * slot;
    u32 r = op[x & 15u];
#pragma unroll
    for (int k = 1; k < 8; k++) r ^= op[16 * k + ((x >> (4 * k)) & 15u)];
    return r;
  };
  const bool ovf = *overflow != 0u;
  // grid-stride over the messages (the host sizes the grid: SUBSPACE_FINAL_BLOCKS_PER_CU)
  const u64 stride = (u64)gridDim.x * blockDim.x;
  for (u64 m0 = (u64)blockIdx.x * blockDim.x; m0 < count; m0 += stride) {
    const u64 m = m0 + threadIdx.x;
    const bool live = m < count;
    // every load of the message at once: its tile range, length and start
    const u64 t0 = live ? tile_base[m] : 0, t1 = live ? tile_base[m + 1] : 0;
    const u64 Lm = live ? lengths[m * lstride] : 0, sm = live ? offsets[m * ostride] : 0;
    // P(t1 - 1) of every message (empty ones included), and P(t0 - 1) = the previous message's
    // P(t1 - 1) from the neighbouring lane: one prefix gather per message instead of two (lane 0
    // gathers its own)
    const u32 pe = (!ovf && live && t1) ? tile_prefix(local, segx, nw, nwb, t1 - 1) : 0u;
    u32 pb = (u32)__shfl_up((int)pe, 1, 64);
    if ((threadIdx.x & 63u) == 0u) pb = (!ovf && live && t0) ? tile_prefix(local, segx, nw, nwb, t0 - 1) : 0u;
    if (live && t1 != t0) {  // (an empty message's result was written by the count kernel)
      u32 v = ovf ? out[m] : pe ^ pb;
      const u32 pad = (u32)(0 - (Lm + (sm & 15))) & 8191u;
#pragma unroll
      for (u32 k = 0; k < 3; k++) {
        const u32 d = (pad >> (4 * k)) & 15u;
        if (d) v = undo(15 * k + d - 1, v);
      }
      if (pad & 0x1000u) v = undo(kNumNibInvOps, v);
      out[m] = v ^ final_xor;
    }
  }
}

}  // namespace subspace_amd
