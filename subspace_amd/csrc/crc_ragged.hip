// Ragged-batch kernels: one CRC32 per message for arbitrary offsets, lengths and
// alignment (BASELINE configs C and D; any subspace_crc32_batch call).
//
// Decomposition (DESIGN.md "Ragged kernel"):
//  * Message m = bytes [s, e). Its n = ceil(L/128) "virtual lines" are aligned to the
//    message END: line g covers [e - 128(n-g), e - 128(n-1-g)). Only line 0 can start
//    before s; its r = 128n - L leading bytes are zero-masked and its lane starts from
//    zinv[r] = Z_r^{-1}(init), so after the r zero bytes the state is exactly init:
//      crc_raw(zinv[r], 0^r || D) = crc_raw(init, D).
//    Every line is a full 128-byte unit, so the combine is uniform:
//      crc(m) = XOR_g Z_{128(n-1-g)}(line_g)                       (linearity)
//  * A tile is 64 consecutive virtual lines of ONE message (end-aligned, so only a
//    message's first tile is partial). Lane i <-> line i of the tile, exactly like the
//    uniform kernel: 64 consecutive 128-B lines per wave load instruction.
//  * Waves stream the global tile list in sweep order (tau = k*nw + w), one tile of
//    loads in flight ahead. Per-tile 16-B descriptors (tile end, tiles after, first-tile
//    flag, message start offset in the first tile) are precomputed by
//    crc32_ragged_desc_kernel.
//  * Per tile, lane l of half h applies its own line-shift operator Z_{128*(31-l)} (the
//    uniform kernel's conflict-free [nibble][value][lane] tables) and a DPP reduction
//    leaves the two half-tile values in lanes 31 and 63. They are parked, one tile per
//    lane, in registers (lane k&63 keeps tile k); every 64 tiles each lane finishes its own tile,
//      tile value = Z_{8192*T}( Z_4096(half0) ^ half1 )     (T = tiles after it)
//    with a per-lane binary decomposition of T over nibble operators -- one wave pass
//    shifts 64 tiles -- and stores tilecrc[tau]. A message's CRC is the XOR of its tiles'
//    values, i.e. the difference of two entries of the inclusive XOR-scan of tilecrc
//    (crc32_ragged_final_kernel). No atomics: huge messages (config D: 8192 tiles each,
//    all in flight at once) would otherwise serialise every tile on one output word.
//    (Batches whose tiles overflow the workspace -- overlapping messages -- fall back to
//    atomicXor into pre-zeroed words.)
//  * End-aligned lines are 16-B misaligned when e is. Each lane loads the 8 aligned 16-B
//    blocks starting at or below its line; the line's last e&15 bytes sit in the next
//    lane's first block, which arrives by a DPP wave shift, and for lane 63 in the tile's
//    last (partial) block, one load shared by the whole wave. The words are realigned
//    with v_alignbyte_b32 (the dword shift (e&15)>>2 is wave-uniform: a 4-way uniform
//    switch). Loads never touch a 16-B block that holds no message byte.
#include <hipcub/hipcub.hpp>

#include "crc_device.h"

namespace subspace_amd {

// 16 B per tile: one vector load and four readfirstlanes per tile in the main kernel.
struct TileDesc {
  u64 tile_end;  // absolute offset (from base) one past the tile's last byte
  u32 after;     // tiles after this one in the message | kFirstTile for its first tile
  u32 lead;      // first tile: message start - tile start (0..8191), else 0
};
static_assert(sizeof(TileDesc) == 16, "TileDesc is 16 B");
constexpr u32 kFirstTile = 0x80000000u;

__host__ __device__ inline u64 tiles_for_length(u64 len) { return (len + 8191) >> 13; }

// Per message: tile count; zero-length messages get their (constant) result here,
// multi-tile messages get their output word zeroed for the tiles' atomicXor.
// `lengths` (and `offsets` below) are read with an element stride (1 for plain arrays, 3 for
// the lengths/payload fields of subspace_crc_slot records).
__global__ void crc32_ragged_count_kernel(const u64* __restrict__ lengths, u32 lstride, u64 count, u32 init,
                                          u32 final_xor, u64* __restrict__ ntiles, u32* __restrict__ out) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i > count) return;
  if (i == count) {
    ntiles[i] = 0;  // scan sentinel: tile_base[count] = total tiles
    return;
  }
  const u64 len = lengths[i * lstride];
  const u64 nt = tiles_for_length(len);
  ntiles[i] = nt;
  if (nt == 0) out[i] = init ^ final_xor;
  else if (nt > 1) out[i] = 0u;
}

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

__device__ inline TileDesc make_desc(const u64* __restrict__ offsets, u32 ostride, const u64* __restrict__ lengths,
                                     u32 lstride, const u64* __restrict__ tile_base, u64 m, u64 tau) {
  const u64 nt = tile_base[m + 1] - tile_base[m];
  const u64 j = tau - tile_base[m];
  const u64 s = offsets[m * ostride];
  const u64 e = s + lengths[m * lstride];
  TileDesc d;
  d.tile_end = e - ((nt - 1 - j) << 13);
  d.after = (u32)(nt - 1 - j) | (j == 0 ? kFirstTile : 0u);
  // first tile: the message starts `lead` bytes into it; the line holding byte s is line
  // lead >> 7 and starts r = lead & 127 bytes before s (lines are end-aligned), so its lane
  // starts from zinv[r]
  d.lead = j == 0 ? (u32)((i64)s - ((i64)d.tile_end - 8192)) : 0u;
  return d;
}

// Per tile (up to `capacity`): its descriptor. Sets *overflow if the batch has more tiles.
__global__ void crc32_ragged_desc_kernel(const u64* __restrict__ offsets, u32 ostride,
                                         const u64* __restrict__ lengths, u32 lstride,
                                         const u64* __restrict__ tile_base, u64 count, u64 capacity,
                                         TileDesc* __restrict__ desc, u32* __restrict__ overflow) {
  const u64 total = tile_base[count];
  const u64 tau = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (tau == 0) *overflow = total > capacity ? 1u : 0u;
  if (tau >= total || tau >= capacity) return;
  desc[tau] = make_desc(offsets, ostride, lengths, lstride, tile_base, find_msg(tile_base, count, tau), tau);
}

// ------------------------------------------------------------------ main kernel
struct LineState {
  u32x4 d[8];  // the 8 aligned 16-B blocks starting at or below the lane's line
  u32x4 x;     // the tile's last aligned block (the same for every lane)
};

template <int Q>
__device__ __forceinline__ u32 word_at(const u32x4 (&d)[9], int j, u32 m3) {
  // word j of the realigned line: bytes [4(j+Q) + m3, +4) of the aligned window
  const int x = j + Q;
  const u32 lo = d[x >> 2][x & 3];
  const u32 hi = d[(x + 1) >> 2][(x + 1) & 3];
  return __builtin_amdgcn_alignbyte(hi, lo, m3);
}

template <int Q, bool MIS>
__device__ __forceinline__ u32 crc_line(const u32x4 (&d)[9], u32 crc, u32 m3, u32 lc0, u32 lc1) {
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const u32 w = MIS ? word_at<Q>(d, j, m3) : d[j >> 2][j & 3];
    crc = step4(crc ^ w, lc0, lc1);
  }
  return crc;
}

// Nibble operator read from global memory (the tile-shift operators for 2^21 tiles and
// more, which only messages of 16 GiB and more need).
__device__ __forceinline__ u32 opmul_global(const u32* __restrict__ op, u32 v) {
  u32 r = op[v & 15u];
#pragma unroll
  for (int k = 1; k < 8; k++) r ^= op[16 * k + ((v >> (4 * k)) & 15u)];
  return r;
}

template <int WG, bool DESC>
__device__ __forceinline__ void ragged_body(const uint8_t* __restrict__ base, const u64* __restrict__ offsets,
                                            u32 ostride, const u64* __restrict__ lengths, u32 lstride,
                                            const u64* __restrict__ tile_base, u64 count,
                                            const TileDesc* __restrict__ desc, const u32* __restrict__ gtab,
                                            const u32* __restrict__ gops, const u32* __restrict__ zinv,
                                            u32 final_xor, u32* __restrict__ out, u32* __restrict__ tilecrc,
                                            u32 sbase) {
  const int lane = threadIdx.x & 63;
  const u32 wid = rfl(threadIdx.x >> 6);
  const u32 lc0 = sbase + ((u32)(lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  const u32 lop = sbase + kLdsOps + 4u * (u32)(31 - (lane & 31));  // this lane's line-shift operator
  const u32 zsb = sbase + kRagZinv;  // zinv[r], r = 0..127 (first-line seeds of this batch's init)
  const u64 total = tile_base[count];
  const u64 w = front_slot(blockIdx.x, gridDim.x, wid);  // sweep front slot (crc_device.h)
  const u64 nw = (u64)gridDim.x * (WG / 64);
  const u64 nk = w < total ? (total - w + nw - 1) / nw : 0;  // tiles tau = k*nw + w, k < nk
  if (total == 0) return;  // every message empty: all waves of all blocks leave before any load
  // An opaque zero in a VGPR: descriptor loads indexed with it are vector loads, so they
  // retire in order with the line loads (vmcnt) instead of coupling with LDS (lgkmcnt).
  u32 vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));

  // Descriptor of tile k as raw dwords (a vector load; DESC false: built by search, with
  // the message id for the atomic path). Past the wave's last tile it is clamped to that
  // tile; a wave without tiles uses the batch's last tile, so every load the kernel issues
  // stays inside a real message.
  auto fetch_desc = [&](u64 k, u32x4& d, u32& dm) {
    const u64 tau = nk ? (k < nk ? k : nk - 1) * nw + w : total - 1;
    if (DESC) {
      d = *reinterpret_cast<const u32x4*>(desc + tau + vzero);
      dm = 0;
    } else {
      const u64 m = find_msg(tile_base, count, tau);
      const TileDesc t = make_desc(offsets, ostride, lengths, lstride, tile_base, m, tau);
      d = u32x4{(u32)t.tile_end, (u32)(t.tile_end >> 32), t.after, t.lead};
      dm = (u32)m;
    }
  };
  auto unpack = [&](const u32x4& d) {
    TileDesc t;
    t.tile_end = rfl64(d[0], d[1]);
    t.after = rfl(d[2]);
    t.lead = rfl(d[3]);
    return t;
  };
  // Issue the loads of tile d, as buffer loads against a scalar resource spanning exactly
  // the tile's blocks that hold message bytes:
  //   [max(aligned tile start, aligned message start), tile end rounded up to 16).
  // Lane l loads the 8 blocks from a - 128*(64-l) (a = tile end rounded down to 16); blocks
  // before the range start (before the message) read as zeros without touching memory (a
  // per-lane offset below the start wraps to a huge value), so every lane issues every
  // load (no divergent branch around loads). The 9th load is the same for all lanes: the
  // tile's last block [a, a+16) when the end is misaligned (it is inside the range), else
  // the dummy [a-16, a). `live` false (a prefetch past the wave's last tile) gives an
  // empty range.
  auto load_line = [&](const TileDesc& d, LineState& L, bool live) {
    const i64 tile_start = (i64)d.tile_end - 8192;
    const i64 t0a = tile_start & ~(i64)15;
    const i64 rb = (d.after & kFirstTile) ? ((tile_start + (i64)d.lead) & ~(i64)15) : t0a;
    const i64 a = (i64)d.tile_end & ~(i64)15;
    const i64 rend = ((i64)d.tile_end + 15) & ~(i64)15;
    const u32 nrec = live ? (u32)(rend - rb) : 0u;
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base + rb), (short)0, (int)nrec,
                                                     kBufferRsrcFlags);
    const u32 vo = (u32)lane * 128u - (u32)(rb - t0a);
#pragma unroll
    for (int b = 0; b < 8; b++) L.d[b] = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 16u * b, 0, 0);
    // the shared block's offset goes in the VGPR (not the scalar offset), so the range
    // check sees it whichever offsets the hardware includes
    const u32 xo = vzero + (u32)((rend > a ? a : a - 16) - rb);
    L.x = __builtin_amdgcn_raw_buffer_load_b128(r, xo, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };

  // Half-tile values parked one tile per lane (slot k & 63), finished every 64 tiles.
  u32 H0 = 0, H1 = 0, AF = 0, MG = 0;  // half 0, half 1, after | kFirstTile, message (DESC false)

  auto process = [&](const LineState& cur, const TileDesc& dcur, u32 dm, u64 k) {
    const bool first = (dcur.after & kFirstTile) != 0;  // wave-uniform, like everything below
    const u32 mis = (u32)(dcur.tile_end & 15);
    u32x4 d[9];
#pragma unroll
    for (int b = 0; b < 8; b++) d[b] = cur.d[b];
    if (mis) {  // lane l's 9th block is lane l+1's first, lane 63's the shared one
#pragma unroll
      for (int x = 0; x < 4; x++)
        d[8][x] = (u32)__builtin_amdgcn_update_dpp((int)cur.x[x], (int)cur.d[0][x], 0x130, 0xF, 0xF, false);
    } else {
      d[8] = u32x4{0u, 0u, 0u, 0u};
    }
    u32 crc = 0;
    if (first) {
      // The message starts `lead` bytes into the tile: zero every byte of each lane's 144-B
      // window below it (the window starts lead + mis - 128*lane bytes before the message),
      // and start the lane holding the first byte from zinv[lead & 127]. Lanes wholly
      // before the message then compute crc_raw(0, zeros) = 0.
      const u32 lead = dcur.lead;
      if (lead) {
        const int zb0 = (int)(lead + mis) - 128 * lane;
        const u32 zb = zb0 <= 0 ? 0u : (zb0 >= 144 ? 144u : (u32)zb0);
#pragma unroll
        for (int b = 0; b < 9; b++) {
#pragma unroll
          for (int x = 0; x < 4; x++) {
            const u32 p = 16u * b + 4u * x;
            u32 keep = 0xFFFFFFFFu;
            if (p + 4u <= zb) keep = 0;
            else if (p < zb) keep = 0xFFFFFFFFu << (8u * (zb - p));
            d[b][x] &= keep;
          }
        }
      }
      const u32 seed = lds_ld(zsb + 4u * (lead & 127u));
      crc = (u32)lane == (lead >> 7) ? seed : 0u;
    }
    const u32 m3 = mis & 3;
    switch (mis >> 2) {
      case 0: crc = mis ? crc_line<0, true>(d, crc, m3, lc0, lc1) : crc_line<0, false>(d, crc, m3, lc0, lc1); break;
      case 1: crc = crc_line<1, true>(d, crc, m3, lc0, lc1); break;
      case 2: crc = crc_line<2, true>(d, crc, m3, lc0, lc1); break;
      default: crc = crc_line<3, true>(d, crc, m3, lc0, lc1); break;
    }

    // line l of half h -> Z_{128*(31-l)}(line): 8 conflict-free nibble lookups; then XOR
    // over each half with DPP (lane 31: lines 0..31, lane 63: lines 32..63)
    u32 v = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) v ^= lds_ld(lop + 2048u * j + (((crc >> (4 * j)) & 15u) << 7));
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
    u32 rem = valid ? (AF & ~kFirstTile) : 0u;   // shift to the message end: Z_{8192 * after}
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
    if (AF & kFirstTile) c ^= final_xor;
    if (valid) {
      if (DESC) {
        tilecrc[(kf + (u64)lane) * nw + w] = c;
      } else if (AF == kFirstTile) {
        out[MG] = c;  // single-tile message
      } else {
        atomicXor(&out[MG], c);
      }
    }
  };

  // Prologue: table loads, then descriptors 0 and 1 and tile 0's line loads, then the LDS
  // stores and the barrier (tile 0's latency hides behind the fill).
  LdsFill<WG, kRagLdsOpWords / 128> fill;
  fill.load(gtab, gops);
  const u32 zv = zinv[threadIdx.x & 127];  // unconditional (a load in a branch drains vmcnt)
  u32x4 dA, dB;
  u32 mA, mB;
  fetch_desc(0, dA, mA);
  fetch_desc(1, dB, mB);
  TileDesc dcur = unpack(dA);
  u32 mcur = mA;
  LineState A, B;
  load_line(dcur, A, nk != 0);
  fill.store(sbase);
  if (threadIdx.x < 128) lds_st(zsb + 4u * threadIdx.x, zv);
  asm volatile("" ::"v"(zv));
  __syncthreads();
  if (nk == 0) return;

  // Ping-pong line buffers, loop unrolled by two, descriptors two tiles ahead. The body
  // has no early exit (a break between the halves would give the loop head a predecessor
  // with fewer loads in flight, and hipcc's waitcnt merge would drain the prefetch there);
  // an odd last tile, already loaded, follows the loop. The parked tiles are finished
  // whenever all 64 slots are full, and once more at the end.
  u64 k = 0;
  for (; k + 1 < nk; k += 2) {
    drain_before_issue();             // at most one tile of loads in flight (crc_uniform.hip)
    const TileDesc d1 = unpack(dB);   // tile k+1
    const u32 m1 = mB;
    fetch_desc(k + 2, dA, mA);        // tile k+2 (clamped)
    load_line(d1, B, true);
    process(A, dcur, mcur, k);
    drain_before_issue();
    const TileDesc d2 = unpack(dA);   // tile k+2 (clamped)
    const u32 m2 = mA;
    fetch_desc(k + 3, dB, mB);        // tile k+3 (clamped)
    load_line(d2, A, k + 2 < nk);
    process(B, d1, m1, k + 1);
    dcur = d2;
    mcur = m2;
    if (((k + 2) & 63) == 0) flush(k + 2 - 64, 64u);
  }
  if (k < nk) process(A, dcur, mcur, k);
  const u64 kf = nk & ~(u64)63;
  if (nk > kf) flush(kf, (u32)(nk - kf));
}

template <int WG>
__global__ __launch_bounds__(WG) void crc32_ragged_kernel(const uint8_t* __restrict__ base,
                                                          const u64* __restrict__ offsets, u32 ostride,
                                                          const u64* __restrict__ lengths, u32 lstride,
                                                          const u64* __restrict__ tile_base, u64 count,
                                                          const TileDesc* __restrict__ desc,
                                                          const u32* __restrict__ overflow,
                                                          const u32* __restrict__ gtab, const u32* __restrict__ gops,
                                                          const u32* __restrict__ zinv, u32 final_xor,
                                                          u32* __restrict__ out, u32* __restrict__ tilecrc) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  const u32 sbase = (u32)(uintptr_t)smem;
  // Precomputed descriptors unless the batch had more tiles than the workspace holds
  // (overlapping messages); then every tile is located by binary search.
  if (*overflow == 0u)
    ragged_body<WG, true>(base, offsets, ostride, lengths, lstride, tile_base, count, desc, gtab, gops, zinv,
                          final_xor, out, tilecrc, sbase);
  else
    ragged_body<WG, false>(base, offsets, ostride, lengths, lstride, tile_base, count, desc, gtab, gops, zinv,
                           final_xor, out, tilecrc, sbase);
}

template __global__ void crc32_ragged_kernel<512>(const uint8_t*, const u64*, u32, const u64*, u32, const u64*, u64,
                                                  const TileDesc*, const u32*, const u32*, const u32*, const u32*,
                                                  u32, u32*, u32*);

// Per message with tiles: out[m] = XOR of its tiles' values = px[last] ^ px[first - 1],
// px = inclusive XOR-scan of tilecrc. Skipped when the batch overflowed the workspace
// (those results were produced with atomics).
__global__ void crc32_ragged_final_kernel(const u64* __restrict__ tile_base, u64 count, const u32* __restrict__ px,
                                          const u32* __restrict__ overflow, u32* __restrict__ out) {
  const u64 m = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= count || *overflow) return;
  const u64 t0 = tile_base[m], t1 = tile_base[m + 1];
  if (t1 == t0) return;  // empty message: written by the count kernel
  out[m] = px[t1 - 1] ^ (t0 ? px[t0 - 1] : 0u);
}

// hipcub scan wrappers: exclusive prefix sum of per-message tile counts; inclusive XOR
// scan of per-tile values.
hipError_t ragged_scan(void* temp, size_t& temp_bytes, const u64* in, u64* out, u64 n, hipStream_t stream) {
  return hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, in, out, (int)n, stream);
}

struct XorOp {
  __host__ __device__ u32 operator()(u32 a, u32 b) const { return a ^ b; }
};

hipError_t xor_scan(void* temp, size_t& temp_bytes, const u32* in, u32* out, u64 n, hipStream_t stream) {
  return hipcub::DeviceScan::InclusiveScan(temp, temp_bytes, in, out, XorOp(), (int)n, stream);
}

}  // namespace subspace_amd
