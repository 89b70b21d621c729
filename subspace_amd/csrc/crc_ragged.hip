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
//    loads in flight ahead. Per-tile descriptors (tile end, message start, message id,
//    tiles after) are precomputed by crc32_ragged_desc_kernel.
//  * Every 4 tiles the 256 line CRCs are transposed through LDS (16 lanes per tile),
//    tree-combined (Z_128..Z_4096), multiplied by Z_{8192*T} (T = tiles after this one
//    in the message, binary decomposition over nibble operators) and stored per tile:
//    tilecrc[tau]. A message's CRC is the XOR of its tiles' values, i.e. the difference of
//    two entries of the inclusive XOR-scan of tilecrc (crc32_ragged_final_kernel). No
//    atomics: huge messages (config D: 8192 tiles each, all in flight at once) would
//    otherwise serialise every tile on one output word.
//    (Batches whose tiles overflow the workspace -- overlapping messages -- fall back to
//    atomicXor into pre-zeroed words.)
//  * End-aligned lines are 16-B misaligned when e is: each lane then loads the 9
//    aligned 16-B blocks covering its line and realigns with v_alignbyte_b32 (the
//    dword shift e&15 >> 2 is wave-uniform, so it is a 4-way uniform switch).
//    Loads never touch a 16-B block that contains no message byte, so nothing outside
//    the messages' own aligned blocks is read.
#include <hipcub/hipcub.hpp>

#include "crc_device.h"

namespace subspace_amd {

struct TileDesc {
  u64 tile_end;   // absolute offset (from base) one past the tile's last byte
  u64 msg_start;  // offset of the message's first byte
  u32 msg;        // message index
  u32 after;      // tiles after this one in the message
  u32 seed;       // first tile only: zinv[r], the start state of the line holding msg_start
  u32 pad;
};
static_assert(sizeof(TileDesc) == 32, "TileDesc is 32 B");

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
                                     u32 lstride, const u64* __restrict__ tile_base, const u32* __restrict__ zinv,
                                     u64 m, u64 tau) {
  const u64 nt = tile_base[m + 1] - tile_base[m];
  const u64 j = tau - tile_base[m];
  const u64 s = offsets[m * ostride];
  const u64 e = s + lengths[m * lstride];
  TileDesc d;
  d.tile_end = e - ((nt - 1 - j) << 13);
  d.msg_start = s;
  d.msg = (u32)m;
  d.after = (u32)(nt - 1 - j);
  // the line holding byte s starts r = (s - tile_start) mod 128 bytes before it (lines are
  // end-aligned, so tile_start == e - 8192*(nt-j) and r only depends on e - s mod 128)
  const i64 tile_start = (i64)d.tile_end - 8192;
  const u64 r = (u64)((i64)s - tile_start) & 127u;
  d.seed = j == 0 ? zinv[r] : 0u;
  d.pad = 0;
  return d;
}

// Per tile (up to `capacity`): its descriptor. Sets *overflow if the batch has more tiles.
__global__ void crc32_ragged_desc_kernel(const u64* __restrict__ offsets, u32 ostride,
                                         const u64* __restrict__ lengths, u32 lstride,
                                         const u64* __restrict__ tile_base, const u32* __restrict__ zinv, u64 count,
                                         u64 capacity, TileDesc* __restrict__ desc, u32* __restrict__ overflow) {
  const u64 total = tile_base[count];
  const u64 tau = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (tau == 0) *overflow = total > capacity ? 1u : 0u;
  if (tau >= total || tau >= capacity) return;
  desc[tau] = make_desc(offsets, ostride, lengths, lstride, tile_base, zinv, find_msg(tile_base, count, tau), tau);
}

// ------------------------------------------------------------------ main kernel
struct LineState {
  u32x4 d[9];  // aligned 16-B blocks covering the lane's line (9th only when misaligned)
};

template <int Q>
__device__ __forceinline__ u32 word_at(const LineState& L, int j, u32 m3) {
  // word j of the realigned line: bytes [4(j+Q) + m3, +4) of the aligned window
  const int x = j + Q;
  const u32 lo = L.d[x >> 2][x & 3];
  const u32 hi = L.d[(x + 1) >> 2][(x + 1) & 3];
  return __builtin_amdgcn_alignbyte(hi, lo, m3);
}

template <int Q, bool MIS>
__device__ __forceinline__ u32 crc_line(const LineState& L, u32 crc, u32 m3, u32 lc0, u32 lc1) {
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const u32 w = MIS ? word_at<Q>(L, j, m3) : L.d[j >> 2][j & 3];
    crc = step4(crc ^ w, lc0, lc1);
  }
  return crc;
}

template <int WG, bool DESC>
__device__ __forceinline__ void ragged_body(const uint8_t* __restrict__ base,
                                                          const u64* __restrict__ offsets, u32 ostride,
                                                          const u64* __restrict__ lengths, u32 lstride,
                                                          const u64* __restrict__ tile_base, u64 count,
                                                          const TileDesc* __restrict__ desc,
                                                          const u32* __restrict__ overflow,
                                                          const u32* __restrict__ gtab, const u32* __restrict__ gops,
                                                          const u32* __restrict__ zinv, u32 final_xor,
                                                          u32* __restrict__ out, u32* __restrict__ tilecrc,
                                                          u32 sbase) {
  const int lane = threadIdx.x & 63;
  const u32 wid = rfl(threadIdx.x >> 6);
  const u32 lc0 = sbase + ((u32)(lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  const u32 xb = sbase + kLdsXpose + wid * kLdsXposePerWave;
  const u64 total = tile_base[count];
  const u64 w = front_slot(blockIdx.x, gridDim.x, wid);  // sweep front slot (crc_device.h)
  const u64 nw = (u64)gridDim.x * (WG / 64);
  const u64 nk = w < total ? (total - w + nw - 1) / nw : 0;  // tiles tau = k*nw + w, k < nk
  if (total == 0) return;  // every message empty: all waves of all blocks leave before any load
  // An opaque zero in a VGPR: descriptor loads indexed with it are vector loads, so they
  // retire in order with the line loads (vmcnt) instead of coupling with LDS (lgkmcnt).
  u32 vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));

  // Descriptor of tile k as raw dwords (a vector load). Past the wave's last tile it is
  // clamped to that tile; a wave without tiles uses the batch's last tile, so every load
  // the kernel issues stays inside a real message.
  auto fetch_desc = [&](u64 k, u32x4 (&d)[2]) {
    const u64 tau = nk ? (k < nk ? k : nk - 1) * nw + w : total - 1;
    if (DESC) {
      const u32x4* p = reinterpret_cast<const u32x4*>(desc + tau + vzero);
      d[0] = p[0];
      d[1] = p[1];
    } else {
      const TileDesc t =
          make_desc(offsets, ostride, lengths, lstride, tile_base, zinv, find_msg(tile_base, count, tau), tau);
      d[0] = u32x4{(u32)t.tile_end, (u32)(t.tile_end >> 32), (u32)t.msg_start, (u32)(t.msg_start >> 32)};
      d[1] = u32x4{t.msg, t.after, t.seed, 0u};
    }
  };
  auto unpack = [&](const u32x4 (&d)[2]) {
    TileDesc t;
    t.tile_end = rfl64(d[0][0], d[0][1]);
    t.msg_start = rfl64(d[0][2], d[0][3]);
    t.msg = rfl(d[1][0]);
    t.after = rfl(d[1][1]);
    t.seed = rfl(d[1][2]);
    t.pad = 0;
    return t;
  };
  // Issue the loads of this lane's line for tile descriptor d, as buffer loads against a
  // scalar resource spanning exactly the tile's blocks that hold message bytes:
  //   [max(aligned tile start, aligned message start), tile end rounded up to 16).
  // Blocks outside it (before the message, or an aligned line's 9th block) read as zeros
  // without touching memory, so every lane issues all 9 loads (no divergent branch around
  // loads) and nothing outside the message's own blocks is ever read. A per-lane offset
  // below the range start wraps to a huge value: out of range as well. `live` false (a
  // prefetch past the wave's last tile) gives an empty range.
  auto load_line = [&](const TileDesc& d, LineState& L, bool live) {
    const i64 t0a = ((i64)d.tile_end - 8192) & ~(i64)15;
    const i64 sa = (i64)d.msg_start & ~(i64)15;
    const i64 rb = t0a > sa ? t0a : sa;
    const i64 rend = ((i64)d.tile_end + 15) & ~(i64)15;
    const u32 nrec = live ? (u32)(rend - rb) : 0u;
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base + rb), (short)0, (int)nrec,
                                                     kBufferRsrcFlags);
    const u32 vo = (u32)lane * 128u - (u32)(rb - t0a);
#pragma unroll
    for (int b = 0; b < 8; b++) L.d[b] = __builtin_amdgcn_raw_buffer_load_b128(r, vo + 16u * b, 0, 0);
    // The 9th block of an aligned tile's last line starts exactly at the range end; its
    // offset goes in the VGPR (not folded into the instruction offset), so the range check
    // sees it whichever offsets the hardware includes.
    u32 vo8;
    asm volatile("v_add_u32 %0, 0x80, %1" : "=v"(vo8) : "v"(vo));
    L.d[8] = __builtin_amdgcn_raw_buffer_load_b128(r, vo8, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };

  u32 part[4] = {0, 0, 0, 0};
  u32 gmsg[4] = {0, 0, 0, 0}, gafter[4] = {0, 0, 0, 0};
  u32 gfirst = 0;  // bit t: tile t of the group is its message's first tile

  auto process = [&](LineState& cur, const TileDesc& dcur, u64 k) {
    const i64 tile_start = (i64)dcur.tile_end - 8192;
    const i64 line_start = tile_start + (i64)lane * 128;
    const i64 s = (i64)dcur.msg_start;
    const bool partial = tile_start < s;  // wave-uniform
    const bool active = line_start + 128 > s;
    u32 crc;
    if (partial) {
      // zero every byte below the message start (this also clears redirected blocks),
      // seed the first line with zinv[r]
      const i64 a0 = line_start & ~(i64)15;
#pragma unroll
      for (int b = 0; b < 9; b++) {
#pragma unroll
        for (int x = 0; x < 4; x++) {
          const i64 addr = a0 + 16 * b + 4 * x;
          u32 keep = 0xFFFFFFFFu;
          if (addr + 4 <= s) keep = 0;
          else if (addr < s) keep = 0xFFFFFFFFu << (8 * (u32)(s - addr));
          cur.d[b][x] &= keep;
        }
      }
    }
    // the line holding the message's first byte starts from zinv[r] (precomputed seed)
    crc = (active && line_start <= s) ? dcur.seed : 0u;
    const u32 mis = (u32)(dcur.tile_end & 15);
    const u32 m3 = mis & 3;
    switch (mis >> 2) {  // wave-uniform
      case 0: crc = mis ? crc_line<0, true>(cur, crc, m3, lc0, lc1) : crc_line<0, false>(cur, crc, m3, lc0, lc1); break;
      case 1: crc = crc_line<1, true>(cur, crc, m3, lc0, lc1); break;
      case 2: crc = crc_line<2, true>(cur, crc, m3, lc0, lc1); break;
      default: crc = crc_line<3, true>(cur, crc, m3, lc0, lc1); break;
    }
    if (!active) crc = 0;

    const int t = (int)(k & 3);
    // static-index stores keep part[] / gmsg[] / gafter[] in registers
#pragma unroll
    for (int tt = 0; tt < 4; tt++)
      if (tt == t) {
        part[tt] = crc;
        gmsg[tt] = dcur.msg;
        gafter[tt] = dcur.after;
      }
    gfirst = (partial || tile_start == s) ? (gfirst | (1u << t)) : (gfirst & ~(1u << t));

    if (t == 3 || k + 1 == nk) {
#pragma unroll
      for (int tt = 0; tt < 4; tt++) lds_st(xb + tt * 256 + lane * 4, part[tt]);
      wave_lds_sync();
      const int T = lane >> 4, q = lane & 15;
      const u32x4 sv = lds_ld4(xb + T * 256 + q * 16);  // lines 4q..4q+3 of group tile T
      const u32 a = opmul(sbase, kOpZ128 + 0, sv[0]) ^ sv[1];
      const u32 b = opmul(sbase, kOpZ128 + 0, sv[2]) ^ sv[3];
      u32 c = opmul(sbase, kOpZ128 + 1, a) ^ b;               // 512 B
      c = opmul(sbase, kOpZ128 + 2, c) ^ __shfl_down(c, 1);   // 1 KiB
      c = opmul(sbase, kOpZ128 + 3, c) ^ __shfl_down(c, 2);   // 2 KiB
      c = opmul(sbase, kOpZ128 + 4, c) ^ __shfl_down(c, 4);   // 4 KiB
      c = opmul(sbase, kOpZ128 + 5, c) ^ __shfl_down(c, 8);   // 8 KiB: tile result at q == 0
      const bool valid = (u64)T <= (u64)t;                     // group slot holds a tile
      u32 after = 0, msg = 0;
#pragma unroll
      for (int tt = 0; tt < 4; tt++)
        if (tt == T) { after = gafter[tt]; msg = gmsg[tt]; }
      // shift to the message end: Z_{8192 * after}, binary decomposition (wave-uniform loop)
      u32 rem = (q == 0 && valid) ? after : 0u;
      for (int bit = 0; bit < kNumTileOps && __any(rem != 0u); bit++) {
        const u32 cm = opmul(sbase, kOpZTile + bit, c);
        c = (rem & 1u) ? cm : c;
        rem >>= 1;
      }
      if (q == 0 && valid) {
        const bool first = (gfirst >> T) & 1u;
        const u32 contrib = first ? (c ^ final_xor) : c;
        if (DESC) {
          tilecrc[((k & ~(u64)3) + (u64)T) * nw + w] = contrib;  // tile tau of group slot T
        } else if (first && after == 0) {
          out[msg] = contrib;  // single-tile message
        } else {
          atomicXor(&out[msg], contrib);
        }
      }
      wave_lds_sync();
    }
  };

  // Prologue: table loads, then descriptors 0 and 1 and tile 0's line loads, then the LDS
  // stores and the barrier (tile 0's latency hides behind the fill).
  LdsFill<WG, kOpZTile + kNumTileOps> fill;
  fill.load(gtab, gops);
  u32x4 dA[2], dB[2];
  fetch_desc(0, dA);
  fetch_desc(1, dB);
  TileDesc dcur = unpack(dA);
  LineState A, B;
  load_line(dcur, A, nk != 0);
  fill.store(sbase);
  __syncthreads();
  if (nk == 0) return;

  // Ping-pong line buffers, loop unrolled by two, descriptors two tiles ahead. The body
  // has no early exit (a break between the halves would give the loop head a predecessor
  // with fewer loads in flight, and hipcc's waitcnt merge would drain the prefetch there);
  // an odd last tile, already loaded, follows the loop.
  u64 k = 0;
  for (; k + 1 < nk; k += 2) {
    const TileDesc d1 = unpack(dB);   // tile k+1
    fetch_desc(k + 2, dA);            // tile k+2 (clamped)
    load_line(d1, B, true);
    process(A, dcur, k);
    const TileDesc d2 = unpack(dA);   // tile k+2 (clamped)
    fetch_desc(k + 3, dB);            // tile k+3 (clamped)
    load_line(d2, A, k + 2 < nk);
    process(B, d1, k + 1);
    dcur = d2;
  }
  if (k < nk) process(A, dcur, k);
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
    ragged_body<WG, true>(base, offsets, ostride, lengths, lstride, tile_base, count, desc, overflow, gtab, gops, zinv,
                          final_xor, out, tilecrc, sbase);
  else
    ragged_body<WG, false>(base, offsets, ostride, lengths, lstride, tile_base, count, desc, overflow, gtab, gops,
                           zinv, final_xor, out, tilecrc, sbase);
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
