// Fixed-size batch kernel: one CRC32 per 4 KiB message (BASELINE configs B and E).
//
// Work decomposition (DESIGN.md "Uniform kernel"):
//  * A tile is 2 messages = 64 lines of 128 B. Lane l of half h (h = lane >> 5)
//    owns line l of message 2*tau + h, so every wave load instruction touches 64
//    consecutive 128-B lines (the access shape measured near the coalesced HBM rate
//    on MI355X; lane-contiguous 1 KiB chunks ran ~40 % slower).
//  * Each wave streams tiles tau = k*nw + w (all waves sweep one compact front) and
//    always has the next tile's 8 loads in flight while it computes the current one.
//  * Per line: 32 slice-by-4 steps from 32-way replicated LDS tables (4 conflict-free
//    ds_read_b32 + 4 v_perm + 4 v_xor per word).
//  * Every 4 tiles the wave holds line CRCs of 8 messages (crc_raw(0, line), or with
//    the batch init for line 0). They are transposed through LDS so lane j holds 4
//    consecutive lines of message j>>3, combined in-lane (Z_128, Z_256) and across 8
//    lanes (Z_512, Z_1024, Z_2048) with nibble-table GF(2) operators:
//      crc(msg) = XOR_i Z_{128*(31-i)}(line_i)     (crc_raw linearity)
#include "crc_device.h"

namespace subspace_amd {

template <int WG, int DEPTH>
__global__ __launch_bounds__(WG) void crc32_uniform4k_kernel(const uint8_t* __restrict__ base, u64 stride, u64 count,
                                                             const u32* __restrict__ gtab, const u32* __restrict__ gops,
                                                             u32 init, u32 final_xor, u32* __restrict__ out,
                                                             int order) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  const u32 sbase = (u32)(uintptr_t)smem;

  const int lane = threadIdx.x & 63;
  // wave-uniform (SGPR) wave index: keeps the tile loop a scalar loop, so hipcc's waitcnt
  // bookkeeping stays exact (a divergent loop makes it drain the prefetch every iteration)
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lc0 = sbase + ((u32)(lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  const u32 xb = sbase + kLdsXpose + (u32)wid * kLdsXposePerWave;
  const int l = lane & 31, h = lane >> 5;
  const u64 ntiles = (count + 1) >> 1;
  // Tile order. Sweep (orders 0 and 2): tau = k*nw + w, all waves advance one compact
  // front. The front position w of a wave: order 0 gives consecutive 16 KiB pairs of tiles
  // to consecutive workgroups, w = (b + G*(wid/2))*2 + wid%2 -- so every XCD (block b runs
  // on XCD b%8) streams from everywhere in the front (tools/ubench/streamread.hip:
  // lines_remap sub2, 6.6 vs 6.0 TB/s for one 256 MiB launch); order 2 gives a workgroup
  // its wpb consecutive tiles, w = b*wpb + wid.
  // Order 1 ("region"): workgroup b owns the contiguous tiles [b*per, (b+1)*per), its waves
  // interleave inside it: tau = b*per + k*wpb + wid.
  constexpr u64 wpb = WG / 64;
  const u64 nw = (u64)gridDim.x * wpb;
  u64 t0, tstep, tend;
  if (order == 0) {
    t0 = front_slot(blockIdx.x, gridDim.x, (u32)wid);
    tstep = nw;
    tend = ntiles;
  } else if (order == 2) {
    t0 = (u64)blockIdx.x * wpb + (u64)wid;
    tstep = nw;
    tend = ntiles;
  } else {
    const u64 per = (ntiles + gridDim.x - 1) / gridDim.x;
    const u64 b0 = (u64)blockIdx.x * per;
    t0 = b0 + (u64)wid;
    tstep = wpb;
    tend = b0 + per < ntiles ? b0 + per : ntiles;
  }
  // waves beyond the work still help fill LDS, then leave (no later block barrier)
  // this wave's tiles: tau = t0 + k*tstep, k < nk. 32-bit tile counters keep the loop
  // control scalar (a 64-bit compare needs VALU temporaries, which hipcc may place in a
  // buffer register still being loaded, forcing a vmcnt drain at the loop head).
  const u32 nk = t0 < tend ? (u32)((tend - t0 + tstep - 1) / tstep) : 0u;
  const u32 s_init = (l == 0) ? init : 0u;

  // Tile k's lines are read with buffer loads: a scalar resource (base = the tile's first
  // message, range = the bytes the tile may touch) and one per-lane offset that never
  // changes (h*stride + l*128). All address arithmetic is scalar, so no VALU temporary can
  // land in a buffer register with a load in flight (which costs a vmcnt drain), and every
  // lane issues every load (no divergent branch around loads either). Reads outside the
  // range return zeros without touching memory: the missing odd message of a batch's last
  // tile, and prefetches past a wave's last tile (range 0).
  const u32 voff = (u32)h * (u32)stride + (u32)l * 128u;  // host guarantees stride < 2^31
  auto tile_rsrc = [&](u32 k) {
    const u64 m0 = 2 * (t0 + (u64)k * tstep);
    const bool live = k < nk;
    const u32 nrec = !live ? 0u : (m0 + 1 != count ? (u32)stride + 4096u : 4096u);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(live ? base + m0 * stride : base), (short)0,
                                             (int)nrec, kBufferRsrcFlags);
  };
  auto load_tile = [&](u32x4 (&d)[8], u32 k) {
    const auto r = tile_rsrc(k);
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 16 * i, 0);
    // keep the loads at this point, in order (hipcc otherwise sinks them into the compute)
    __builtin_amdgcn_sched_barrier(0);
  };

  // Table loads first, then tile 0's loads, then the LDS stores: tile 0's latency hides
  // behind the fill and the barrier.
  LdsFill<WG, kOpZ128 + 5> fill;  // step tables + Z_128 .. Z_2048
  fill.load(gtab, gops);
  // DEPTH + 1 line buffers: tile k is processed while tiles k+1 .. k+DEPTH are in flight
  u32x4 buf[DEPTH + 1][8];
#pragma unroll
  for (int d = 0; d < DEPTH; d++) load_tile(buf[d], (u32)d);  // (range 0 for waves without work)
  fill.store(sbase);
  __syncthreads();
  if (nk == 0) return;
  u32 part0 = 0, part1 = 0, part2 = 0, part3 = 0;

  // Line CRC of one tile, then (every 4th tile, or the wave's last) the combine tree.
  auto process = [&](const u32x4 (&d)[8], u32 k) {
    u32 crc = s_init;
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) crc = step4(crc ^ d[i][j], lc0, lc1);
    const int t = (int)(k & 3);
    part0 = t == 0 ? crc : part0;
    part1 = t == 1 ? crc : part1;
    part2 = t == 2 ? crc : part2;
    part3 = t == 3 ? crc : part3;
    if (t == 3 || k + 1 == nk) {
      // transpose: message slot M = 2t + h, line l -> xb + M*128 + l*4
      lds_st(xb + (0 + h) * 128 + l * 4, part0);
      lds_st(xb + (2 + h) * 128 + l * 4, part1);
      lds_st(xb + (4 + h) * 128 + l * 4, part2);
      lds_st(xb + (6 + h) * 128 + l * 4, part3);
      wave_lds_sync();
      const int M = lane >> 3, q8 = lane & 7;
      const u32x4 s = lds_ld4(xb + M * 128 + q8 * 16);  // lines 4*q8 .. 4*q8+3 of slot M
      const u32 a = opmul(sbase, kOpZ128 + 0, s[0]) ^ s[1];
      const u32 b = opmul(sbase, kOpZ128 + 0, s[2]) ^ s[3];
      u32 c = opmul(sbase, kOpZ128 + 1, a) ^ b;              // 4 lines (512 B)
      c = opmul(sbase, kOpZ128 + 2, c) ^ __shfl_down(c, 1);  // 1 KiB, valid at even q8
      c = opmul(sbase, kOpZ128 + 3, c) ^ __shfl_down(c, 2);  // 2 KiB, valid at q8 % 4 == 0
      c = opmul(sbase, kOpZ128 + 4, c) ^ __shfl_down(c, 4);  // 4 KiB, valid at q8 == 0
      const u64 kt = (k & ~3ull) + (u64)(M >> 1);
      if (q8 == 0 && kt <= k) {
        const u64 msg = 2 * (t0 + kt * tstep) + (u64)(M & 1);
        if (msg < count) out[msg] = c ^ final_xor;
      }
      wave_lds_sync();
    }
  };

  // Rotating buffers, loop unrolled DEPTH + 1 times: no register copies between
  // iterations, and tile k+DEPTH's loads are issued before tile k's data is waited for
  // (vmcnt(8*DEPTH)): with DEPTH 2 a wave keeps a tile in flight even while it computes.
  // The body has no early exit: a break between phases would give the loop head a
  // predecessor with fewer loads in flight, and hipcc's waitcnt merge would then drain
  // more than tile k at the head. The last 0..DEPTH tiles (already loaded) follow it.
  u32 k = 0;
  for (; k + DEPTH < nk; k += DEPTH + 1) {
#pragma unroll
    for (int s = 0; s <= DEPTH; s++) {
      load_tile(buf[(s + DEPTH) % (DEPTH + 1)], k + s + DEPTH);
      process(buf[s], k + s);
    }
  }
#pragma unroll
  for (int s = 0; s < DEPTH; s++)
    if (k + s < nk) process(buf[s], k + s);
}


#define SUBSPACE_UNIFORM_INST(WG, D)                                                                         \
  template __global__ void crc32_uniform4k_kernel<WG, D>(const uint8_t*, u64, u64, const u32*, const u32*, u32, u32, \
                                                         u32*, int);
SUBSPACE_UNIFORM_INST(256, 1)
SUBSPACE_UNIFORM_INST(256, 2)
SUBSPACE_UNIFORM_INST(512, 1)
SUBSPACE_UNIFORM_INST(512, 2)
SUBSPACE_UNIFORM_INST(768, 1)
SUBSPACE_UNIFORM_INST(768, 2)
SUBSPACE_UNIFORM_INST(1024, 1)
SUBSPACE_UNIFORM_INST(1024, 2)
#undef SUBSPACE_UNIFORM_INST

}  // namespace subspace_amd
