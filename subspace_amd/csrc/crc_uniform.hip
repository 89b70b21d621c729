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

template <int WG>
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
  // Tile order. order 0 ("sweep"): tau = k*nw + w, all waves advance one compact front.
  // order 1 ("region"): workgroup b owns the contiguous tiles [b*per, (b+1)*per), its waves
  // interleave inside it: tau = b*per + k*wpb + wid.
  constexpr u64 wpb = WG / 64;
  const u64 nw = (u64)gridDim.x * wpb;
  u64 t0, tstep, tend;
  if (order == 0) {
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
  const u64 nk = t0 < tend ? (tend - t0 + tstep - 1) / tstep : 0;  // this wave's tiles: tau = t0 + k*tstep
  const u32 s_init = (l == 0) ? init : 0u;

  // Lane's line of tile k. The missing odd message of the last tile (odd count) re-reads
  // the even message instead, so every lane loads unconditionally (no divergent branch
  // around the loads, which would force vmcnt(0) waits); its CRC is never stored.
  auto line_ptr = [&](u64 k) {
    u64 msg = 2 * (t0 + k * tstep) + (u64)h;
    msg = msg < count ? msg : msg - 1;
    return reinterpret_cast<const u32x4*>(base + msg * stride + (u64)l * 128);
  };

  // Table loads first, then tile 0's loads, then the LDS stores: tile 0's latency hides
  // behind the fill and the barrier.
  LdsFill<WG, kOpZ128 + 5> fill;  // step tables + Z_128 .. Z_2048
  fill.load(gtab, gops);
  u32x4 v[8];
  {
    // waves without work (nk == 0) load tile "0" of wave 0 -- harmless, keeps the load unconditional
    const u32x4* q = nk > 0 ? line_ptr(0) : reinterpret_cast<const u32x4*>(base + (u64)l * 128 * (h == 0));
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = q[i];
  }
  fill.store(sbase);
  __syncthreads();
  if (nk == 0) return;
  u32 part0 = 0, part1 = 0, part2 = 0, part3 = 0;

  // Line CRC of one tile, then (every 4th tile, or the wave's last) the combine tree.
  auto process = [&](const u32x4 (&d)[8], u64 k) {
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
  // Unconditional prefetch (past the wave's last tile it re-reads that tile): a load inside
  // a branch makes hipcc drain it with vmcnt(0) in the middle of the compute.
  auto prefetch = [&](u32x4 (&d)[8], u64 k) {
    const u32x4* q = line_ptr(k < nk ? k : nk - 1);
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = q[i];
    // keep the loads at this point (hipcc otherwise sinks them into the compute)
    __builtin_amdgcn_sched_barrier(0);
  };

  // Ping-pong buffers, loop unrolled by two: no register copies between iterations, and
  // the next tile's loads are always issued before this tile's data is waited for.
  u32x4 (&A)[8] = v;
  u32x4 B[8];
  for (u64 k = 0; k < nk; k += 2) {
    prefetch(B, k + 1);
    process(A, k);
    if (k + 1 >= nk) break;
    prefetch(A, k + 2);
    process(B, k + 1);
  }
}

template __global__ void crc32_uniform4k_kernel<768>(const uint8_t*, u64, u64, const u32*, const u32*, u32, u32, u32*, int);
template __global__ void crc32_uniform4k_kernel<512>(const uint8_t*, u64, u64, const u32*, const u32*, u32, u32, u32*, int);
template __global__ void crc32_uniform4k_kernel<640>(const uint8_t*, u64, u64, const u32*, const u32*, u32, u32, u32*, int);
template __global__ void crc32_uniform4k_kernel<256>(const uint8_t*, u64, u64, const u32*, const u32*, u32, u32, u32*, int);
template __global__ void crc32_uniform4k_kernel<1024>(const uint8_t*, u64, u64, const u32*, const u32*, u32, u32, u32*, int);

}  // namespace subspace_amd
