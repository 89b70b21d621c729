// Fixed-size batch kernel: one CRC32 per 4 KiB message (BASELINE configs B and E).
//
// Work decomposition (DESIGN.md "Uniform kernel"):
//  * A tile is 2 messages = 64 lines of 128 B. Lane l of half h (h = lane >> 5)
//    owns line l of message 2*tau + h, so every wave load instruction touches 64
//    consecutive 128-B lines (the access shape measured near the coalesced HBM rate
//    on MI355X; lane-contiguous 1 KiB chunks ran ~40 % slower).
//  * Each wave streams tiles tau = t0 + k*tstep (all waves sweep one compact front) and
//    always has the next tile's 8 loads in flight while it computes the current one.
//  * Per line: 32 slice-by-4 steps from 32-way replicated LDS tables (4 conflict-free
//    ds_read_b32 + 4 v_perm + 4 v_xor per word).
//  * Every 4 tiles the wave holds line CRCs of 8 messages (crc_raw(0, line), or with
//    the batch init for line 0). They are transposed through LDS so lane j holds 4
//    consecutive lines of message j>>3, combined in-lane (Z_128, Z_256) and across 8
//    lanes (Z_512, Z_1024, Z_2048) with nibble-table GF(2) operators:
//      crc(msg) = XOR_i Z_{128*(31-i)}(line_i)     (crc_raw linearity)
//  * Results go to a per-wave LDS ring and are stored to HBM only when the ring is full
//    (every 256 tiles at 8 waves per CU) and at the end. vmcnt counts stores with the
//    loads, in order, so a store in the stream makes the wait for the next tile's loads
//    wait for the store's write-back too: a store every 4 tiles cost ~10 % of a
//    streaming kernel's rate (tools/ubench/streamread.hip lines_store: 6.0 vs 6.6 TB/s).
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
  constexpr int kWaves = WG / 64;
  constexpr int kRing = uniform_ring(kWaves);  // results per wave ring
  const u32 xb = sbase + kUniXpose + (u32)wid * kLdsXposePerWave;
  const u32 ring = sbase + kUniXpose + kWaves * kLdsXposePerWave + (u32)wid * (4u * kRing);
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
  // this wave's tiles: tau = t0 + k*tstep, k < nk. 32-bit tile counters keep the loop
  // control scalar (a 64-bit compare needs VALU temporaries, which hipcc may place in a
  // buffer register still being loaded, forcing a vmcnt drain at the loop head).
  const u32 nk = t0 < tend ? (u32)((tend - t0 + tstep - 1) / tstep) : 0u;
  const u32 s_init = (l == 0) ? init : 0u;

  // Tile k's lines. Past the wave's last tile it re-reads that tile, and the missing odd
  // message of the batch's last tile re-reads the even one (its CRC is never stored): every
  // lane issues every load, no divergent branch around loads (which forces vmcnt(0)).
  // Waves without tiles read message 0. (Buffer loads against a per-tile scalar resource,
  // which make all this address math scalar, measured 7-10 % slower: DESIGN.md 4.1.)
  auto load_tile = [&](u32x4 (&d)[8], u32 k) {
    const u32 kk = k < nk ? k : (nk ? nk - 1 : 0u);
    u64 msg = nk ? 2 * (t0 + (u64)kk * tstep) + (u64)h : 0;
    msg = msg < count ? msg : msg - 1;
    const u32x4* q = reinterpret_cast<const u32x4*>(base + msg * stride + (u64)l * 128);
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = q[i];
    // keep the loads at this point, in order (hipcc otherwise sinks them into the compute)
    __builtin_amdgcn_sched_barrier(0);
  };

  // CRC of this lane's line of a tile (from the batch init for line 0, else from 0).
  auto line_crc = [&](const u32x4 (&d)[8]) {
    u32 crc = s_init;
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) crc = step4(crc ^ d[i][j], lc0, lc1);
    return crc;
  };

  // Results of the group of tiles kb .. kb+3 (nv of them real): transpose, tree, into the
  // ring slots 2*(kb - kf + t) + h (kf = first tile of the ring's window).
  auto group_result = [&](u32 p0, u32 p1, u32 p2, u32 p3, u32 kb, u32 nv, u32 kf) {
    // transpose: message slot M = 2t + h, line l -> xb + M*128 + l*4
    lds_st(xb + (0 + h) * 128 + l * 4, p0);
    lds_st(xb + (2 + h) * 128 + l * 4, p1);
    lds_st(xb + (4 + h) * 128 + l * 4, p2);
    lds_st(xb + (6 + h) * 128 + l * 4, p3);
    wave_lds_sync();
    const int M = lane >> 3, q8 = lane & 7;
    const u32x4 s = lds_ld4(xb + M * 128 + q8 * 16);  // lines 4*q8 .. 4*q8+3 of slot M
    const u32 a = opmul(sbase, kOpZ128 + 0, s[0]) ^ s[1];
    const u32 b = opmul(sbase, kOpZ128 + 0, s[2]) ^ s[3];
    u32 c = opmul(sbase, kOpZ128 + 1, a) ^ b;              // 4 lines (512 B)
    c = opmul(sbase, kOpZ128 + 2, c) ^ __shfl_down(c, 1);  // 1 KiB, valid at even q8
    c = opmul(sbase, kOpZ128 + 3, c) ^ __shfl_down(c, 2);  // 2 KiB, valid at q8 % 4 == 0
    c = opmul(sbase, kOpZ128 + 4, c) ^ __shfl_down(c, 4);  // 4 KiB, valid at q8 == 0
    if (q8 == 0 && (u32)(M >> 1) < nv) lds_st(ring + 4u * (2u * (kb - kf) + (u32)M), c ^ final_xor);
    wave_lds_sync();
  };
  // Store the ring's results of tiles kf .. kf+nt-1 (messages 2*tau, 2*tau+1 of each).
  auto flush = [&](u32 kf, u32 nt) {
#pragma unroll
    for (int i = 0; i < kRing / 64; i++) {
      const u32 slot = (u32)(i * 64 + lane);
      const u32 t = slot >> 1;
      const u64 msg = 2 * (t0 + (u64)(kf + t) * tstep) + (u64)(slot & 1u);
      if (t < nt && msg < count) out[msg] = lds_ld(ring + 4u * slot);
    }
    wave_lds_sync();
  };

  // Table loads first, then tile 0's loads, then the LDS stores: tile 0's latency hides
  // behind the fill and the barrier.
  LdsFill<WG, kUniformOps> fill;  // step tables + Z_64, Z_128 .. Z_2048
  fill.load(gtab, gops);
  u32x4 A[8], B[8];
  load_tile(A, 0);
  fill.store(sbase);
  __syncthreads();
  if (nk == 0) return;

  // Whole groups: ping-pong buffers, the next tile's loads always issued before this
  // tile's data is waited for; the ring is stored when full.
  u32 k = 0, kf = 0;
  for (; k + 3 < nk; k += 4) {
    load_tile(B, k + 1);
    const u32 p0 = line_crc(A);
    load_tile(A, k + 2);
    const u32 p1 = line_crc(B);
    load_tile(B, k + 3);
    const u32 p2 = line_crc(A);
    load_tile(A, k + 4);
    const u32 p3 = line_crc(B);
    group_result(p0, p1, p2, p3, k, 4u, kf);
    if (k + 4 - kf == (u32)(kRing / 2)) {
      flush(kf, kRing / 2);
      kf = k + 4;
    }
  }
  // The last 1..3 tiles (tile k already in A); loads past the end re-read the last tile.
  if (k < nk) {
    load_tile(B, k + 1);
    const u32 p0 = line_crc(A);
    load_tile(A, k + 2);
    const u32 p1 = line_crc(B);
    const u32 p2 = line_crc(A);
    group_result(p0, p1, p2, 0u, k, nk - k, kf);
  }
  if (nk > kf) flush(kf, nk - kf);
}

template __global__ void crc32_uniform4k_kernel<256>(const uint8_t*, u64, u64, const u32*, const u32*, u32, u32, u32*,
                                                     int);
template __global__ void crc32_uniform4k_kernel<512>(const uint8_t*, u64, u64, const u32*, const u32*, u32, u32, u32*,
                                                     int);
template __global__ void crc32_uniform4k_kernel<768>(const uint8_t*, u64, u64, const u32*, const u32*, u32, u32, u32*,
                                                     int);
template __global__ void crc32_uniform4k_kernel<1024>(const uint8_t*, u64, u64, const u32*, const u32*, u32, u32, u32*,
                                                      int);

}  // namespace subspace_amd
