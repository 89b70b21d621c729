// Deterministic synthetic-payload generators (device side) for tests and bench.py.
// Not part of the reference API; exported with a subspace_crc_testutil_ prefix.
//
// Byte j of message `id` = byte (j mod 8), little-endian, of
//   splitmix64(seed ^ (id << 32) ^ (j >> 3))                 
// oracle/crc32_oracle.c:oracle_synth_fill is the host twin of this generator.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "crc_device.h"

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// One message per block iteration (grid-stride over messages), threads over 8-B units.
__global__ void synth_fill_kernel(uint8_t* __restrict__ base, const uint64_t* __restrict__ offsets,
                                  const uint64_t* __restrict__ lengths, uint64_t stride, uint64_t length,
                                  uint64_t count, uint64_t first_id, uint64_t id_stride, uint64_t seed) {
  for (uint64_t m = blockIdx.x; m < count; m += gridDim.x) {
    const uint64_t off = offsets ? offsets[m] : m * stride;
    const uint64_t len = lengths ? lengths[m] : length;
    const uint64_t id = first_id + m * id_stride;
    const uint64_t key = seed ^ (id << 32);
    uint8_t* dst = base + off;
    const uint64_t units = (len + 7) >> 3;
    const bool aligned8 = (off & 7) == 0;
    for (uint64_t u = threadIdx.x; u < units; u += blockDim.x) {
      const uint64_t w = splitmix64(key ^ u);
      const uint64_t j = u << 3;
      if (aligned8 && j + 8 <= len) {
        *reinterpret_cast<uint64_t*>(dst + j) = w;
      } else {
        for (uint64_t b = 0; b < 8 && j + b < len; b++) dst[j + b] = (uint8_t)(w >> (8 * b));
      }
    }
  }
}

// Streaming-read ceiling probe: the CRC kernels' load shape (lane <-> 128-B line, 8 x
// 16-B loads per lane, 64 consecutive lines per wave instruction, the same order-0 sweep
// front) with the CRC replaced by an XOR fold and one tile in flight per wave (each tile's
// loads issued after the previous tile landed) -- what HBM gives this access pattern at
// this launch size (profiles/r01/ceiling.md "8 loads then wait": 41.0 us per 256 MiB).
// bench.py reports it next to the CRC kernel as the measured read ceiling.
using subspace_amd::u32x4;
__global__ __launch_bounds__(512) void stream_read_kernel(const u32x4* __restrict__ p, uint64_t ntiles,
                                                          unsigned* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const uint64_t w = subspace_amd::front_slot(blockIdx.x, gridDim.x, subspace_amd::rfl(threadIdx.x >> 6));
  const uint64_t nw = (uint64_t)gridDim.x * 8;
  unsigned acc = 0;
  for (uint64_t t = w; t < ntiles; t += nw) {
    u32x4 a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = p[t * 512 + lane * 8 + i];
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
  }
  out[blockIdx.x * 512 + threadIdx.x] = acc;
}

// The same with a dynamic LDS allocation it does not use (the cost of the CRC kernels' ~152 KiB
// LDS per workgroup alone, without the table fill)
__global__ __launch_bounds__(512) void stream_read_lds_kernel(const u32x4* __restrict__ p, uint64_t ntiles,
                                                              unsigned* __restrict__ out) {
  extern __shared__ unsigned lds_unused[];
  const int lane = threadIdx.x & 63;
  const uint64_t w = subspace_amd::front_slot(blockIdx.x, gridDim.x, subspace_amd::rfl(threadIdx.x >> 6));
  const uint64_t nw = (uint64_t)gridDim.x * 8;
  unsigned acc = 0;
  for (uint64_t t = w; t < ntiles; t += nw) {
    u32x4 a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = p[t * 512 + lane * 8 + i];
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
  }
  if (acc == 0x12345678u) lds_unused[threadIdx.x] = acc;  // (keeps the allocation)
  out[blockIdx.x * 512 + threadIdx.x] = acc;
}

// Slot-list read probe (S_list): the small-message kernel's access shape over a
// device slot list (subspace_crc_slot records {prefix, payload, size}) with the CRC replaced by
// an XOR fold -- the same grid rule (small_run: no wave gets more than 32 tiles), sweep front and
// tile (lane l of half h reads line l of slot 2 tau + h), one tile in flight per wave, and the
// first window's prefix words (56 B of each slot's MessagePrefix, one slot per lane) loaded in
// the prologue after tile 0's lines. MODE (what differs, for the read ceiling and its causes):
//   0  each tile's two records loaded one tile ahead, 8 clamped block addresses per lane
//      (crc_small.hip's general loop)
//   1  the wave's records in registers from the prologue, 8 clamped addresses
//   2  no records: slot m's payload at recs[0].payload + m * stride, 8 clamped addresses
//   3  as 2, one address and 8 immediate offsets (crc_uniform.hip's load issue)
//   4  the window's records in registers, one address and 8 immediate offsets (crc_small.hip's
//      FAST loop)
//   5  as 4 with two tiles in flight per wave (three line buffers)
//   6  as 3 with two tiles in flight per wave
template <int MODE>
__global__ __launch_bounds__(512) void slot_list_read_kernel(const uint64_t* __restrict__ recs, uint64_t count,
                                                             uint64_t stride, unsigned* __restrict__ out) {
  using namespace subspace_amd;
  extern __shared__ unsigned lds_unused2[];
  const int lane = threadIdx.x & 63;
  const u32 wid = rfl(threadIdx.x >> 6);
  const u32 l = (u32)lane & 31u, h = (u32)lane >> 5;
  const u64 ntiles = (count + 1) >> 1;
  const u64 nw = (u64)gridDim.x * 8;
  const u64 t0 = front_slot(blockIdx.x, gridDim.x, wid);
  u32 nk = t0 < ntiles ? (u32)((ntiles - t0 + nw - 1) / nw) : 0u;
  if (nk > 32u) nk = 32u;  // (the host's grid gives no wave more)
  const u64 fm = 2 * (t0 + (u64)((u32)lane >> 1) * nw) + ((u32)lane & 1u);
  const u64 fmc = fm < count ? fm : count - 1;
  u64 wS = 0, wL = 0;
  constexpr bool kRegs = MODE == 1 || MODE == 4 || MODE == 5;
  if (kRegs) {
    wS = recs[3 * fmc + 1];
    wL = recs[3 * fmc + 2];
  }
  const u64 s00 = recs[1];
  const u64 fpre = recs[3 * fmc];
  auto fetch = [&](u32 k, u64& s, u64& L) {
    const u32 kk = k < nk ? k : (nk ? nk - 1 : 0u);
    if (kRegs) {
      const int i0 = (int)(2u * kk);
      const u64 s0 = ((u64)(u32)__builtin_amdgcn_readlane((int)(wS >> 32), i0) << 32) |
                     (u64)(u32)__builtin_amdgcn_readlane((int)(u32)wS, i0);
      const u64 s1 = ((u64)(u32)__builtin_amdgcn_readlane((int)(wS >> 32), i0 + 1) << 32) |
                     (u64)(u32)__builtin_amdgcn_readlane((int)(u32)wS, i0 + 1);
      const u32 L0 = (u32)__builtin_amdgcn_readlane((int)(u32)wL, i0);
      const u32 L1 = (u32)__builtin_amdgcn_readlane((int)(u32)wL, i0 + 1);
      s = h ? s1 : s0;
      L = h ? L1 : L0;
    } else {
      u64 m = nk ? 2 * (t0 + (u64)kk * nw) + h : 0;
      m = m < count ? m : count - 1;
      if (MODE == 0) {
        s = recs[3 * m + 1];
        L = recs[3 * m + 2];
      } else {  // modes 2, 3, 6
        s = s00 + m * stride;
        L = 4096;
      }
    }
  };
  // (global-address-space pointers: addresses built from integers are generic, and generic
  // loads compile to flat loads, which the kernels' loads are not)
  using gptr = const __attribute__((address_space(1))) u32x4*;
  auto load_lines = [&](u32x4 (&D)[8], u64 s, u64 L) {
    if (MODE >= 3) {
      const gptr q = (gptr)(s + 128u * l);
#pragma unroll
      for (int b = 0; b < 8; b++) D[b] = q[b];
      asm volatile("" ::"v"(q));  // (no load's destination in its address VGPRs: crc_small.hip load_at)
    } else {
      u64 E = L + (s & 15u);
      E = E < 16 ? 16 : (E > 4096 ? 4096 : E);
      const u64 p0 = s & ~(u64)15;
      const u32 lastb = ((u32)E - 1u) & ~15u;
      gptr q[8];
#pragma unroll
      for (int b = 0; b < 8; b++) {
        const u32 off = 128u * l + 16u * (u32)b;
        q[b] = (gptr)(p0 + (off < lastb ? off : lastb));
        D[b] = *q[b];
      }
#pragma unroll
      for (int b = 0; b < 8; b++) asm volatile("" ::"v"(q[b]));
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  unsigned acc = 0;
  auto fold = [&](const u32x4 (&D)[8]) {
#pragma unroll
    for (int b = 0; b < 8; b++) acc ^= D[b].x ^ D[b].y ^ D[b].z ^ D[b].w;
  };
  if constexpr (MODE >= 5) {
    // two tiles in flight: wait until at most one tile's 8 loads are outstanding
    auto wait_one = []() { __builtin_amdgcn_s_waitcnt(0x0F78); };  // vmcnt(8)
    u32x4 A[8], B[8], C[8];
    u64 s, L;
    fetch(0, s, L);
    load_lines(A, s, L);
    fetch(1, s, L);
    load_lines(B, s, L);
    {
      const __attribute__((address_space(1))) uint64_t* q = (const __attribute__((address_space(1))) uint64_t*)fpre;
      uint64_t x = 0;
#pragma unroll
      for (int i = 0; i < 7; i++) x ^= q[i];
      acc ^= (unsigned)x ^ (unsigned)(x >> 32);
    }
    u32 k = 0;
    for (; k + 2 < nk; k += 3) {
      wait_one();
      fetch(k + 2, s, L);
      load_lines(C, s, L);
      fold(A);
      wait_one();
      fetch(k + 3, s, L);
      load_lines(A, s, L);
      fold(B);
      wait_one();
      fetch(k + 4, s, L);
      load_lines(B, s, L);
      fold(C);
    }
    subspace_amd::drain_before_issue();
    if (k < nk) fold(A);
    if (k + 1 < nk) fold(B);
    if (acc == 0x12345678u && count == 1) lds_unused2[threadIdx.x] = acc;  // (keeps the allocation)
    out[blockIdx.x * 512 + threadIdx.x] = acc;
    return;
  }
  u64 sA, LA, sB, LB;
  fetch(0, sA, LA);
  fetch(1, sB, LB);
  u32x4 A[8], B[8];
  load_lines(A, sA, LA);
  {
    const __attribute__((address_space(1))) uint64_t* q = (const __attribute__((address_space(1))) uint64_t*)fpre;
    uint64_t x = 0;
#pragma unroll
    for (int i = 0; i < 7; i++) x ^= q[i];
    acc ^= (unsigned)x ^ (unsigned)(x >> 32);
  }
  u32 k = 0;
  for (; k + 1 < nk; k += 2) {
    subspace_amd::drain_before_issue();
    const u64 s1 = sB, L1 = LB;
    fetch(k + 2, sA, LA);
    load_lines(B, s1, L1);
    fold(A);
    subspace_amd::drain_before_issue();
    const u64 s2 = sA, L2 = LA;
    fetch(k + 3, sB, LB);
    load_lines(A, s2, L2);
    fold(B);
  }
  if (k < nk) {
    subspace_amd::drain_before_issue();
    fold(A);
  }
  if (acc == 0x12345678u && count == 1) lds_unused2[threadIdx.x] = acc;  // (keeps the allocation)
  out[blockIdx.x * 512 + threadIdx.x] = acc;
}

// Tile-list read probe (S_large): the ragged kernel's access shape over an
// explicit list of 8 KiB tiles {16-B-aligned start address, bytes <= 8192} -- the same sweep
// front (tile tau = k * nw + w), lane l reading line l of its wave's tile as 8 x 16-B buffer
// loads against a per-tile scalar resource (blocks past the tile's bytes read as zeros without
// touching memory), one tile in flight per wave -- with the CRC replaced by an XOR fold: the read
// ceiling of a ragged or slot-list drain of large messages.
__global__ __launch_bounds__(512) void tile_list_read_kernel(const uint64_t* __restrict__ tiles, uint64_t ntiles,
                                                             unsigned* __restrict__ out) {
  using namespace subspace_amd;
  extern __shared__ unsigned lds_unused3[];
  const int lane = threadIdx.x & 63;
  const u64 w = front_slot(blockIdx.x, gridDim.x, rfl(threadIdx.x >> 6));
  const u64 nw = (u64)gridDim.x * 8;
  const u64 nk = w < ntiles ? (ntiles - w + nw - 1) / nw : 0;
  u32 vzero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(vzero));
  auto desc = [&](u64 k, u64& a, u32& n) {
    const u64 tau = nk ? (k < nk ? k : nk - 1) * nw + w : 0;
    const u32x4 d = *reinterpret_cast<const u32x4*>(tiles + 2 * (tau + vzero));
    a = rfl64(d[0], d[1]);
    n = k < nk ? ((rfl(d[2]) + 15u) & ~15u) : 0u;
  };
  auto load = [&](u32x4 (&L)[8], u64 a, u32 n) {
    const auto r = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(a), (short)0, (int)n, kBufferRsrcFlags);
#pragma unroll
    for (int b = 0; b < 8; b++) L[b] = __builtin_amdgcn_raw_buffer_load_b128(r, (u32)lane * 128u + 16u * b, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
  };
  unsigned acc = 0;
  auto fold = [&](const u32x4 (&D)[8]) {
#pragma unroll
    for (int b = 0; b < 8; b++) acc ^= D[b].x ^ D[b].y ^ D[b].z ^ D[b].w;
  };
  u64 a0, a1;
  u32 n0, n1;
  desc(0, a0, n0);
  u32x4 A[8], B[8];
  load(A, a0, n0);
  u64 k = 0;
  for (; k + 1 < nk; k += 2) {
    desc(k + 1, a1, n1);
    drain_before_issue();
    load(B, a1, n1);
    fold(A);
    desc(k + 2, a0, n0);
    drain_before_issue();
    load(A, a0, n0);
    fold(B);
  }
  drain_before_issue();
  if (k < nk) fold(A);
  if (acc == 0x12345678u && ntiles == 1) lds_unused3[threadIdx.x] = acc;  // (keeps the allocation)
  out[blockIdx.x * 512 + threadIdx.x] = acc;
}

}  // namespace

extern "C" {

// The tile-list read probe over `ntiles` records {u64 start (16-B aligned), u64 bytes <= 8192}
// in device memory, one 512-thread workgroup per CU with the ragged kernel's LDS allocation;
// dev_out holds num_cus * 512 words.
int subspace_crc_testutil_tile_list_read(const void* dev_tiles, uint64_t ntiles, unsigned* dev_out,
                                         uint64_t out_words, void* stream) {
  if (!dev_tiles || !dev_out || ntiles == 0) return -1;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -2;
  if (out_words < (uint64_t)cus * 512) return -1;
  const size_t ldsb = subspace_amd::ragged_lds_bytes();
  if (hipFuncSetAttribute((const void*)tile_list_read_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsb) !=
      hipSuccess)
    return -2;
  tile_list_read_kernel<<<(unsigned)cus, 512, ldsb, (hipStream_t)stream>>>(static_cast<const uint64_t*>(dev_tiles),
                                                                             ntiles, dev_out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// The slot-list read probe over `count` device records (MODE above; stride: modes 2 and 3's
// channel stride; lds: allocate the small-message kernel's dynamic LDS, as it runs); dev_out holds
// out_words >= grid * 512 words, grid = the small-message kernel's for this count on this device.
int subspace_crc_testutil_slot_list_read(const void* dev_records, uint64_t count, uint32_t mode, uint64_t stride,
                                         uint32_t lds, unsigned* dev_out, uint64_t out_words, void* stream) {
  if (!dev_records || !dev_out || count == 0 || mode > 6) return -1;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -2;
  const uint64_t tiles = (count + 1) / 2;
  uint64_t grid = (tiles + 7) / 8;
  if (grid > (uint64_t)cus) grid = (uint64_t)cus;
  const uint64_t need = (tiles + 8 * 32 - 1) / (8 * 32);
  if (grid < need) grid = need;
  if (grid < 1) grid = 1;
  if (out_words < grid * 512) return -1;
  const auto* r = static_cast<const uint64_t*>(dev_records);
  const size_t ldsb = lds ? subspace_amd::small_lds_bytes() + 16 : 0;
  const void* fns[7] = {(const void*)slot_list_read_kernel<0>, (const void*)slot_list_read_kernel<1>,
                        (const void*)slot_list_read_kernel<2>, (const void*)slot_list_read_kernel<3>,
                        (const void*)slot_list_read_kernel<4>, (const void*)slot_list_read_kernel<5>,
                        (const void*)slot_list_read_kernel<6>};
  if (hipFuncSetAttribute(fns[mode], hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsb) != hipSuccess) return -2;
  const hipStream_t st = (hipStream_t)stream;
  switch (mode) {
    case 0: slot_list_read_kernel<0><<<(unsigned)grid, 512, ldsb, st>>>(r, count, stride, dev_out); break;
    case 1: slot_list_read_kernel<1><<<(unsigned)grid, 512, ldsb, st>>>(r, count, stride, dev_out); break;
    case 2: slot_list_read_kernel<2><<<(unsigned)grid, 512, ldsb, st>>>(r, count, stride, dev_out); break;
    case 3: slot_list_read_kernel<3><<<(unsigned)grid, 512, ldsb, st>>>(r, count, stride, dev_out); break;
    case 4: slot_list_read_kernel<4><<<(unsigned)grid, 512, ldsb, st>>>(r, count, stride, dev_out); break;
    case 5: slot_list_read_kernel<5><<<(unsigned)grid, 512, ldsb, st>>>(r, count, stride, dev_out); break;
    default: slot_list_read_kernel<6><<<(unsigned)grid, 512, ldsb, st>>>(r, count, stride, dev_out); break;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// bytes must be a multiple of 8 KiB; out holds 256 * 512 words.
int subspace_crc_testutil_stream_read(const void* dev_base, uint64_t bytes, unsigned* dev_out, void* stream) {
  if (!dev_base || !dev_out || bytes < 8192 || (bytes % 8192)) return -1;
  stream_read_kernel<<<256, 512, 0, (hipStream_t)stream>>>(static_cast<const u32x4*>(dev_base), bytes / 8192,
                                                           dev_out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// The same read with lds_bytes (<= 160 KiB) of dynamic LDS allocated per workgroup, unused.
int subspace_crc_testutil_stream_read_lds(const void* dev_base, uint64_t bytes, unsigned* dev_out, uint32_t lds_bytes,
                                          void* stream) {
  if (!dev_base || !dev_out || bytes < 8192 || (bytes % 8192) || lds_bytes > 160u * 1024u) return -1;
  if (hipFuncSetAttribute((const void*)stream_read_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds_bytes) != hipSuccess)
    return -2;
  stream_read_lds_kernel<<<256, 512, lds_bytes, (hipStream_t)stream>>>(static_cast<const u32x4*>(dev_base),
                                                                       bytes / 8192, dev_out);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}


int subspace_crc_testutil_fill_uniform(void* dev_base, uint64_t stride, uint64_t length, uint64_t count,
                                       uint64_t first_id, uint64_t id_stride, uint64_t seed, void* stream) {
  if (!dev_base && count) return -1;
  if (!count) return 0;
  const unsigned blocks = (unsigned)(count < 65536 ? count : 65536);
  synth_fill_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(static_cast<uint8_t*>(dev_base), nullptr, nullptr,
                                                              stride, length, count, first_id, id_stride, seed);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int subspace_crc_testutil_fill_ragged(void* dev_base, const uint64_t* dev_offsets, const uint64_t* dev_lengths,
                                      uint64_t count, uint64_t first_id, uint64_t id_stride, uint64_t seed,
                                      void* stream) {
  if ((!dev_base || !dev_offsets || !dev_lengths) && count) return -1;
  if (!count) return 0;
  const unsigned blocks = (unsigned)(count < 65536 ? count : 65536);
  synth_fill_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(static_cast<uint8_t*>(dev_base), dev_offsets,
                                                              dev_lengths, 0, 0, count, first_id, id_stride, seed);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
