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

}  // namespace

extern "C" {

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
