// Message-slot checksums: the reference's 3-span CRC (common/channel.h:527-542) for a
// batch of slots, stored into the prefix (publisher, client/publisher.cc:664-675) or
// verified against it (subscriber, client/client.cc:1346-1356).
//
// The payload span dominates and runs through the batch kernels with init 0 and no
// final XOR (crc0 = crc_raw(0, payload)). This kernel finishes each slot with one thread:
//   h   = crc_raw(0xFFFFFFFF, span0 || span1)         (44 + metadata_size prefix bytes)
//   crc = ~(Z_L(h) ^ crc0),  L = message_size          (linearity, crc_math.h)
// Z_L is applied by binary decomposition over Z_{2^k} nibble operators (gpow2, 64 ops; the
// first 16 staged in LDS per workgroup, the rest read from global memory). The prefix bytes
// go through slice-by-4 tables staged in LDS (4 KiB per workgroup).
#include "crc_device.h"

namespace subspace_amd {

constexpr int kSlotWG = 256;
constexpr u32 kHasChecksum = 4u;  // kMessageHasChecksum, common/channel.h:65

__device__ __forceinline__ u32 tab_step4(const u32* __restrict__ t, u32 x) {
  return t[768 + (x & 0xFFu)] ^ t[512 + ((x >> 8) & 0xFFu)] ^ t[256 + ((x >> 16) & 0xFFu)] ^ t[x >> 24];
}
__device__ __forceinline__ u32 tab_step1(const u32* __restrict__ t, u32 crc, u32 b) {
  return (crc >> 8) ^ t[(crc ^ b) & 0xFFu];
}

// crc_raw over n bytes at p (any alignment): bytes up to a 4-B boundary, dwords, tail bytes.
__device__ u32 crc_bytes(const u32* __restrict__ t, u32 crc, const uint8_t* p, u64 n) {
  while (n && ((uintptr_t)p & 3u)) {
    crc = tab_step1(t, crc, *p++);
    n--;
  }
  const u32* q = reinterpret_cast<const u32*>(p);
  for (; n >= 4; n -= 4) crc = tab_step4(t, crc ^ *q++);
  p = reinterpret_cast<const uint8_t*>(q);
  while (n--) crc = tab_step1(t, crc, *p++);
  return crc;
}

// Slot i: prefix = slots ? slots[3i] : buf + i*stride; payload size = slots ? slots[3i+2]
// : (sizes ? sizes[i] : usize). CALCULATE also writes the stored value to crc_out[i] when
// crc_out is not null. A size above max_len (strided layouts: the slot's payload area) is
// SUBSPACE_CRC_SLOT_OVERSIZE: nothing stored or compared.
__global__ __launch_bounds__(kSlotWG) void crc32_slot_finish_kernel(
    const u64* __restrict__ slots, uint8_t* __restrict__ buf, u64 stride, const u64* __restrict__ sizes, u64 usize,
    u64 count, u64 max_len, int checksum_size, int metadata_size, u32 mode, const u32* __restrict__ crc0,
    const u32* __restrict__ gtab, const u32* __restrict__ gpow2, u32* __restrict__ status,
    u32* __restrict__ error_count, u32* __restrict__ crc_out) {
  __shared__ u32 t[1024];
  // Z_{2^k}, k < kPowLds, staged too: the shift by the payload length is a chain of up to 16
  // dependent operator applications, each 8 lookups (from global memory: 12.5-12.9 us for
  // S_large's 1 .. 32,767-B payloads, r06s)
  constexpr int kPowLds = 16;
  __shared__ u32 pw2[kPowLds * 128];
  for (int i = threadIdx.x; i < 1024; i += kSlotWG) t[i] = gtab[i];
  for (int i = threadIdx.x; i < kPowLds * 128; i += kSlotWG) pw2[i] = gpow2[i];
  __syncthreads();
  const u64 i = (u64)blockIdx.x * kSlotWG + threadIdx.x;
  if (i >= count) return;
  uint8_t* prefix = slots ? reinterpret_cast<uint8_t*>(slots[3 * i]) : buf + i * stride;
  const u64 len = slots ? slots[3 * i + 2] : (sizes ? sizes[i] : usize);
  u32* pw = reinterpret_cast<u32*>(prefix);  // 8-B aligned (int64 fields)
  if (len > max_len) {
    if (status) status[i] = 4u;  // SUBSPACE_CRC_SLOT_OVERSIZE
    return;
  }

  // span 0: prefix[4, 48) = dwords 1..11; flags (int64 at offset 32) is dword 8
  u32 w[12];
#pragma unroll
  for (int k = 1; k < 12; k++) w[k] = pw[k];
  const bool calc = mode == 0u;
  const bool has = (w[8] & kHasChecksum) != 0u;
  if (calc && !has) {
    w[8] |= kHasChecksum;  // SetHasChecksum() precedes the CRC (client/publisher.cc:665)
    pw[8] = w[8];
  }
  if (!calc && !has) {  // not checksummed by its publisher: nothing to verify
    if (status) status[i] = 2u;
    return;
  }
  u32 h = 0xFFFFFFFFu;
#pragma unroll
  for (int k = 1; k < 12; k++) h = tab_step4(t, h ^ w[k]);
  // span 1: the metadata after the checksum area
  if (metadata_size > 0) h = crc_bytes(t, h, prefix + 48 + checksum_size, (u64)metadata_size);
  // span 2: the payload, from its init-0 CRC
  u32 zh = h;
  {
    u64 n = len;
    for (int k = 0; n; k++, n >>= 1) {
      if (!(n & 1u)) continue;
      const u32* op = k < kPowLds ? pw2 + 128 * k : gpow2 + 128 * k;
      u32 r = 0;
#pragma unroll
      for (int j = 0; j < 8; j++) r ^= op[16 * j + ((zh >> (4 * j)) & 15u)];
      zh = r;
    }
  }
  const u32 crc = ~(zh ^ crc0[i]);
  if (calc) {
    pw[12] = crc;  // *reinterpret_cast<uint32_t*>(checksum.data()) = ~crc (client/checksum.h:36)
    if (status) status[i] = 0u;
    if (crc_out) crc_out[i] = crc;  // compact copy for the host-slot path's write-back
  } else {
    const bool ok = pw[12] == crc;  // client/checksum.h:46
    if (status) status[i] = ok ? 0u : 1u;
    if (!ok && error_count) atomicAdd(error_count, 1u);
  }
}

// Payload offsets of the contiguous layout (relative to the first prefix), and the per-slot
// sizes the payload kernels read: a size beyond the slot's payload area (max_len) as 0, so no
// kernel reads an oversize slot's bytes (crc32_slot_finish_kernel labels it OVERSIZE).
__global__ void slot_payload_offsets_kernel(u64 stride, u64 prefix_size, u64 count, u64* __restrict__ offsets,
                                            const u64* __restrict__ sizes, u64 max_len, u64* __restrict__ clamped) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  offsets[i] = i * stride + prefix_size;
  const u64 L = sizes[i];
  clamped[i] = L > max_len ? 0 : L;
}

}  // namespace subspace_amd
