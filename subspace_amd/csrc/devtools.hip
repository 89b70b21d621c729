// libsubspace_crc_dev.so: development entry points for tests, bench.py and tools/ -- never
// linked by a reference client, and nothing in libsubspace_crc.so depends on it (VERDICT r05
// item 7: the product library exports only include/subspace_crc.h's and checksum.h's symbols).
//   * path knobs of a context (subspace_crc_testutil_set / _tune): A/B and parity tests of the
//     alternative paths (ragged instead of small, two-kernel slots, separate descriptor kernel);
//   * fault injection (a stale look-back ticket) and the fault words' read-back;
//   * the timestamp-recording PROBE instantiations of the uniform, fused-slot and small-slot
//     kernels, installed as the context's DevHooks (tools/wave_timeline.py,
//     tools/small_timeline.py);
//   * the headline kernel over aliased messages (the compute-only ledger row);
//   * with testutil.hip: the synthetic-payload generators and the read-ceiling probes.
// Contexts come from the product library; this library reads and sets their fields through
// ctx.h (the same header, the same Makefile), after checking the layout tag.
#define SUBSPACE_DEV_TU 1
#include "crc_small.hip"
#include "crc_uniform.hip"
#include "ctx.h"

#include <algorithm>
#include <cstring>

namespace subspace_amd {
template __global__ void crc32_small_kernel<512, true, true, 32>(const u32*, const u32*, SmallArgs);
template __global__ void crc32_uniform4k_kernel<512, false, true>(const uint8_t*, u64, u64, const u32*, const u32*, u32,
                                                                  u32, u32*, int, u32*, SlotArgs);
template __global__ void crc32_uniform4k_kernel<512, true, true>(const uint8_t*, u64, u64, const u32*, const u32*, u32,
                                                                 u32, u32*, int, u32*, SlotArgs);
// this library's own copy of the headline instantiation (uniform_alias)
template __global__ void crc32_uniform4k_kernel<512, false, false>(const uint8_t*, u64, u64, const u32*, const u32*,
                                                                   u32, u32, u32*, int, u32*, SlotArgs);
}  // namespace subspace_amd

using namespace subspace_amd;

namespace {

bool ctx_ok(const subspace_crc_ctx* c) {
  return c && c->magic == kCtxMagic && c->layout_bytes == (uint32_t)sizeof(subspace_crc_ctx);
}

int blocks_for(const subspace_crc_ctx* c, u64 tiles) {  // capi.hip grid_for(c, tiles, 8)
  u64 b = (tiles + 7) / 8;
  if (b > (u64)c->num_cus) b = (u64)c->num_cus;
  return (int)(b ? b : 1);
}

hipError_t uniform_probe(bool slot, unsigned blocks, hipStream_t st, const uint8_t* base, u64 stride, u64 count,
                         const u32* tab, const u32* ops, u32 init, u32 final_xor, u32* out, u32* zero_word,
                         SlotArgs sa) {
  if (slot)
    crc32_uniform4k_kernel<512, true, true><<<blocks, 512, uniform_slot_lds_bytes(8), st>>>(
        base, stride, count, tab, ops, init, final_xor, out, 0, zero_word, sa);
  else
    crc32_uniform4k_kernel<512, false, true><<<blocks, 512, uniform_lds_bytes(8), st>>>(
        base, stride, count, tab, ops, init, final_xor, out, 0, zero_word, sa);
  return hipGetLastError();
}

hipError_t small_slot_probe(unsigned blocks, size_t lds, hipStream_t st, const u32* tab, const u32* ops,
                            const SmallArgs& a) {
  crc32_small_kernel<512, true, true, 32><<<blocks, 512, lds, st>>>(tab, ops, a);
  return hipGetLastError();
}

hipError_t set_lds_attributes() {
  static hipError_t e = [] {
    hipError_t r = hipFuncSetAttribute((const void*)crc32_uniform4k_kernel<512, false, true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)uniform_lds_bytes(8));
    if (r == hipSuccess)
      r = hipFuncSetAttribute((const void*)crc32_uniform4k_kernel<512, true, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)uniform_slot_lds_bytes(8));
    if (r == hipSuccess)
      r = hipFuncSetAttribute((const void*)crc32_uniform4k_kernel<512, false, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)uniform_lds_bytes(8));
    if (r == hipSuccess)
      r = hipFuncSetAttribute((const void*)crc32_small_kernel<512, true, true, 32>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)small_lds_bytes() + 16);
    return r;
  }();
  return e;
}

}  // namespace

extern "C" {

// Named knobs of a context (defaults = the product's choice):
//   "long_path":    1 whole-8 KiB-piece uniform batches take crc32_long_kernel, 0 the ragged path
//   "fused_slots":  1 contiguous 4 KiB slot batches without metadata take the fused slot kernel,
//                   0 the payload kernel + crc32_slot_finish_kernel
//   "fused_prep":   1 ragged batches with a known arena of at most 2^37 bytes take the fused
//                   tile-count scan + descriptor kernel, 0 the two kernels
//   "small_path":   1 messages <= 4 KiB take the small-message kernel, 0 the ragged path
//   "stale_ticket": plant a stale tile-count scan ticket (the state a racing or half-finished
//                   call could leave; the context's ragged workspace must exist, e.g. after
//                   subspace_crc_ctx_reserve): the next ragged call must report
//                   SUBSPACE_CRC_EFAULT through subspace_crc_ctx_check
int subspace_crc_testutil_set(subspace_crc_ctx* c, const char* key, int value) {
  if (!ctx_ok(c) || !key) return SUBSPACE_CRC_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  if (!std::strcmp(key, "stale_ticket")) {
    if (!c->d_scan_state) return SUBSPACE_CRC_EINVAL;
    const u32 v = (u32)value;
    if (hipSetDevice(c->device) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(c->d_scan_state, &v, sizeof(u32), hipMemcpyHostToDevice) != hipSuccess)
      return SUBSPACE_CRC_EHIP;
    return SUBSPACE_CRC_OK;
  }
  bool* knob = !std::strcmp(key, "long_path")     ? &c->long_path
               : !std::strcmp(key, "fused_slots") ? &c->fused_slots
               : !std::strcmp(key, "fused_prep")  ? &c->fused_prep
               : !std::strcmp(key, "small_path")  ? &c->small_path
                                                  : nullptr;
  if (!knob) return SUBSPACE_CRC_EINVAL;
  *knob = value != 0;
  return SUBSPACE_CRC_OK;
}

// The uniform 4 KiB kernel's grid: an optional cap on the workgroups and the tile order (0
// XCD-spread sweep, 1 per-workgroup region, 2 plain sweep, 3 XCD-grouped). The workgroup size
// is 512 (the other sizes were measured and dropped; anything else is EINVAL).
int subspace_crc_testutil_tune(subspace_crc_ctx* c, int uniform_wg, int uniform_blocks, int uniform_order) {
  if (!ctx_ok(c) || uniform_wg != 512 || uniform_order < 0 || uniform_order > 3 || uniform_blocks < 0)
    return SUBSPACE_CRC_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  c->uniform_blocks = uniform_blocks;
  c->uniform_order = uniform_order;
  return SUBSPACE_CRC_OK;
}

// While dev_words is non-null, fixed-size 4 KiB batches, fused slot batches and fused small-slot
// batches run this library's PROBE instantiations, which write kProbeWords u64 per wave
// (timestamps, HW_ID, XCC_ID, tile count) to dev_words; the caller sizes it for
// subspace_crc_testutil_probe_waves records. Null uninstalls the hooks.
int subspace_crc_testutil_probe(subspace_crc_ctx* c, void* dev_words) {
  if (!ctx_ok(c)) return SUBSPACE_CRC_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  if (dev_words) {
    if (hipSetDevice(c->device) != hipSuccess || set_lds_attributes() != hipSuccess) return SUBSPACE_CRC_EHIP;
    c->dev.uniform = uniform_probe;
    c->dev.small_slot = small_slot_probe;
  }
  c->dev.probe = static_cast<u64*>(dev_words);
  return SUBSPACE_CRC_OK;
}

// The number of waves (records) the PROBE launch of a count-message batch has.
uint64_t subspace_crc_testutil_probe_waves(subspace_crc_ctx* c, uint64_t count) {
  if (!ctx_ok(c)) return 0;
  // the larger of the uniform kernel's grid and the slot kernels' (more workgroups than CUs
  // when a wave would get more than 32 tiles)
  const u64 tiles = (count + 1) / 2;
  return std::max<u64>((u64)blocks_for(c, tiles), (tiles + 8ull * kRp2MaxTilesPerWave - 1) / (8ull * kRp2MaxTilesPerWave)) * 8u;
}

// The uniform 4 KiB kernel over `count` messages that all alias the same 4 KiB at dev_base
// (stride 0), so every line load hits the cache: the kernel's compute-only time at the
// headline's grid and tile count (the ledger's "compute" row, tools/pmc_ledger.sh). out[i] =
// the CRC of that one message for every i.
int subspace_crc_testutil_uniform_alias(subspace_crc_ctx* c, const void* dev_base, uint64_t count, uint32_t* dev_out,
                                        void* stream) {
  if (!ctx_ok(c) || !dev_base || !dev_out || count == 0 || ((uintptr_t)dev_base % 16)) return SUBSPACE_CRC_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  if (hipSetDevice(c->device) != hipSuccess || set_lds_attributes() != hipSuccess) return SUBSPACE_CRC_EHIP;
  const u64 tiles = (count + 1) / 2;
  crc32_uniform4k_kernel<512, false, false><<<blocks_for(c, tiles), 512, uniform_lds_bytes(8), (hipStream_t)stream>>>(
      static_cast<const uint8_t*>(dev_base), 0, count, c->d_tab, c->d_laneops, 0u, 0u, dev_out, 0, nullptr, SlotArgs{});
  return hipGetLastError() == hipSuccess ? SUBSPACE_CRC_OK : SUBSPACE_CRC_EHIP;
}

// The context's fault words after `stream` finishes: [0] the kFault* bits, [1] the generation
// mark of the last call whose look-back scan faulted (tests/test_gpu_fault.py).
int subspace_crc_testutil_fault_words(subspace_crc_ctx* c, uint32_t* host_words, void* stream) {
  if (!ctx_ok(c) || !host_words) return SUBSPACE_CRC_EINVAL;
  std::lock_guard<std::recursive_mutex> lk(c->mu);
  if (hipSetDevice(c->device) != hipSuccess ||
      hipMemcpyAsync(host_words, c->d_fault, 2 * sizeof(u32), hipMemcpyDeviceToHost, (hipStream_t)stream) != hipSuccess ||
      hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
    return SUBSPACE_CRC_EHIP;
  return SUBSPACE_CRC_OK;
}

// The generation of the context's latest ragged / long call (its scans' fault mark).
uint32_t subspace_crc_testutil_call_gen(subspace_crc_ctx* c) { return ctx_ok(c) ? c->call_gen : 0u; }

}  // extern "C"
