// The context of libsubspace_crc.so (include/subspace_crc.h's opaque subspace_crc_ctx):
// device tables, workspaces, call ordering. Internal to the library; libsubspace_crc_dev.so
// (tests, bench and tools only: devtools.hip) includes it to set the development knobs and
// hooks below on a context the product library created, so the product library exports
// nothing but the public header's symbols.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>

#include "../../include/subspace_crc.h"
#include "crc_device.h"
#include "crc_math.h"

namespace subspace_amd {

// Development hooks, installed by libsubspace_crc_dev.so (subspace_crc_testutil_probe) and
// null in every product context: while `probe` is set, the fixed-size 4 KiB batches, the
// fused slot kernel and the fused small-slot kernel launch the dev library's timestamp-
// recording instantiations of the same kernels instead (tools/wave_timeline.py,
// tools/small_timeline.py). The product library holds no such instantiation.
struct DevHooks {
  u64* probe = nullptr;  // kProbeWords per wave
  hipError_t (*uniform)(bool slot, unsigned blocks, hipStream_t st, const uint8_t* base, u64 stride, u64 count,
                        const u32* tab, const u32* ops, u32 init, u32 final_xor, u32* out, u32* zero_word,
                        SlotArgs sa) = nullptr;
  hipError_t (*small_slot)(unsigned blocks, size_t lds, hipStream_t st, const u32* tab, const u32* ops,
                           const SmallArgs& a) = nullptr;
};

// Layout tag checked by the dev library before it touches a context (both libraries are
// built from this header by the same Makefile; a mismatch means a stale dev library).
constexpr uint32_t kCtxMagic = 0x43524353u;  // "SCRC"

}  // namespace subspace_amd

struct subspace_crc_ctx {
  uint32_t magic = subspace_amd::kCtxMagic;
  uint32_t layout_bytes = 0;  // sizeof(subspace_crc_ctx) of the library that created it
  int device = 0;
  uint32_t poly = subspace_amd::kPoly;  // reflected CRC polynomial of every table and operator below
  int num_cus = 256;
  subspace_amd::u32* d_tab = nullptr;      // 4 x 256 slice tables
  subspace_amd::u32* d_rops = nullptr;     // ragged kernel: line-shift operators, Z_4096, tile shifts, padding inverses
  subspace_amd::u32* d_pow2 = nullptr;     // Z_{2^k}, k = 0..63, nibble operators (slot checksums)
  subspace_amd::u32* d_laneops = nullptr;  // uniform kernel: Z_{128*s}, s = 0..31, as [nibble][value][s]; Z_4096
  subspace_amd::Tables host_tab;
  subspace_amd::Mat32 zinv1;  // Z_1^{-1}: the ragged kernel's head seeds Z_r^{-1}(init)
  // ragged workspace
  subspace_amd::u64* d_tbase = nullptr;  // count + 1: tiles before each message (exclusive scan)
  subspace_amd::u64 ws_messages = 0;
  uint8_t* d_desc = nullptr;
  subspace_amd::u32* d_tilecrc = nullptr;  // per-tile values, wave-major (desc_capacity + one tile per wave)
  subspace_amd::u32* d_local = nullptr;    // per-segment inclusive XOR prefixes of the values, tile order
  subspace_amd::u32* d_segx = nullptr;     // per-segment XORs, then their exclusive XOR prefixes
  subspace_amd::u64 desc_capacity = 0;
  // look-back scan state: word 0 = the two workgroup tickets (u32 each), then the
  // tile-count scan's status words (scan_a_words), then the segment scan's (scan_b_words).
  // Zeroed at allocation; each call's later kernels zero what its scans used
  // (crc_device.h reset_scan_state). scan_dirty: a call failed between a scan and its reset.
  subspace_amd::u64* d_scan_state = nullptr;
  subspace_amd::u64 scan_a_words = 0, scan_b_words = 0;
  bool scan_dirty = false;
  subspace_amd::u64 mem_tiles = 0;  // device memory / 8 KiB: bounds the descriptor workspace
  subspace_amd::u32* d_overflow = nullptr;  // [0] overflow, [1] wide batch, [2] a tile past the fused kernel's 8-B range
  // path knobs (defaults = the product's choice; the dev library's subspace_crc_testutil_set
  // switches them for A/B and parity tests of the alternative paths)
  bool fused_prep = true;   // known-arena batches take crc32_ragged_count_desc_kernel
  int uniform_blocks = 0;   // 0 = one workgroup per CU
  int uniform_order = 0;    // tile order: 0 XCD-spread sweep, 1 per-workgroup region, 2 plain sweep, 3 XCD-grouped
  bool long_path = true;    // whole-8 KiB-piece uniform batches take crc32_long_kernel
  subspace_amd::u32* zero_word = nullptr;  // zeroed by the next uniform or ragged launch (slot mismatch count)
  subspace_amd::u64* d_uoff = nullptr;     // offsets/lengths materialised for non-4K uniform batches
  subspace_amd::u64* d_ulen = nullptr;
  subspace_amd::u64 u_capacity = 0;
  // host-slot pipeline (subspace_crc32_host_slots): one compute stream (the kernels share
  // the context's workspaces), a copy stream and staging per in-flight chunk
  hipStream_t hcompute = nullptr;
  struct HostStage {
    hipStream_t stream = nullptr;  // H2D copies of this stage's chunks
    hipEvent_t copied = nullptr;   // the chunk is on the device
    hipEvent_t done = nullptr;     // its results are on the host
    uint8_t* dbuf = nullptr;              // device copy of a chunk of slots
    subspace_amd::u64* dsizes = nullptr;  // its message sizes (optional)
    subspace_amd::u32* dres = nullptr;    // per-slot results: stored checksum (CALCULATE) / status (VERIFY)
    subspace_amd::u32* derr = nullptr;    // mismatch count of the chunk
    subspace_amd::u32* hres = nullptr;    // pinned host copies of dres / derr
    subspace_amd::u32* herr = nullptr;
  } hstage[2];
  subspace_amd::u64 h_bytes = 0, h_slots = 0;  // staging capacities
  // host slot lists (subspace_crc32_host_slot_list): translated records and statuses
  subspace_crc_slot* l_hrec = nullptr;
  subspace_crc_slot* l_drec = nullptr;
  subspace_amd::u32* l_dstatus = nullptr;  // count statuses + the mismatch count
  subspace_amd::u32* l_hstatus = nullptr;
  subspace_amd::u64 l_capacity = 0;
  subspace_amd::u32* d_crc0 = nullptr;  // slot batches: payload CRCs from init 0
  subspace_amd::u64* d_soff = nullptr;  // slot batches: payload offsets of the contiguous layout
  subspace_amd::u64* d_slen = nullptr;  // strided slots with per-slot sizes: the sizes, an oversize one as 0
  subspace_amd::u64 s_capacity = 0;
  // fused slot kernel: a ring of counter words, (workgroups done << 32) | mismatches, each 0
  // between calls (the last workgroup resets its word); consecutive calls take consecutive
  // words, so even calls that overlap on the device never share one
  subspace_amd::u64* d_slot_counter = nullptr;
  subspace_amd::u32 slot_counter_next = 0;
  bool fused_slots = true;  // contiguous 4 KiB slot batches take the fused uniform kernel
  bool small_path = true;   // batches of messages <= 4 KiB take the small-message kernel (crc_small.hip)
  subspace_amd::DevHooks dev;           // development hooks (null in a product context)
  subspace_amd::u32* d_fault = nullptr;  // fault words (crc_device.h FaultRef): [0] kFault* bits, read and cleared by
                                         // subspace_crc_ctx_check; [1] the generation of the last call whose scan faulted
  subspace_amd::u32 call_gen = 0;        // generation of the latest ragged / long call (never 0 once used)
  // One call at a time per context (a recursive mutex: the host-slot paths call the device
  // paths), and device workspace use ordered across streams: a call that uses the context's
  // device workspaces (ragged / long / two-kernel slot paths, the host-slot staging) on another
  // stream than the previous such call first waits for ws_done, recorded at the end of every
  // such call on its own stream. Calls that use no context workspace (the uniform 4 KiB kernel,
  // the fused slot kernel) take neither step.
  std::recursive_mutex mu;
  int depth = 0;  // nesting of public calls on this thread (under mu)
  hipEvent_t ws_done = nullptr;
  hipStream_t ws_stream = nullptr;
  bool ws_recorded = false;  // ws_done holds the last workspace call
  bool ws_waited = false;    // the current (outermost) call has ordered its stream
  hipStream_t ws_call_stream = nullptr;
};
