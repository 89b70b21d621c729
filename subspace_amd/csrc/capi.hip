// C ABI of libsubspace_crc.so (include/subspace_crc.h): contexts, table upload,
// workspace management and kernel launches. No torch, no Python: plain pointers,
// sizes, int status codes, thread-local error strings.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/subspace_crc.h"
#include "crc_device.h"
#include "crc_math.h"
#include "ctx.h"

namespace subspace_amd {

template <int WG, bool SLOT, bool PROBE>
__global__ void crc32_uniform4k_kernel(const uint8_t*, u64, u64, const u32*, const u32*, u32, u32, u32*, int, u32*,
                                       SlotArgs);

struct TileDesc;
struct TileDesc8;
__global__ void crc32_ragged_count_desc_kernel(const u64*, u32, const u64*, u32, u64, u32, u32, u64*, u32*, u32*,
                                               u64*, u32*, u64, TileDesc8*, u32*, FaultRef);
__global__ void crc32_ragged_count_desc16_kernel(const u64*, u32, const u64*, u32, u64, u32, u32, u64*, u32*, u32*,
                                                 u64*, u32*, u64, TileDesc*, u32*, FaultRef);
__global__ void crc32_ragged_count_scan_kernel(const u64*, u32, const u64*, u32, u64, u32, u32, u64*, u32*, u32*,
                                               u64*, u32*, u32*, FaultRef);
__global__ void tile_segment_scan_kernel(const u32*, u32, u32, u32, const u64*, u64, u32*, u32*);
__global__ void segment_prefix_kernel(u32*, u64, u32, u32, const u64*, u64, u64*, u32*, FaultRef);
__global__ void crc32_ragged_desc_kernel(const u64*, u32, const u64*, u32, const u64*, u64, u64, TileDesc*, u32*,
                                         u64*, u64, u32*, FaultRef);
template <int WG>
__global__ void crc32_ragged_kernel(const uint8_t*, const u64*, u32, const u64*, u32, const u64*, u64,
                                    const TileDesc*, const u32*, const u32*, const u32*, HeadSeeds, u32*, u32*, u32,
                                    u64*, u64, u32*, FaultRef);
__global__ void crc32_ragged_final_kernel(const u64*, const u64*, u32, const u64*, u32, u64, const u32*, const u32*,
                                          u32, u32, u32*, const u32*, u32, u32*, u64*, u64, u32*, FaultRef);
__global__ void crc32_slot_finish_kernel(const u64*, uint8_t*, u64, const u64*, u64, u64, u64, int, int, u32,
                                         const u32*, const u32*, const u32*, u32*, u32*, u32*);
__global__ void slot_payload_offsets_kernel(u64, u64, u64, u64*, const u64*, u64, u64*);
__global__ void uniform_offsets_kernel(u64 stride, u64 length, u64 count, u64* offsets, u64* lengths);
template <int WG>
__global__ void crc32_long_kernel(const uint8_t*, u64, u32, u32, const u32*, const u32*, u32, u32, u32*, u32);
__global__ void crc32_long_final_kernel(const u32*, const u32*, u32, u32, u32, u32, u32*, u64*, u64, u32*);
template <int WG, bool SLOT, bool PROBE, int G>
__global__ void crc32_small_kernel(const u32*, const u32*, SmallArgs);

}  // namespace subspace_amd

using namespace subspace_amd;

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
int hip_fail(hipError_t e, const char* what) {
  return fail(SUBSPACE_CRC_EHIP, "%s: %s", what, hipGetErrorString(e));
}
#define HIP_TRY(call)                                   \
  do {                                                  \
    hipError_t e_ = (call);                             \
    if (e_ != hipSuccess) return hip_fail(e_, #call);   \
  } while (0)

constexpr int kRaggedWG = 512;

// Host regions registered with subspace_crc_host_register: host range -> device alias
// (hipHostRegisterMapped), for the zero-copy host slot-list path.
struct HostRegion {
  uintptr_t host;
  uint64_t bytes;
  uintptr_t dev;
};
std::mutex g_regions_mu;
std::vector<HostRegion> g_regions;

// Device alias of host range [p, p+n), or 0 if no registered region holds all of it.
uintptr_t host_alias(uintptr_t p, uint64_t n) {
  for (const auto& r : g_regions)
    if (p >= r.host && p - r.host <= r.bytes && n <= r.bytes - (p - r.host)) return r.dev + (p - r.host);
  return 0;
}
#ifndef SUBSPACE_FINAL_BLOCKS_PER_CU
#define SUBSPACE_FINAL_BLOCKS_PER_CU 2  // ragged final kernel: a persistent grid (0: one workgroup per 1,024 messages)
#endif
constexpr size_t kTileDescBytes = 16;  // the wide form; 8 B (TileDesc8) for most batches
constexpr u64 ceil_div(u64 a, u64 b) { return (a + b - 1) / b; }

}  // namespace

namespace subspace_amd {
// The thread-local error string for the library's host-only sources (split_alloc.cpp).
int set_error(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
}  // namespace subspace_amd


namespace {

constexpr u32 kSlotCounters = 64;  // the fused slot kernel's counter ring (subspace_crc_ctx::d_slot_counter)

bool capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

// Scope of a public call: the context's mutex; when the outermost call ends, ws_done is
// recorded on the stream on which the call used the context's workspaces (if it did).
struct CallScope {
  subspace_crc_ctx* c;
  std::lock_guard<std::recursive_mutex> lk;
  explicit CallScope(subspace_crc_ctx* ctx) : c(ctx), lk(ctx->mu) {
    if (c->depth++ == 0) c->ws_waited = false;
  }
  ~CallScope() {
    if (--c->depth == 0 && c->ws_waited) {
      // (a captured call is ordered by the graph's launch stream; nothing is recorded)
      if (!capturing(c->ws_call_stream) && hipEventRecord(c->ws_done, c->ws_call_stream) == hipSuccess) {
        c->ws_stream = c->ws_call_stream;
        c->ws_recorded = true;
      }
      c->ws_waited = false;
    }
  }
  CallScope(const CallScope&) = delete;
  CallScope& operator=(const CallScope&) = delete;
};

// Before the first kernel of a call that uses the context's device workspaces on stream st:
// wait for the previous such call if it ran on another stream.
int use_workspace(subspace_crc_ctx* c, hipStream_t st) {
  if (c->ws_waited) return SUBSPACE_CRC_OK;
  if (!c->ws_done) HIP_TRY(hipEventCreateWithFlags(&c->ws_done, hipEventDisableTiming));
  if (c->ws_recorded && c->ws_stream != st && !capturing(st)) HIP_TRY(hipStreamWaitEvent(st, c->ws_done, 0));
  c->ws_waited = true;
  c->ws_call_stream = st;
  return SUBSPACE_CRC_OK;
}

const char* fault_text(u32 f) {
  if (f & kFaultTicket) return "a look-back scan ticket was beyond its grid (stale scan state)";
  if (f & kFaultLookbackSpin) return "a look-back scan predecessor never published (stale scan state)";
  if (f & kFaultSlotRing) return "a fused slot kernel finishing wave never received a payload CRC";
  return "unknown fault";
}

// Read (after synchronising st) and clear the context's fault word; EFAULT if it was set. The
// scan state and the slot counters are reset before the next call.
int fault_status(subspace_crc_ctx* c, hipStream_t st) {
  u32 f = 0;
  HIP_TRY(hipMemcpyAsync(&f, c->d_fault, sizeof(u32), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (f == 0) return SUBSPACE_CRC_OK;
  if (f & kFaultSlotRing) {
    // (rarest path) a fused slot kernel gave up on its ring: its counter word may be left
    // non-zero, and fused slot kernels of this context on other streams (they record nothing)
    // may still hold the others -- let every stream finish before the counters are reset
    // (ADVICE r03), then report everything raised
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(&f, c->d_fault, sizeof(u32), hipMemcpyDeviceToHost));
    HIP_TRY(hipMemset(c->d_slot_counter, 0, kSlotCounters * kCountWords * sizeof(u64)));
    HIP_TRY(hipDeviceSynchronize());
  }
  // a scan fault: the scan kernels of this context run on the workspace stream, which st
  // follows (use_workspace) -- the reset is ordered on st, no device-wide synchronisation (a
  // hipDeviceSynchronize would stall other contexts' streams and break another thread's
  // global-mode graph capture). A bit raised by a kernel still running elsewhere
  // is reported by the next check.
  // Only word[0] (the kFault* bits): word[1], the generation mark of a faulted scan, stays
  // until a later scan of that generation clears it (a graph replay's first scan) or the
  // context moves on to a new generation (every non-graph call). Clearing it here would let
  // a replay still running on another stream -- graph replays record no workspace event, so
  // the check cannot wait for them -- stop skipping and index with its untrusted tile_base
  // (ADVICE r05).
  HIP_TRY(hipMemsetAsync(c->d_fault, 0, sizeof(u32), st));
  HIP_TRY(hipStreamSynchronize(st));
  c->scan_dirty = true;
  return fail(SUBSPACE_CRC_EFAULT, "device fault 0x%x: %s; the results of the calls since the last check are not valid",
              f, fault_text(f));
}

// Geometry of the wave-major tile values of the persistent ragged / long kernels: nw waves,
// nkmax values per wave, segments of 64 tiles of one sweep row (crc_combine.hip).
struct TileGeom {
  u64 nw, nkmax, nwb, nseg, nblk;
};
TileGeom tile_geom(const subspace_crc_ctx* c, u64 tiles) {
  TileGeom g;
  g.nw = (u64)c->num_cus * (kRaggedWG / 64);
  g.nkmax = ceil_div(tiles ? tiles : 1, g.nw);
  g.nwb = ceil_div(g.nw, 64);
  g.nseg = g.nkmax * g.nwb;
  g.nblk = ceil_div(g.nkmax, 64) * g.nwb;  // 64 x 64 blocks of the tile values and prefixes
  return g;
}

int ensure_ragged_ws(subspace_crc_ctx* c, u64 messages, u64 tiles) {
  bool state = false;
  if (messages > c->ws_messages) {
    (void)hipFree(c->d_tbase);
    c->d_tbase = nullptr;
    c->ws_messages = 0;
    HIP_TRY(hipMalloc(&c->d_tbase, (messages + 1) * sizeof(u64)));
    c->ws_messages = messages;
    state = true;
  }
  if (tiles > c->desc_capacity) {
    (void)hipFree(c->d_desc);
    (void)hipFree(c->d_tilecrc);
    (void)hipFree(c->d_local);
    (void)hipFree(c->d_segx);
    c->d_desc = nullptr;
    c->d_tilecrc = c->d_local = c->d_segx = nullptr;
    c->desc_capacity = 0;
    const TileGeom g = tile_geom(c, tiles);
    HIP_TRY(hipMalloc(&c->d_desc, tiles * kTileDescBytes));
    // blocked (crc_device.h tilecrc_index): whole 64 x 64 blocks of (w, k)
    HIP_TRY(hipMalloc(&c->d_tilecrc, g.nblk * 4096 * sizeof(u32)));
    HIP_TRY(hipMalloc(&c->d_local, g.nblk * 4096 * sizeof(u32)));
    HIP_TRY(hipMalloc(&c->d_segx, g.nseg * sizeof(u32)));
    c->desc_capacity = tiles;
    state = true;
  }
  if (state || !c->d_scan_state) {
    (void)hipFree(c->d_scan_state);
    c->d_scan_state = nullptr;
    c->scan_a_words = ceil_div(c->ws_messages + 1, kCountTile);
    c->scan_b_words = ceil_div(tile_geom(c, c->desc_capacity).nseg, kScanTile);
    HIP_TRY(hipMalloc(&c->d_scan_state, (1 + c->scan_a_words + c->scan_b_words) * sizeof(u64)));
    HIP_TRY(hipMemset(c->d_scan_state, 0, (1 + c->scan_a_words + c->scan_b_words) * sizeof(u64)));
    // hipMemset runs on the null stream, which does not order non-blocking streams (the
    // host-slot pipeline's compute stream, a caller's): finish it before any scan can start
    // (a scan that ran first read a recycled allocation's stale ticket, r03ac)
    HIP_TRY(hipDeviceSynchronize());
    c->scan_dirty = false;
  }
  if (!c->d_overflow) {  // [0] overflow (written by every call), [1] wide batch (zero between calls)
    HIP_TRY(hipMalloc(&c->d_overflow, 16));
    HIP_TRY(hipMemset(c->d_overflow, 0, 16));
    HIP_TRY(hipDeviceSynchronize());  // the null stream does not order non-blocking streams
  }
  return SUBSPACE_CRC_OK;
}

// Before a call's first scan: a call that failed after a scan may have left state behind.
int scan_state_clean(subspace_crc_ctx* c, hipStream_t st) {
  if (c->scan_dirty) {
    HIP_TRY(hipMemsetAsync(c->d_scan_state, 0, (1 + c->scan_a_words + c->scan_b_words) * sizeof(u64), st));
    c->scan_dirty = false;
  }
  return SUBSPACE_CRC_OK;
}

// Descriptor capacity of a call: the caller's bound (exact for non-overlapping messages),
// limited to what device memory can hold plus a tile per message, and below 2^32 (tile
// indices are u32 in the combine). A batch with more tiles takes the overflow path.
u64 clamp_capacity(const subspace_crc_ctx* c, u64 cap, u64 count) {
  const u64 lim = std::min<u64>(c->mem_tiles + count + 1, (1ull << 32) - (1ull << 20));
  return std::min(cap, lim);
}

// The tile-value combine after a ragged or long kernel: segment scans of the wave-major
// values, then the look-back over the segment XORs. total_ptr: the device's tile count
// (ragged) or null (long: `tiles` exact).
// A new call generation for the look-back scans' fault marks (crc_device.h FaultRef).
FaultRef new_call_fault(subspace_crc_ctx* c) {
  if (++c->call_gen == 0) c->call_gen = 1;
  return FaultRef{c->d_fault, c->call_gen};
}

int combine_tiles(subspace_crc_ctx* c, const TileGeom& g, const u64* total_ptr, u64 tiles, FaultRef fr,
                  hipStream_t st) {
  const dim3 grid((unsigned)ceil_div(g.nkmax, 64), (unsigned)g.nwb);
  tile_segment_scan_kernel<<<grid, 256, 0, st>>>(c->d_tilecrc, (u32)g.nw, (u32)g.nkmax, (u32)g.nwb, total_ptr, tiles,
                                                  c->d_local, c->d_segx);
  HIP_TRY(hipGetLastError());
  u32* tickets = reinterpret_cast<u32*>(c->d_scan_state);
  segment_prefix_kernel<<<(unsigned)ceil_div(g.nseg, kScanTile), 256, 0, st>>>(
      c->d_segx, g.nseg, (u32)g.nw, (u32)g.nwb, total_ptr, tiles, c->d_scan_state + 1 + c->scan_a_words, tickets + 1,
      fr);
  HIP_TRY(hipGetLastError());
  return SUBSPACE_CRC_OK;
}

// Persistent grid: enough blocks for one wave per work unit, at most one block per CU.
int grid_for(subspace_crc_ctx* c, u64 work_units, int waves_per_block) {
  const u64 waves = work_units ? work_units : 1;
  u64 blocks = (waves + waves_per_block - 1) / waves_per_block;
  if (blocks > (u64)c->num_cus) blocks = c->num_cus;
  return (int)(blocks ? blocks : 1);
}

// Ragged path: per-message tile counts -> scan -> tile descriptors -> main kernel.
// Offsets/lengths are read with element strides (1 = plain arrays, 3 = slot records).
// `cap` sizes the descriptor workspace; a batch with more tiles takes the search path.
int ragged_run(subspace_crc_ctx* c, const uint8_t* base, u64 cap, const u64* offsets, u32 ostride, const u64* lengths,
               u32 lstride, u64 count, u32 init, u32 final_xor, u32* out, hipStream_t st, u64 arena) {
  int rc = use_workspace(c, st);
  if (rc) return rc;
  cap = clamp_capacity(c, cap, count);
  rc = ensure_ragged_ws(c, count, cap);
  if (rc) return rc;
  const TileGeom g = tile_geom(c, cap);
  const u64 n1 = count + 1;
  rc = scan_state_clean(c, st);
  if (rc) return rc;
  c->scan_dirty = true;  // until the final kernel is launched
  const FaultRef fr = new_call_fault(c);
  u32* tickets = reinterpret_cast<u32*>(c->d_scan_state);
  // a known arena of at most 2^37 bytes: every tile fits the 8-B descriptor (its start is below
  // the arena's end, its message shorter than the arena), so the tile-count scan writes the
  // descriptors itself (crc32_ragged_count_desc_kernel); a many-long-message batch (few
  // messages per tile: config D) keeps the separate kernel, whose rows share the long messages
  const bool fused = c->fused_prep && arena != 0 && arena <= (1ull << kDesc8StartBits) && cap / count <= 64;
  // absolute addresses (arena 0: slot lists past the small kernel's 4 KiB, S_large) with few
  // tiles per message: the same fused scan with 16-B descriptors (round 6)
  const bool fused16 = c->fused_prep && arena == 0 && cap / count <= 64;
  if (fused) {
    crc32_ragged_count_desc_kernel<<<(unsigned)ceil_div(n1, kCountTile), 1024, 0, st>>>(
        offsets, ostride, lengths, lstride, count, init, final_xor, c->d_tbase, out, c->zero_word, c->d_scan_state + 1,
        reinterpret_cast<u32*>(c->d_scan_state), cap, reinterpret_cast<TileDesc8*>(c->d_desc), c->d_overflow, fr);
    c->zero_word = nullptr;
    HIP_TRY(hipGetLastError());
  } else if (fused16) {
    crc32_ragged_count_desc16_kernel<<<(unsigned)ceil_div(n1, kCountTile), 1024, 0, st>>>(
        offsets, ostride, lengths, lstride, count, init, final_xor, c->d_tbase, out, c->zero_word, c->d_scan_state + 1,
        reinterpret_cast<u32*>(c->d_scan_state), cap, reinterpret_cast<TileDesc*>(c->d_desc), c->d_overflow, fr);
    c->zero_word = nullptr;
    HIP_TRY(hipGetLastError());
  } else {
    crc32_ragged_count_scan_kernel<<<(unsigned)ceil_div(n1, kCountTile), 256, 0, st>>>(
        offsets, ostride, lengths, lstride, count, init, final_xor, c->d_tbase, out, c->zero_word, c->d_scan_state + 1,
        reinterpret_cast<u32*>(c->d_scan_state), c->d_overflow + 1, fr);
    c->zero_word = nullptr;
    HIP_TRY(hipGetLastError());
    // one thread per message; rows of workgroups share the later tiles of long messages when a
    // batch has few messages for its tiles (config D: 256 x 8,192 tiles: 2,048 rows), up to ~8 Ki
    // waves and no more rows than tiles per message
    const u64 dx = ceil_div(count, 256), waves_x = ceil_div(count, 64);
    const u64 dy = std::max<u64>(1, std::min<u64>({4096, ceil_div(8192, waves_x), cap / count}));
    crc32_ragged_desc_kernel<<<dim3((unsigned)dx, (unsigned)dy), 256, 0, st>>>(
        offsets, ostride, lengths, lstride, c->d_tbase, count, cap, reinterpret_cast<TileDesc*>(c->d_desc),
        c->d_overflow, c->d_scan_state + 1, ceil_div(n1, kCountTile), tickets, fr);
    HIP_TRY(hipGetLastError());
  }
  const int blocks = c->num_cus;  // persistent: one 8-wave workgroup per CU
  HeadSeeds seeds;  // Z_r^{-1}(init), r = 0..15: the seed of a message's first line, mis = r
  seeds.v[0] = init;
  for (int r = 1; r < 16; r++) seeds.v[r] = apply(c->zinv1, seeds.v[r - 1]);
  crc32_ragged_kernel<kRaggedWG><<<blocks, kRaggedWG, ragged_lds_bytes(), st>>>(
      base, offsets, ostride, lengths, lstride, c->d_tbase, count, reinterpret_cast<const TileDesc*>(c->d_desc),
      c->d_overflow, c->d_tab, c->d_rops, seeds, out, c->d_tilecrc, (u32)g.nwb, c->d_scan_state + 1,
      ceil_div(n1, kCountTile), tickets, fr);
  HIP_TRY(hipGetLastError());
  // padded message CRC = XOR of its tiles' values = difference of two entries of their
  // XOR prefix (only the batch's real tiles are combined); the final kernel undoes the last
  // tile's zero padding and applies the final XOR
  rc = combine_tiles(c, g, c->d_tbase + count, cap, fr, st);
  if (rc) return rc;
  const u64 fb = SUBSPACE_FINAL_BLOCKS_PER_CU ? std::min<u64>(ceil_div(count, 1024), (u64)SUBSPACE_FINAL_BLOCKS_PER_CU * c->num_cus)
                                              : ceil_div(count, 1024);
  crc32_ragged_final_kernel<<<(unsigned)fb, 1024, 0, st>>>(
      c->d_tbase, offsets, ostride, lengths, lstride, count, c->d_local, c->d_segx, (u32)g.nw, (u32)g.nwb,
      c->d_overflow, c->d_rops, final_xor, out, c->d_scan_state + 1 + c->scan_a_words, ceil_div(g.nseg, kScanTile),
      tickets + 1, fr);
  HIP_TRY(hipGetLastError());
  c->scan_dirty = false;
  return SUBSPACE_CRC_OK;
}

// Messages of at most max_len bytes fit one half-tile of the small-message kernel: 4,096 if
// they start on 16-B boundaries, else 4,081 (the extended length adds offset & 15).
bool small_fits(u64 max_len, bool aligned16) { return max_len <= (aligned16 ? kSmallMaxExt : kSmallMaxExt - 15); }

// Lanes per message for the small-message kernel (crc_small.hip G): the smallest power of two
// whose 128-B lines hold `max_ext` extended bytes (a message's length + its start & 15), at
// most 32 (a half-tile). A longer message than the bound is still computed whole (long path).
u32 small_lanes(u64 max_ext) {
  if (max_ext == 0) return 32;  // (no bound given: the half-tile form; waves still repack)
  u32 g = 1;
  while (g < 32 && 128ull * g < max_ext) g <<= 1;
  return g;
}

// Small-message path (crc_small.hip): messages of at most 4 KiB in one kernel, g lanes (128-B
// lines) per message, 64 / g messages per tile (a message longer than its g lines is computed
// whole by its wave's flush). Same arguments and results as ragged_run (offsets == null: a
// uniform batch, message m at base + m * ustride, ulen bytes); with `slot` the kernel also
// finishes the slots (span terms, flag + checksum or status, mismatch count) and `out` is
// unused.
struct SmallSlot {
  const u64* prefixes;
  u32 pstride;
  u64 pdelta;
  u64 max_len;  // larger sizes: SUBSPACE_CRC_SLOT_OVERSIZE (~0: no bound)
  u32 mode;
  int32_t checksum_size, metadata_size;
  u32 *status, *crc_out, *error_count;
};
int small_run(subspace_crc_ctx* c, const uint8_t* base, const u64* offsets, u32 ostride, const u64* lengths,
              u32 lstride, u64 count, u32 init, u32 final_xor, u32* out, hipStream_t st,
              const SmallSlot* slot = nullptr, u32 g = 32, u64 ustride = 0, u64 ulen = 0) {
  SmallArgs a{};
  a.ustride = ustride;  // (offsets == null: a uniform batch)
  a.ulen = ulen;
  a.base = base;
  a.offsets = offsets;
  a.ostride = ostride;
  a.lengths = lengths;
  a.lstride = lstride;
  a.count = count;
  a.init = init;
  a.final_xor = final_xor;
  a.out = out;
  a.rops = c->d_rops;
  a.pow2 = c->d_pow2;
  a.probe = c->dev.probe;
  // one workgroup per CU, or more, so that no wave gets more than 32 tiles (G = 32: one ring
  // window, the kernel's in-loop flush then never runs: crc_small.hip); g lanes per message
  const bool probe = c->dev.probe && c->dev.small_slot;
  if (probe) g = 32;  // (the dev library's timestamp-recording instantiation is G = 32's)
  const u64 tiles = ceil_div(count, 64ull / g);
  // slot waves of the half-tile form take at most kRp2MaxTilesPerWave tiles (32 messages), so a
  // workgroup's messages fit the workgroup repack's LDS tables (crc_small.hip REPACK2)
  const u64 per_wave = slot && g == 32 ? kRp2MaxTilesPerWave : kSmallRingTiles;
  const unsigned blocks = (unsigned)std::max<u64>(grid_for(c, tiles, 8), ceil_div(tiles, 8ull * per_wave));
  const size_t lds = small_lds_bytes() + 16;  // + the mismatch word
  if (slot) {
    a.prefixes = slot->prefixes;
    a.pstride = slot->pstride;
    a.pdelta = slot->pdelta;
    a.max_len = slot->max_len;
    a.mode = slot->mode;
    a.checksum_size = (u32)slot->checksum_size;
    a.metadata_size = (u32)slot->metadata_size;
    a.status = slot->status;
    a.crc_out = slot->crc_out;
    a.error_count = slot->error_count;
    a.counter = c->d_slot_counter + kCountWords * (c->slot_counter_next++ % kSlotCounters);
    if (probe) {  // development hook (libsubspace_crc_dev.so: tools/small_timeline.py)
      HIP_TRY(c->dev.small_slot(blocks, lds, st, c->d_tab, c->d_laneops, a));
    } else {
      switch (g) {
#define SMALL_SLOT_CASE(G) \
  case G: crc32_small_kernel<512, true, false, G><<<blocks, 512, lds, st>>>(c->d_tab, c->d_laneops, a); break;
        SMALL_SLOT_CASE(1) SMALL_SLOT_CASE(2) SMALL_SLOT_CASE(4) SMALL_SLOT_CASE(8) SMALL_SLOT_CASE(16)
        default: crc32_small_kernel<512, true, false, 32><<<blocks, 512, lds, st>>>(c->d_tab, c->d_laneops, a);
#undef SMALL_SLOT_CASE
      }
    }
  } else {
    a.zero_word = c->zero_word;
    c->zero_word = nullptr;
    switch (g) {
#define SMALL_CASE(G) \
  case G: crc32_small_kernel<512, false, false, G><<<blocks, 512, lds, st>>>(c->d_tab, c->d_laneops, a); break;
      SMALL_CASE(1) SMALL_CASE(2) SMALL_CASE(4) SMALL_CASE(8) SMALL_CASE(16)
      default: crc32_small_kernel<512, false, false, 32><<<blocks, 512, lds, st>>>(c->d_tab, c->d_laneops, a);
#undef SMALL_CASE
    }
  }
  HIP_TRY(hipGetLastError());
  return SUBSPACE_CRC_OK;
}

// The fused small-slot kernel finishes slots whose checksum and metadata areas are at most
// kSlotFusedMaxMeta bytes each (its lanes without a slot read their spans from the 4 KiB
// step table); others take the small kernel + crc32_slot_finish_kernel.
bool small_slot_fused(int32_t checksum_size, int32_t metadata_size) {
  return (u32)checksum_size <= kSlotFusedMaxMeta && (u32)metadata_size <= kSlotFusedMaxMeta;
}

int ensure_slot_ws(subspace_crc_ctx* c, u64 count) {
  if (count <= c->s_capacity) return SUBSPACE_CRC_OK;
  (void)hipFree(c->d_crc0);
  (void)hipFree(c->d_soff);
  (void)hipFree(c->d_slen);
  c->d_crc0 = nullptr;
  c->d_soff = nullptr;
  c->d_slen = nullptr;
  c->s_capacity = 0;
  HIP_TRY(hipMalloc(&c->d_crc0, count * sizeof(u32)));
  HIP_TRY(hipMalloc(&c->d_soff, count * sizeof(u64)));
  HIP_TRY(hipMalloc(&c->d_slen, count * sizeof(u64)));
  c->s_capacity = count;
  return SUBSPACE_CRC_OK;
}

int check_slot_args(int32_t checksum_size, int32_t metadata_size, uint32_t mode) {
  if (mode != SUBSPACE_CRC_SLOT_CALCULATE && mode != SUBSPACE_CRC_SLOT_VERIFY)
    return fail(SUBSPACE_CRC_EINVAL, "unknown slot mode %u", mode);
  if (checksum_size < 4) return fail(SUBSPACE_CRC_EINVAL, "checksum_size %d < 4", checksum_size);
  if (metadata_size < 0) return fail(SUBSPACE_CRC_EINVAL, "metadata_size %d < 0", metadata_size);
  return SUBSPACE_CRC_OK;
}

// Payload kernels of a slot batch: the uniform or ragged launch zeroes the mismatch count
// (c->zero_word) on the way; slot_finish memsets it only if neither ran.
void want_zeroed(subspace_crc_ctx* c, u32* err) { c->zero_word = err; }
bool was_zeroed(subspace_crc_ctx* c, u32* err) {
  const bool z = err && c->zero_word == nullptr;
  c->zero_word = nullptr;
  return z;
}

int slot_finish(subspace_crc_ctx* c, const u64* slots, uint8_t* buf, u64 stride, const u64* sizes, u64 usize,
                u64 count, u64 max_len, int32_t cs, int32_t ms, u32 mode, u32* status, u32* err, hipStream_t st,
                u32* crc_out = nullptr, bool err_zeroed = false) {
  if (err && !err_zeroed) HIP_TRY(hipMemsetAsync(err, 0, sizeof(u32), st));
  crc32_slot_finish_kernel<<<(unsigned)((count + 255) / 256), 256, 0, st>>>(
      slots, buf, stride, sizes, usize, count, max_len, cs, ms, mode, c->d_crc0, c->d_tab, c->d_pow2, status, err,
      crc_out);
  HIP_TRY(hipGetLastError());
  return SUBSPACE_CRC_OK;
}

}  // namespace

extern "C" {

int subspace_crc_version(void) { return 100; }  // 0.1.0

const char* subspace_crc_last_error(void) { return g_err; }

int subspace_crc_ctx_create(int device, subspace_crc_ctx** out) {
  return subspace_crc_ctx_create_poly(device, SUBSPACE_CRC_POLY_IEEE, out);
}

int subspace_crc_ctx_create_poly(int device, uint32_t poly, subspace_crc_ctx** out) {
  g_err[0] = 0;
  if (!out) return fail(SUBSPACE_CRC_EINVAL, "out is null");
  *out = nullptr;
  // reflected form: bit 31 is the x^0 coefficient, which makes every Z_n invertible
  if (!(poly & 0x80000000u)) return fail(SUBSPACE_CRC_EINVAL, "polynomial 0x%08x has no x^0 term", poly);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    return fail(SUBSPACE_CRC_ENODEV, "no HIP device available");
  if (device < 0 || device >= ndev) return fail(SUBSPACE_CRC_EINVAL, "device %d out of range [0,%d)", device, ndev);
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(SUBSPACE_CRC_ENODEV, "device %d is %s, this library is built for gfx950", device, prop.gcnArchName);
  HIP_TRY(hipSetDevice(device));

  auto* c = new subspace_crc_ctx();
  c->layout_bytes = (uint32_t)sizeof(subspace_crc_ctx);
  c->device = device;
  c->num_cus = prop.multiProcessorCount;
  c->mem_tiles = (u64)prop.totalGlobalMem / 8192;
  c->poly = poly;
  c->host_tab = make_tables(poly);
  c->zinv1 = inverse(z_one(c->host_tab));

  std::vector<u32> tab(1024), pow2(64 * 128, 0u), laneops(kSmallLaneOpSlots * 128, 0u), rops(kRagOpWords, 0u);
  for (int k = 0; k < 4; k++)
    for (int b = 0; b < 256; b++) tab[k * 256 + b] = c->host_tab.t[k][b];

  {
    Mat32 z = z_one(c->host_tab);
    for (int k = 0; k < 64; k++, z = mul(z, z)) nibble_tables(z, &pow2[(size_t)k * 128]);
  }

  for (int sl = 0; sl < 32; sl++) {
    u32 nt[128];
    nibble_tables(z_bytes(c->host_tab, 128ull * sl), nt);
    for (int k = 0; k < 8; k++)
      for (int n = 0; n < 16; n++) laneops[((size_t)k * 16 + n) * 32 + sl] = nt[k * 16 + n];
  }
  // ragged kernel: the line-shift operators, Z_4096, Z_{8192 * 2^k} for k = 0..20, Z_64 (x4)
  // -- the LDS part -- then Z_{8192 * 2^k} for k = 21..30 (crc_device.h ragged layout)
  std::copy(laneops.begin(), laneops.begin() + kLaneOpWords, rops.begin());
  nibble_tables(z_bytes(c->host_tab, 4096), &laneops[128 * kUniSlotOpZ4096]);
  {  // Z_64, replicated 4x as [nibble k][value n][copy] (crc_device.h kUniSlotOpZ64)
    u32 nt[128];
    nibble_tables(z_bytes(c->host_tab, 64), nt);
    for (int k = 0; k < 8; k++)
      for (int n = 0; n < 16; n++)
        for (int cp = 0; cp < 4; cp++) laneops[128 * kUniSlotOpZ64 + k * 64 + n * 4 + cp] = nt[k * 16 + n];
  }
  nibble_tables(z_bytes(c->host_tab, 4096), &rops[kLaneOpWords]);
  for (int k = 0; k < 31; k++)
    nibble_tables(z_bytes(c->host_tab, 8192ull << k),
                  &rops[k < kNumTileOps ? kLaneOpWords + 128 * (1 + k) : kRagHighOps + 128 * (k - kNumTileOps)]);
  {  // Z_64 replicated 4x, the same table as the uniform kernel's slots 33..36
    std::copy(laneops.begin() + 128 * kUniSlotOpZ64, laneops.begin() + 128 * (kUniSlotOpZ64 + 4), rops.begin() + kRagZ64Words);
  }
  // the ragged final kernel's padding inverses Z_{2^b}^{-1}, b = 0..12; the small-message
  // kernel's (b = 0..11) after the uniform kernel's slots
  for (int b = 0; b < kNumInvOps; b++)
    nibble_tables(inverse(z_bytes(c->host_tab, 1ull << b)), &rops[kRagInvOps + 128 * b]);
  std::copy(rops.begin() + kRagInvOps, rops.begin() + kRagInvOps + 128 * kSmallInvOps,
            laneops.begin() + 128 * kSmallOpInv);
  for (int j = 0; j < 5; j++)  // Z_{128 * 2^j}: the packed small-message forms' Z_C
    nibble_tables(z_bytes(c->host_tab, 128ull << j), &laneops[128 * (kSmallOpZC + j)]);
  for (int k = 0; k < 3; k++)
    for (u64 d = 1; d < 16; d++)
      nibble_tables(inverse(z_bytes(c->host_tab, d << (4 * k))), &rops[kRagNibInvOps + 128 * (15 * k + (int)d - 1)]);

  hipError_t e = hipMalloc(&c->d_tab, tab.size() * 4);
  if (e == hipSuccess) e = hipMalloc(&c->d_laneops, laneops.size() * 4);
  if (e == hipSuccess) e = hipMemcpy(c->d_laneops, laneops.data(), laneops.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(&c->d_rops, rops.size() * 4);
  if (e == hipSuccess) e = hipMalloc(&c->d_pow2, pow2.size() * 4);
  if (e == hipSuccess) e = hipMemcpy(c->d_pow2, pow2.data(), pow2.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->d_tab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(c->d_rops, rops.data(), rops.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)crc32_uniform4k_kernel<512, false, false>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)uniform_lds_bytes(8));
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)crc32_uniform4k_kernel<512, true, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)uniform_slot_lds_bytes(8));
  if (e == hipSuccess) e = hipMalloc(&c->d_slot_counter, kSlotCounters * kCountWords * sizeof(u64));
  if (e == hipSuccess) e = hipMemset(c->d_slot_counter, 0, kSlotCounters * kCountWords * sizeof(u64));
  if (e == hipSuccess) e = hipMalloc(&c->d_fault, 4 * sizeof(u32));
  if (e == hipSuccess) e = hipMemset(c->d_fault, 0, 4 * sizeof(u32));
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ws_done, hipEventDisableTiming);
  // the zeroed words above must be zero before a kernel on a non-blocking stream reads them
  if (e == hipSuccess) e = hipDeviceSynchronize();
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)crc32_ragged_kernel<kRaggedWG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)ragged_lds_bytes());
  if (e == hipSuccess)
    e = hipFuncSetAttribute((const void*)crc32_long_kernel<kRaggedWG>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)ragged_lds_bytes());
  {
    const void* small_fns[] = {
        (const void*)crc32_small_kernel<512, false, false, 1>,  (const void*)crc32_small_kernel<512, true, false, 1>,
        (const void*)crc32_small_kernel<512, false, false, 2>,  (const void*)crc32_small_kernel<512, true, false, 2>,
        (const void*)crc32_small_kernel<512, false, false, 4>,  (const void*)crc32_small_kernel<512, true, false, 4>,
        (const void*)crc32_small_kernel<512, false, false, 8>,  (const void*)crc32_small_kernel<512, true, false, 8>,
        (const void*)crc32_small_kernel<512, false, false, 16>, (const void*)crc32_small_kernel<512, true, false, 16>,
        (const void*)crc32_small_kernel<512, false, false, 32>, (const void*)crc32_small_kernel<512, true, false, 32>};
    for (const void* f : small_fns)
      if (e == hipSuccess)
        e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)small_lds_bytes() + 16);
  }
  if (e != hipSuccess) {
    subspace_crc_ctx_destroy(c);
    return hip_fail(e, "context setup");
  }
  *out = c;
  return SUBSPACE_CRC_OK;
}

void subspace_crc_ctx_destroy(subspace_crc_ctx* c) {
  if (!c) return;
  if (c->ws_done && c->ws_recorded) (void)hipEventSynchronize(c->ws_done);
  if (c->hcompute) (void)hipStreamSynchronize(c->hcompute);
  for (auto& h : c->hstage) {
    if (h.stream) (void)hipStreamSynchronize(h.stream);
    if (h.copied) (void)hipEventDestroy(h.copied);
    (void)hipFree(h.dbuf);
    (void)hipFree(h.dsizes);
    (void)hipFree(h.dres);
    (void)hipFree(h.derr);
    (void)hipHostFree(h.hres);
    (void)hipHostFree(h.herr);
    if (h.done) (void)hipEventDestroy(h.done);
    if (h.stream) (void)hipStreamDestroy(h.stream);
  }
  if (c->hcompute) (void)hipStreamDestroy(c->hcompute);
  (void)hipHostFree(c->l_hrec);
  (void)hipFree(c->l_drec);
  (void)hipFree(c->l_dstatus);
  (void)hipHostFree(c->l_hstatus);
  (void)hipFree(c->d_tab);
  (void)hipFree(c->d_rops);
  (void)hipFree(c->d_pow2);
  (void)hipFree(c->d_laneops);
  (void)hipFree(c->d_crc0);
  (void)hipFree(c->d_soff);
  (void)hipFree(c->d_slen);
  (void)hipFree(c->d_tbase);
  (void)hipFree(c->d_desc);
  (void)hipFree(c->d_tilecrc);
  (void)hipFree(c->d_local);
  (void)hipFree(c->d_segx);
  (void)hipFree(c->d_scan_state);
  (void)hipFree(c->d_overflow);
  (void)hipFree(c->d_uoff);
  (void)hipFree(c->d_ulen);
  (void)hipFree(c->d_slot_counter);
  (void)hipFree(c->d_fault);
  if (c->ws_done) (void)hipEventDestroy(c->ws_done);
  delete c;
}

int subspace_crc_ctx_check(subspace_crc_ctx* c, void* stream) {
  g_err[0] = 0;
  if (!c) return fail(SUBSPACE_CRC_EINVAL, "ctx is null");
  CallScope scope(c);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  // the last workspace call may have run on another stream
  if (c->ws_recorded) HIP_TRY(hipEventSynchronize(c->ws_done));
  return fault_status(c, st);
}

int subspace_crc_ctx_reserve(subspace_crc_ctx* c, uint64_t max_messages, uint64_t max_tiles) {
  g_err[0] = 0;
  if (!c) return fail(SUBSPACE_CRC_EINVAL, "ctx is null");
  CallScope scope(c);
  HIP_TRY(hipSetDevice(c->device));
  return ensure_ragged_ws(c, max_messages, clamp_capacity(c, max_tiles, max_messages));
}

int subspace_crc32_batch(subspace_crc_ctx* c, const void* dev_base, uint64_t arena_bytes, const uint64_t* dev_offsets,
                         const uint64_t* dev_lengths, uint64_t count, uint32_t init, uint32_t flags,
                         uint32_t* dev_out, void* stream) {
  g_err[0] = 0;
  if (!c) return fail(SUBSPACE_CRC_EINVAL, "ctx is null");
  if (count == 0) return SUBSPACE_CRC_OK;
  CallScope scope(c);
  if (!dev_base || !dev_offsets || !dev_lengths || !dev_out)
    return fail(SUBSPACE_CRC_EINVAL, "null device pointer");
  if (flags & ~SUBSPACE_CRC_FINALIZE) return fail(SUBSPACE_CRC_EINVAL, "unknown flags 0x%x", flags);
  if (count >= (1ull << 32)) return fail(SUBSPACE_CRC_EINVAL, "count %llu exceeds 2^32-1", (unsigned long long)count);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const u32 final_xor = (flags & SUBSPACE_CRC_FINALIZE) ? 0xFFFFFFFFu : 0u;
  // Tile capacity: exact for non-overlapping messages inside the arena; if the device
  // finds more tiles (overlapping messages) the kernel falls back to per-tile search.
  // (a message's tiles cover its extended length L + (offset & 15))
  const u64 cap = (arena_bytes + 15 * count) / 8192 + count + 1;
  return ragged_run(c, static_cast<const uint8_t*>(dev_base), cap, dev_offsets, 1, dev_lengths, 1, count, init,
                    final_xor, dev_out, st, arena_bytes);
}

int subspace_crc32_batch_uniform(subspace_crc_ctx* c, const void* dev_base, uint64_t stride, uint64_t length,
                                 uint64_t count, uint32_t init, uint32_t flags, uint32_t* dev_out, void* stream) {
  g_err[0] = 0;
  if (!c) return fail(SUBSPACE_CRC_EINVAL, "ctx is null");
  if (count == 0) return SUBSPACE_CRC_OK;
  CallScope scope(c);
  if (!dev_base || !dev_out) return fail(SUBSPACE_CRC_EINVAL, "null device pointer");
  if (flags & ~SUBSPACE_CRC_FINALIZE) return fail(SUBSPACE_CRC_EINVAL, "unknown flags 0x%x", flags);
  if (stride < length && count > 1) return fail(SUBSPACE_CRC_EINVAL, "stride %llu < length %llu",
                                                (unsigned long long)stride, (unsigned long long)length);
  HIP_TRY(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const u32 final_xor = (flags & SUBSPACE_CRC_FINALIZE) ? 0xFFFFFFFFu : 0u;
  const bool fast = length == 4096 && (stride % 16) == 0 && ((uintptr_t)dev_base % 16) == 0;
  if (fast) {
    const u64 tiles = (count + 1) / 2;
    int blocks = grid_for(c, tiles, 8);
    if (c->uniform_blocks > 0 && (u64)c->uniform_blocks < (u64)blocks) blocks = c->uniform_blocks;
    const auto* b = static_cast<const uint8_t*>(dev_base);
    const int ord = c->uniform_order;
    if (c->dev.probe && c->dev.uniform) {  // development hook (libsubspace_crc_dev.so: tools/wave_timeline.py)
      SlotArgs sa{};
      sa.probe = c->dev.probe;
      HIP_TRY(c->dev.uniform(false, (unsigned)grid_for(c, tiles, 8), st, b, stride, count, c->d_tab, c->d_laneops, init,
                             final_xor, dev_out, c->zero_word, sa));
      c->zero_word = nullptr;
      return SUBSPACE_CRC_OK;
    }
    crc32_uniform4k_kernel<512, false, false><<<blocks, 512, uniform_lds_bytes(8), st>>>(
        b, stride, count, c->d_tab, c->d_laneops, init, final_xor, dev_out, ord, c->zero_word, SlotArgs{});
    c->zero_word = nullptr;
    HIP_TRY(hipGetLastError());
    return SUBSPACE_CRC_OK;
  }
  // Long messages in whole 8 KiB pieces, 16-B aligned (config D): the long-message kernel
  // (implicit tiles, plain loads), then the segment-scan combine of the ragged path (crc_combine.hip).
  const u64 pieces = length / 8192;
  const bool long_fast = length >= 8192 && length % 8192 == 0 && (stride % 16) == 0 &&
                         ((uintptr_t)dev_base % 16) == 0 && pieces <= (1ull << kNumTileOps) &&
                         count < (1ull << 32) && pieces * count < (1ull << 32);
  if (long_fast && c->long_path) {
    const u64 tiles = pieces * count;
    int rc = use_workspace(c, st);
    if (rc) return rc;
    rc = ensure_ragged_ws(c, 0, tiles);
    if (rc) return rc;
    const TileGeom g = tile_geom(c, tiles);
    rc = scan_state_clean(c, st);
    if (rc) return rc;
    c->scan_dirty = true;  // until the final kernel is launched
    crc32_long_kernel<kRaggedWG><<<c->num_cus, kRaggedWG, ragged_lds_bytes(), st>>>(
        static_cast<const uint8_t*>(dev_base), stride, (u32)pieces, (u32)count, c->d_tab, c->d_rops, init, final_xor,
        c->d_tilecrc, (u32)g.nwb);
    HIP_TRY(hipGetLastError());
    rc = combine_tiles(c, g, nullptr, tiles, new_call_fault(c), st);
    if (rc) return rc;
    crc32_long_final_kernel<<<(unsigned)ceil_div(count, 256), 256, 0, st>>>(
        c->d_local, c->d_segx, (u32)g.nw, (u32)g.nwb, (u32)pieces, (u32)count, dev_out,
        c->d_scan_state + 1 + c->scan_a_words, ceil_div(g.nseg, kScanTile), reinterpret_cast<u32*>(c->d_scan_state) + 1);
    HIP_TRY(hipGetLastError());
    c->scan_dirty = false;
    return SUBSPACE_CRC_OK;
  }
  // Messages of at most 4 KiB: the small-message kernel straight from stride and length (no
  // record arrays, no workspace).
  const bool aligned = (stride % 16) == 0 && ((uintptr_t)dev_base % 16) == 0;
  if (small_fits(length, aligned) && c->small_path && count > 1)
    return small_run(c, static_cast<const uint8_t*>(dev_base), nullptr, 0, nullptr, 0, count, init, final_xor,
                     dev_out, st, nullptr, small_lanes(length + (aligned ? 0 : 15)), stride, length);
  // Any other shape: materialise offsets/lengths (context workspace: ordered after the last
  // workspace call first) and take the ragged path.
  int rc = use_workspace(c, st);
  if (rc) return rc;
  if (count > c->u_capacity) {
    (void)hipFree(c->d_uoff);
    (void)hipFree(c->d_ulen);
    c->d_uoff = c->d_ulen = nullptr;
    c->u_capacity = 0;
    HIP_TRY(hipMalloc(&c->d_uoff, count * sizeof(u64)));
    HIP_TRY(hipMalloc(&c->d_ulen, count * sizeof(u64)));
    c->u_capacity = count;
  }
  uniform_offsets_kernel<<<(unsigned)((count + 255) / 256), 256, 0, st>>>(stride, length, count, c->d_uoff,
                                                                           c->d_ulen);
  HIP_TRY(hipGetLastError());
  const u64 arena = stride * (count - 1) + length;
  return subspace_crc32_batch(c, dev_base, arena, c->d_uoff, c->d_ulen, count, init, flags, dev_out, stream);
}

int subspace_crc32_slots(subspace_crc_ctx* c, const subspace_crc_slot* dev_slots, uint64_t count,
                         uint64_t max_message_size, int32_t checksum_size, int32_t metadata_size, uint32_t mode,
                         uint32_t* dev_status, uint32_t* dev_error_count, void* stream) {
  g_err[0] = 0;
  if (!c) return fail(SUBSPACE_CRC_EINVAL, "ctx is null");
  CallScope scope(c);
  int rc = check_slot_args(checksum_size, metadata_size, mode);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (count == 0) {
    if (dev_error_count) HIP_TRY(hipMemsetAsync(dev_error_count, 0, sizeof(u32), st));
    return SUBSPACE_CRC_OK;
  }
  if (!dev_slots) return fail(SUBSPACE_CRC_EINVAL, "null device pointer");
  if (count >= (1ull << 32)) return fail(SUBSPACE_CRC_EINVAL, "count %llu exceeds 2^32-1", (unsigned long long)count);
  HIP_TRY(hipSetDevice(c->device));
  // payload CRCs from init 0 at absolute addresses (base 0; fields 1 and 2 of each record):
  // slots of at most 4 KiB through the small-message kernel, larger ones the ragged path
  const u64* rec = reinterpret_cast<const u64*>(dev_slots);
  const bool small = max_message_size <= kSmallMaxExt && c->small_path;
  if (small && small_slot_fused(checksum_size, metadata_size)) {
    // one kernel, the slots finished in it; no context workspace (the counter ring, as the
    // fused uniform slot kernel)
    // (lanes per slot from the bound: payloads of a channel's slots start on 16-B boundaries; one
    // that does not and overruns its lines is still computed whole)
    const SmallSlot ss{rec, 3, 0, ~0ull, mode, checksum_size, metadata_size, dev_status, nullptr, dev_error_count};
    return small_run(c, nullptr, rec + 1, 3, rec + 2, 3, count, 0u, 0u, nullptr, st, &ss, small_lanes(max_message_size));
  }
  rc = use_workspace(c, st);
  if (rc) return rc;
  rc = ensure_slot_ws(c, count);
  if (rc) return rc;
  want_zeroed(c, dev_error_count);
  if (small) {
    rc = small_run(c, nullptr, rec + 1, 3, rec + 2, 3, count, 0u, 0u, c->d_crc0, st, nullptr,
                   small_lanes(max_message_size));
  } else {
    const u64 cap = count * ((max_message_size + 15 + 8191) / 8192) + 1;
    rc = ragged_run(c, nullptr, cap, rec + 1, 3, rec + 2, 3, count, 0u, 0u, c->d_crc0, st, 0);  // absolute addresses
  }
  const bool zeroed = was_zeroed(c, dev_error_count);
  if (rc) return rc;
  return slot_finish(c, rec, nullptr, 0, nullptr, 0, count, ~0ull, checksum_size, metadata_size, mode, dev_status,
                     dev_error_count, st, nullptr, zeroed);
}

}  // extern "C"

namespace {

// Device-buffer strided slots (subspace_crc32_slots_strided), with an optional compact copy
// of the stored checksums (the host-slot path's write-back source).
int slots_strided_impl(subspace_crc_ctx* c, void* dev_buffer, uint64_t slot_stride, uint64_t count,
                       uint64_t message_size, const uint64_t* dev_message_sizes, int32_t checksum_size,
                       int32_t metadata_size, uint32_t mode, uint32_t* dev_status, uint32_t* dev_error_count,
                       u32* dev_crc_out, hipStream_t st) {
  int rc = check_slot_args(checksum_size, metadata_size, mode);
  if (rc) return rc;
  if (count == 0) {
    if (dev_error_count) HIP_TRY(hipMemsetAsync(dev_error_count, 0, sizeof(u32), st));
    return SUBSPACE_CRC_OK;
  }
  if (!dev_buffer) return fail(SUBSPACE_CRC_EINVAL, "null device pointer");
  if (((uintptr_t)dev_buffer % 8) || (slot_stride % 8))
    return fail(SUBSPACE_CRC_EINVAL, "prefixes must be 8-B aligned (buffer %p, stride %llu)", dev_buffer,
                (unsigned long long)slot_stride);
  if (count >= (1ull << 32)) return fail(SUBSPACE_CRC_EINVAL, "count %llu exceeds 2^32-1", (unsigned long long)count);
  // ComputePrefixSize (common/channel.h:914-919)
  const u64 prefix_size = ((u64)(48 + checksum_size + metadata_size) + 63) & ~63ull;
  if (!dev_message_sizes && slot_stride < prefix_size + message_size && count > 1)
    return fail(SUBSPACE_CRC_EINVAL, "slot_stride %llu < prefix %llu + message %llu",
                (unsigned long long)slot_stride, (unsigned long long)prefix_size, (unsigned long long)message_size);
  if (dev_message_sizes && slot_stride < prefix_size && count > 1)
    return fail(SUBSPACE_CRC_EINVAL, "slot_stride %llu < prefix %llu", (unsigned long long)slot_stride,
                (unsigned long long)prefix_size);
  HIP_TRY(hipSetDevice(c->device));
  auto* buf = static_cast<uint8_t*>(dev_buffer);
  // Fused path (crc_uniform.hip SLOT): 4 KiB payloads, 16-B aligned, no metadata span -- the
  // payload CRC, the span-0 term and the flag/checksum store or status in one kernel
  if (!dev_message_sizes && message_size == 4096 && (u32)metadata_size <= kSlotFusedMaxMeta && slot_stride % 16 == 0 &&
      ((uintptr_t)(buf + prefix_size) % 16) == 0 && c->fused_slots) {
    // 8 waves per workgroup, tile order 0 (the finishing waves replay it), and at most
    // kSlotRingRounds tiles per wave (a workgroup is one ring window): more workgroups than
    // CUs for channels above 256 x 8 x 32 tiles
    const u64 tiles = (count + 1) / 2;
    const u64 blocks = std::max<u64>(grid_for(c, tiles, 512 / 64), ceil_div(tiles, 8ull * kSlotRingRounds));
    SlotArgs sa{prefix_size, mode, dev_status, dev_crc_out, dev_error_count,
                c->d_slot_counter + kCountWords * (c->slot_counter_next++ % kSlotCounters), c->dev.probe, c->d_fault,
                (u32)checksum_size, (u32)metadata_size};
    if (c->dev.probe && c->dev.uniform)  // development hook (libsubspace_crc_dev.so)
      HIP_TRY(c->dev.uniform(true, (unsigned)blocks, st, buf + prefix_size, slot_stride, count, c->d_tab, c->d_laneops,
                             0u, 0xFFFFFFFFu, nullptr, nullptr, sa));
    else
      crc32_uniform4k_kernel<512, true, false><<<(unsigned)blocks, 512, uniform_slot_lds_bytes(8), st>>>(
          buf + prefix_size, slot_stride, count, c->d_tab, c->d_laneops, 0u, 0xFFFFFFFFu, nullptr, 0, nullptr, sa);
    HIP_TRY(hipGetLastError());
    return SUBSPACE_CRC_OK;
  }
  rc = use_workspace(c, st);
  if (rc) return rc;
  rc = ensure_slot_ws(c, count);
  if (rc) return rc;
  want_zeroed(c, dev_error_count);
  if (dev_message_sizes) {
    // payload offsets, and the sizes with every one beyond the slot's payload area as 0: the
    // payload kernels read nothing of an oversize slot (its bytes would run into the next slot
    // or past the buffer), slot_finish labels it from the raw sizes
    const u64 area = count > 1 ? slot_stride - prefix_size : ~0ull;
    slot_payload_offsets_kernel<<<(unsigned)((count + 255) / 256), 256, 0, st>>>(
        slot_stride, prefix_size, count, c->d_soff, dev_message_sizes, area, c->d_slen);
    HIP_TRY(hipGetLastError());
    const bool aligned = slot_stride % 16 == 0 && ((uintptr_t)(buf + prefix_size) % 16) == 0;
    if (count > 1 && small_fits(slot_stride - prefix_size, aligned) && c->small_path) {
      // slots of at most 4 KiB (a size beyond the slot's payload area is OVERSIZE); the prefix
      // of slot i is its payload offset - prefix_size
      if (small_slot_fused(checksum_size, metadata_size)) {
        was_zeroed(c, dev_error_count);  // the fused kernel writes the count itself
        const SmallSlot ss{c->d_soff, 1, prefix_size, slot_stride - prefix_size, mode, checksum_size, metadata_size,
                           dev_status, dev_crc_out, dev_error_count};
        return small_run(c, buf, c->d_soff, 1, dev_message_sizes, 1, count, 0u, 0u, nullptr, st, &ss,
                         small_lanes(slot_stride - prefix_size + (aligned ? 0 : 15)));
      }
      rc = small_run(c, buf, c->d_soff, 1, c->d_slen, 1, count, 0u, 0u, c->d_crc0, st, nullptr,
                     small_lanes(slot_stride - prefix_size + (aligned ? 0 : 15)));
    } else {
      const u64 cap = (slot_stride * count + 15 * count) / 8192 + count + 1;
      rc = ragged_run(c, buf, cap, c->d_soff, 1, c->d_slen, 1, count, 0u, 0u, c->d_crc0, st,
                      slot_stride * count);
    }
  } else {
    rc = subspace_crc32_batch_uniform(c, buf + prefix_size, slot_stride, message_size, count, 0u, 0u, c->d_crc0,
                                      st);
  }
  const bool zeroed = was_zeroed(c, dev_error_count);
  if (rc) return rc;
  // a per-slot size beyond the payload area: SUBSPACE_CRC_SLOT_OVERSIZE (one slot: no bound)
  const u64 max_len = dev_message_sizes && count > 1 ? slot_stride - prefix_size : ~0ull;
  return slot_finish(c, nullptr, buf, slot_stride, dev_message_sizes, message_size, count, max_len, checksum_size,
                     metadata_size, mode, dev_status, dev_error_count, st, dev_crc_out, zeroed);
}

}  // namespace

extern "C" {

int subspace_crc32_slots_strided(subspace_crc_ctx* c, void* dev_buffer, uint64_t slot_stride, uint64_t count,
                                 uint64_t message_size, const uint64_t* dev_message_sizes, int32_t checksum_size,
                                 int32_t metadata_size, uint32_t mode, uint32_t* dev_status,
                                 uint32_t* dev_error_count, void* stream) {
  g_err[0] = 0;
  if (!c) return fail(SUBSPACE_CRC_EINVAL, "ctx is null");
  CallScope scope(c);
  return slots_strided_impl(c, dev_buffer, slot_stride, count, message_size, dev_message_sizes, checksum_size,
                            metadata_size, mode, dev_status, dev_error_count, nullptr, (hipStream_t)stream);
}

// ------------------------------------------------------------------ host-memory slots
int subspace_crc_host_register(void* ptr, uint64_t bytes) {
  g_err[0] = 0;
  if (!ptr || !bytes) return fail(SUBSPACE_CRC_EINVAL, "null pointer or zero size");
  HIP_TRY(hipHostRegister(ptr, bytes, hipHostRegisterMapped | hipHostRegisterPortable));
  void* dev = nullptr;
  hipError_t e = hipHostGetDevicePointer(&dev, ptr, 0);
  if (e != hipSuccess) {
    (void)hipHostUnregister(ptr);
    return hip_fail(e, "hipHostGetDevicePointer");
  }
  std::lock_guard<std::mutex> lock(g_regions_mu);
  g_regions.push_back({reinterpret_cast<uintptr_t>(ptr), bytes, reinterpret_cast<uintptr_t>(dev)});
  return SUBSPACE_CRC_OK;
}

int subspace_crc_host_unregister(void* ptr) {
  g_err[0] = 0;
  if (!ptr) return fail(SUBSPACE_CRC_EINVAL, "null pointer");
  {
    std::lock_guard<std::mutex> lock(g_regions_mu);
    for (size_t i = 0; i < g_regions.size(); i++)
      if (g_regions[i].host == reinterpret_cast<uintptr_t>(ptr)) {
        g_regions.erase(g_regions.begin() + (long)i);
        break;
      }
  }
  HIP_TRY(hipHostUnregister(ptr));
  return SUBSPACE_CRC_OK;
}

}  // extern "C"

namespace {

int ensure_host_stage(subspace_crc_ctx* c, u64 bytes, u64 slots) {
  if (!c->hcompute) HIP_TRY(hipStreamCreateWithFlags(&c->hcompute, hipStreamNonBlocking));
  for (auto& h : c->hstage) {
    if (!h.stream) HIP_TRY(hipStreamCreateWithFlags(&h.stream, hipStreamNonBlocking));
    if (!h.copied) HIP_TRY(hipEventCreateWithFlags(&h.copied, hipEventDisableTiming));
    if (!h.done) HIP_TRY(hipEventCreateWithFlags(&h.done, hipEventDisableTiming));
  }
  if (bytes > c->h_bytes) {
    for (auto& h : c->hstage) {
      (void)hipFree(h.dbuf);
      h.dbuf = nullptr;
    }
    c->h_bytes = 0;
    for (auto& h : c->hstage) HIP_TRY(hipMalloc(&h.dbuf, bytes));
    c->h_bytes = bytes;
  }
  if (slots > c->h_slots) {
    for (auto& h : c->hstage) {
      (void)hipFree(h.dsizes);
      (void)hipFree(h.dres);
      (void)hipFree(h.derr);
      (void)hipHostFree(h.hres);
      (void)hipHostFree(h.herr);
      h.dsizes = nullptr;
      h.dres = h.derr = h.hres = h.herr = nullptr;
    }
    c->h_slots = 0;
    for (auto& h : c->hstage) {
      HIP_TRY(hipMalloc(&h.dsizes, slots * sizeof(u64)));
      HIP_TRY(hipMalloc(&h.dres, slots * sizeof(u32)));
      HIP_TRY(hipMalloc(&h.derr, sizeof(u32)));
      HIP_TRY(hipHostMalloc(&h.hres, slots * sizeof(u32), hipHostMallocDefault));
      HIP_TRY(hipHostMalloc(&h.herr, sizeof(u32), hipHostMallocDefault));
    }
    c->h_slots = slots;
  }
  return SUBSPACE_CRC_OK;
}

// Host side of a finished chunk: CALCULATE writes kMessageHasChecksum and the checksum into
// each host prefix (what the device computed them with); VERIFY copies the statuses out.
void host_writeback(const subspace_crc_ctx::HostStage& h, uint8_t* host, u64 stride, u64 first, u64 n, u32 mode,
                    uint32_t* host_status, u64* errors) {
  if (mode == SUBSPACE_CRC_SLOT_CALCULATE) {
    for (u64 i = 0; i < n; i++) {
      uint8_t* prefix = host + (first + i) * stride;
      int64_t flags;
      std::memcpy(&flags, prefix + 32, sizeof(flags));  // MessagePrefix::flags (common/channel.h:88-112)
      flags |= 4;                                        // kMessageHasChecksum
      std::memcpy(prefix + 32, &flags, sizeof(flags));
      std::memcpy(prefix + 48, &h.hres[i], sizeof(u32)); // checksum area, first 4 B
      if (host_status) host_status[first + i] = SUBSPACE_CRC_SLOT_OK;
    }
  } else {
    if (host_status) std::memcpy(host_status + first, h.hres, n * sizeof(u32));
    *errors += *h.herr;
  }
}

}  // namespace

extern "C" {

int subspace_crc32_host_slots(subspace_crc_ctx* c, void* host_buffer, uint64_t slot_stride, uint64_t count,
                              uint64_t message_size, const uint64_t* host_message_sizes, int32_t checksum_size,
                              int32_t metadata_size, uint32_t mode, uint32_t* host_status,
                              uint32_t* host_error_count) {
  g_err[0] = 0;
  if (!c) return fail(SUBSPACE_CRC_EINVAL, "ctx is null");
  CallScope scope(c);
  int rc = check_slot_args(checksum_size, metadata_size, mode);
  if (rc) return rc;
  if (host_error_count) *host_error_count = 0;
  if (count == 0) return SUBSPACE_CRC_OK;
  if (!host_buffer) return fail(SUBSPACE_CRC_EINVAL, "null host buffer");
  if (((uintptr_t)host_buffer % 8) || (slot_stride % 8))
    return fail(SUBSPACE_CRC_EINVAL, "prefixes must be 8-B aligned (buffer %p, stride %llu)", host_buffer,
                (unsigned long long)slot_stride);
  const u64 prefix_size = ((u64)(48 + checksum_size + metadata_size) + 63) & ~63ull;
  if (!host_message_sizes && slot_stride < prefix_size + message_size)
    return fail(SUBSPACE_CRC_EINVAL, "slot_stride %llu < prefix %llu + message %llu",
                (unsigned long long)slot_stride, (unsigned long long)prefix_size, (unsigned long long)message_size);
  if (host_message_sizes)
    for (u64 i = 0; i < count; i++)
      if (prefix_size + host_message_sizes[i] > slot_stride)
        return fail(SUBSPACE_CRC_EINVAL, "slot %llu: message size %llu does not fit the slot stride %llu",
                    (unsigned long long)i, (unsigned long long)host_message_sizes[i],
                    (unsigned long long)slot_stride);
  HIP_TRY(hipSetDevice(c->device));
  // ~32 MiB chunks: each H2D copy is long enough to run at the link rate, and two chunks
  // in flight let one chunk's copy overlap the previous chunk's kernels.
  const u64 chunk = std::max<u64>(1, std::min<u64>(count, (32ull << 20) / slot_stride));
  rc = ensure_host_stage(c, chunk * slot_stride, chunk);
  if (rc) return rc;
  rc = use_workspace(c, c->hcompute);  // the staging buffers and the slot workspaces
  if (rc) return rc;
  auto* host = static_cast<uint8_t*>(host_buffer);
  const u64 nchunks = (count + chunk - 1) / chunk;
  u64 errors = 0;
  int first_rc = SUBSPACE_CRC_OK;
  for (u64 k = 0; k < nchunks + 2; k++) {
    auto& h = c->hstage[k & 1];
    if (k >= 2) {  // chunk k-2 used this stage: finish it on the host
      const u64 f = (k - 2) * chunk, n = std::min(chunk, count - f);
      hipError_t e = hipEventSynchronize(h.done);
      if (e != hipSuccess && !first_rc) first_rc = hip_fail(e, "hipEventSynchronize");
      if (!first_rc) host_writeback(h, host, slot_stride, f, n, mode, host_status, &errors);
    }
    if (k >= nchunks || first_rc) continue;
    const u64 f = k * chunk, n = std::min(chunk, count - f);
    hipError_t e = hipMemcpyAsync(h.dbuf, host + f * slot_stride, n * slot_stride, hipMemcpyHostToDevice, h.stream);
    if (e == hipSuccess && host_message_sizes)
      e = hipMemcpyAsync(h.dsizes, host_message_sizes + f, n * sizeof(u64), hipMemcpyHostToDevice, h.stream);
    if (e == hipSuccess) e = hipEventRecord(h.copied, h.stream);
    if (e == hipSuccess) e = hipStreamWaitEvent(c->hcompute, h.copied, 0);
    if (e != hipSuccess) {
      first_rc = hip_fail(e, "hipMemcpyAsync (host slots to device)");
      continue;
    }
    const bool calc = mode == SUBSPACE_CRC_SLOT_CALCULATE;
    rc = slots_strided_impl(c, h.dbuf, slot_stride, n, message_size, host_message_sizes ? h.dsizes : nullptr,
                            checksum_size, metadata_size, mode, calc ? nullptr : h.dres, calc ? nullptr : h.derr,
                            calc ? h.dres : nullptr, c->hcompute);
    if (rc) {
      first_rc = rc;
      continue;
    }
    e = hipMemcpyAsync(h.hres, h.dres, n * sizeof(u32), hipMemcpyDeviceToHost, c->hcompute);
    if (e == hipSuccess && !calc)
      e = hipMemcpyAsync(h.herr, h.derr, sizeof(u32), hipMemcpyDeviceToHost, c->hcompute);
    if (e == hipSuccess) e = hipEventRecord(h.done, c->hcompute);
    if (e != hipSuccess) first_rc = hip_fail(e, "hipMemcpyAsync (results to host)");
  }
  if (first_rc) {
    for (auto& h : c->hstage) (void)hipStreamSynchronize(h.stream);
    (void)hipStreamSynchronize(c->hcompute);
    return first_rc;
  }
  rc = fault_status(c, c->hcompute);
  if (rc) return rc;
  if (host_error_count) *host_error_count = (u32)errors;
  return SUBSPACE_CRC_OK;
}

// Zero-copy slot list in host memory (a subscriber drain): translate each record's host
// addresses to their device aliases, then the device slot path reads payloads and prefixes
// straight from host memory over PCIe; CALCULATE writes flag + checksum into the host
// prefixes through the same mapping.
int subspace_crc32_host_slot_list(subspace_crc_ctx* c, const subspace_crc_slot* host_slots, uint64_t count,
                                  uint64_t max_message_size, int32_t checksum_size, int32_t metadata_size,
                                  uint32_t mode, uint32_t* host_status, uint32_t* host_error_count) {
  g_err[0] = 0;
  if (!c) return fail(SUBSPACE_CRC_EINVAL, "ctx is null");
  CallScope scope(c);
  int rc = check_slot_args(checksum_size, metadata_size, mode);
  if (rc) return rc;
  if (host_error_count) *host_error_count = 0;
  if (count == 0) return SUBSPACE_CRC_OK;
  if (!host_slots) return fail(SUBSPACE_CRC_EINVAL, "null slot list");
  if (count >= (1ull << 32)) return fail(SUBSPACE_CRC_EINVAL, "count %llu exceeds 2^32-1", (unsigned long long)count);
  HIP_TRY(hipSetDevice(c->device));
  rc = ensure_host_stage(c, 0, 0);  // the compute stream
  if (rc) return rc;
  if (count > c->l_capacity) {
    (void)hipHostFree(c->l_hrec);
    (void)hipFree(c->l_drec);
    (void)hipFree(c->l_dstatus);
    (void)hipHostFree(c->l_hstatus);
    c->l_hrec = nullptr;
    c->l_drec = nullptr;
    c->l_dstatus = c->l_hstatus = nullptr;
    c->l_capacity = 0;
    HIP_TRY(hipHostMalloc(&c->l_hrec, count * sizeof(subspace_crc_slot), hipHostMallocDefault));
    HIP_TRY(hipMalloc(&c->l_drec, count * sizeof(subspace_crc_slot)));
    HIP_TRY(hipMalloc(&c->l_dstatus, (count + 1) * sizeof(u32)));
    HIP_TRY(hipHostMalloc(&c->l_hstatus, (count + 1) * sizeof(u32), hipHostMallocDefault));
    c->l_capacity = count;
  }
  const u64 prefix_size = ((u64)(48 + checksum_size + metadata_size) + 63) & ~63ull;
  {
    std::lock_guard<std::mutex> lock(g_regions_mu);
    for (u64 i = 0; i < count; i++) {
      const subspace_crc_slot& h = host_slots[i];
      const uintptr_t pre = host_alias((uintptr_t)h.prefix, prefix_size);
      const uintptr_t pay = h.message_size ? host_alias((uintptr_t)h.payload, h.message_size) : pre;
      if (!pre || !pay)
        return fail(SUBSPACE_CRC_EINVAL, "slot %llu: prefix or payload outside every registered host region",
                    (unsigned long long)i);
      if (pre % 8) return fail(SUBSPACE_CRC_EINVAL, "slot %llu: prefix not 8-B aligned", (unsigned long long)i);
      c->l_hrec[i] = subspace_crc_slot{(uint64_t)pre, (uint64_t)pay, h.message_size};
    }
  }
  hipStream_t st = c->hcompute;
  u32* dstatus = c->l_dstatus;
  u32* derr = c->l_dstatus + count;
  HIP_TRY(hipMemcpyAsync(c->l_drec, c->l_hrec, count * sizeof(subspace_crc_slot), hipMemcpyHostToDevice, st));
  rc = subspace_crc32_slots(c, c->l_drec, count, max_message_size, checksum_size, metadata_size, mode, dstatus, derr,
                            st);
  if (rc) {
    (void)hipStreamSynchronize(st);
    return rc;
  }
  HIP_TRY(hipMemcpyAsync(c->l_hstatus, dstatus, (count + 1) * sizeof(u32), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  rc = fault_status(c, st);
  if (rc) return rc;
  if (host_status) std::memcpy(host_status, c->l_hstatus, count * sizeof(u32));
  if (host_error_count) *host_error_count = c->l_hstatus[count];
  return SUBSPACE_CRC_OK;
}

}  // extern "C"

namespace subspace_amd {
__global__ void uniform_offsets_kernel(u64 stride, u64 length, u64 count, u64* offsets, u64* lengths) {
  const u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) {
    offsets[i] = i * stride;
    lengths[i] = length;
  }
}
}  // namespace subspace_amd
