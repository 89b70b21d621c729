// Scans and the tile-value combine of the ragged and long-message paths, hand-written for
// gfx950 (no library scan): one single-pass scan per call for the per-message tile counts,
// and a transpose + segment scan for the per-tile CRC values.
//
//  * Tile bases. crc32_ragged_count_scan_kernel computes every message's tile count and
//    its exclusive prefix sum in ONE pass (decoupled look-back): tile_base[m] = tiles before
//    message m, tile_base[count] = the batch's total. It also writes the (constant) result
//    of zero-length messages, zeroes every other output word (the overflow path XORs tile
//    values into it) and a slot batch's mismatch count, and flags a batch whose tiles the
//    8-B descriptors cannot hold (crc_ragged.hip TileDesc8).
//  * Tile values. The main kernels store one value per tile, tile tau = k*nw + w at
//    tilecrc[tilecrc_index(w, k)] (64 x 64 blocks of (w, k), w-major inside a block: contiguous
//    per flush, crc_device.h). A message's CRC is the
//    XOR of its tiles' values, i.e. P(t1 - 1) ^ P(t0 - 1) for the inclusive XOR prefix P in
//    tile order. P is kept in two levels instead of as a full scan:
//      segment s = 64 consecutive tiles of one sweep row k (tau = k*nw + 64*b + x, x < 64;
//                  s = k*nwb + b, nwb = ceil(nw / 64)), ordered like tau;
//      local[tau] = XOR of the values of tau's segment up to tau (inclusive; stored blocked),
//      segx[s]    = XOR of all tile values before segment s (exclusive),
//      P(tau)     = segx[s(tau)] ^ local[tau]                          (tile_prefix, crc_device.h).
//    tile_segment_scan_kernel reads one 16 KiB block of tilecrc through LDS, scans each 64-tile
//    row segment with a wave-wide XOR scan, writes the block of local[] (k-major, local_index)
//    and each segment's XOR; the segment
//    XORs (1/64 of the tiles) get a single-pass exclusive look-back scan in place. (Storing
//    local[] only at message-last tiles, the only ones the final kernels read, from a
//    per-tile end mask written by the descriptor kernel, was slower: 36 -> 43 us at config
//    C, r02f -- the masked partial-line stores cost as much as full ones.)
//
// Look-back scans (Merrill & Garland's decoupled look-back): a workgroup takes a ticket (its
// position in the scan, so every workgroup it waits for was started before it), scans its
// 4,096 elements, publishes its aggregate, then wave 0 reads its predecessors' status words
// 64 at a time -- an inclusive prefix ends the walk -- and publishes its own inclusive
// prefix. A status word is one 64-bit agent-scope atomic (flag and value together), so no
// other ordering is needed. The status words and tickets are zeroed at allocation and then
// by the next kernel of the call that runs after the scan (reset_scan_state, crc_device.h:
// the descriptor kernel for the tile-count scan, the final kernels for the segment scan),
// so every call -- and every replay of a captured hipGraph -- starts from a zeroed state.
#include "crc_desc.h"

namespace subspace_amd {

constexpr int kScanThreads = 256;
constexpr int kScanItems = (int)(kScanTile / kScanThreads);  // segment-prefix scan: elements per thread
static_assert(kScanTile % kScanThreads == 0, "segment-prefix scan: whole items per thread");
constexpr int kCountItems = (int)(kCountTile / kScanThreads);
static_assert(kCountTile % kScanThreads == 0, "tile-count scan: whole items per thread");
constexpr u64 kFlagAggregate = 1, kFlagInclusive = 2;

// Sum of u64 values below 2^62 (tile counts): flag in the top two bits.
struct SumOp {
  using T = u64;
  static __device__ __forceinline__ T identity() { return 0; }
  static __device__ __forceinline__ T op(T a, T b) { return a + b; }
  static __device__ __forceinline__ u64 pack(u64 flag, T v) { return (flag << 62) | v; }
  static __device__ __forceinline__ u64 flag(u64 s) { return s >> 62; }
  static __device__ __forceinline__ T value(u64 s) { return s & ((1ull << 62) - 1); }
};

// XOR of u32 values (tile CRC values): flag in the high word.
struct XorOp {
  using T = u32;
  static __device__ __forceinline__ T identity() { return 0; }
  static __device__ __forceinline__ T op(T a, T b) { return a ^ b; }
  static __device__ __forceinline__ u64 pack(u64 flag, T v) { return (flag << 32) | v; }
  static __device__ __forceinline__ u64 flag(u64 s) { return s >> 32; }
  static __device__ __forceinline__ T value(u64 s) { return (u32)s; }
};

template <class Op>
__device__ __forceinline__ typename Op::T shfl_up_t(typename Op::T v, int d) {
  if constexpr (sizeof(typename Op::T) == 8) {
    const u32 lo = (u32)__shfl_up((int)(u32)v, d, 64), hi = (u32)__shfl_up((int)(u32)(v >> 32), d, 64);
    return ((u64)hi << 32) | lo;
  } else {
    return (typename Op::T)__shfl_up((int)v, d, 64);
  }
}

template <class Op>
__device__ __forceinline__ typename Op::T shfl_xor_t(typename Op::T v, int m) {
  if constexpr (sizeof(typename Op::T) == 8) {
    const u32 lo = (u32)__shfl_xor((int)(u32)v, m, 64), hi = (u32)__shfl_xor((int)(u32)(v >> 32), m, 64);
    return ((u64)hi << 32) | lo;
  } else {
    return (typename Op::T)__shfl_xor((int)v, m, 64);
  }
}

// Workgroup ticket: the scan position of this workgroup (0, 1, ... in start order). A ticket
// beyond the grid means the counter was not zero at launch (stale state, or a call racing
// another on the context's workspace): kFaultTicket is raised and the caller leaves at once
// (its status word would lie past the scan's words), workgroup-uniformly.
// first_scan (the tile-count scan, a ragged call's first kernel): the workgroup holding ticket
// 0 clears the fault mark word[1] when it holds this call's generation -- left by an earlier
// replay of the same captured hipGraph (its generation is a kernel argument), whose fault must
// not make every later replay skip its work. No scan of this call can have marked
// it yet: with a stale counter no workgroup holds ticket 0, and a look-back wait gives up only
// after kSpinBound polls, long after ticket 0's workgroup started.
__device__ __forceinline__ u64 scan_ticket(u32* ticket, FaultRef fault, bool* stale, bool first_scan = false) {
  __shared__ u32 s_tile;
  if (threadIdx.x == 0) {
    s_tile = atomicAdd(ticket, 1u);
    if (first_scan && s_tile == 0 && fault.word &&
        __hip_atomic_load(fault.word + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == fault.gen)
      __hip_atomic_store(fault.word + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const u64 t = s_tile;
  *stale = t >= gridDim.x;
  if (*stale && threadIdx.x == 0) raise_scan_fault(fault, kFaultTicket);
  return t;
}

// Exclusive scan of the workgroup's kScanThreads * ITEMS elements x (thread t holds elements
// t*ITEMS .. +ITEMS-1 of tile `tile`), in place, continued from every earlier tile's
// elements through the look-back on `status`. A predecessor that never publishes (stale
// state: it cannot happen in a correct call) ends the wait after a bound and raises
// kFaultLookbackSpin in the context's fault word, so the call reports an error
// (subspace_crc_ctx_check) instead of returning wrong CRCs as OK, and the GPU never hangs.
template <class Op, int ITEMS, int THREADS = kScanThreads>
__device__ __forceinline__ void scan_tile_lookback(typename Op::T (&x)[ITEMS], u64 tile, u64* status, FaultRef fault) {
  using T = typename Op::T;
  __shared__ T s_wave[THREADS / 64];
  __shared__ T s_prefix;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T agg = Op::identity();
#pragma unroll
  for (int j = 0; j < ITEMS; j++) agg = Op::op(agg, x[j]);
  T inc = agg;  // inclusive scan of the thread aggregates over the wave
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T o = shfl_up_t<Op>(inc, d);
    if (lane >= d) inc = Op::op(o, inc);
  }
  T excl = shfl_up_t<Op>(inc, 1);
  if (lane == 0) excl = Op::identity();
  if (lane == 63) s_wave[wid] = inc;
  __syncthreads();
  T wpre = Op::identity(), total = Op::identity();
#pragma unroll
  for (int q = 0; q < THREADS / 64; q++) {
    if (q < wid) wpre = Op::op(wpre, s_wave[q]);
    total = Op::op(total, s_wave[q]);
  }
  if (wid == 0) {
    T prefix = Op::identity();
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(&status[0], Op::pack(kFlagInclusive, total), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&status[tile], Op::pack(kFlagAggregate, total), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
      i64 base = (i64)tile - 1;
      while (true) {
        const i64 idx = base - lane;  // lane 0: the nearest predecessor
        u64 s = Op::pack(kFlagInclusive, Op::identity());
        if (idx >= 0) {
          // every predecessor holds an earlier ticket and publishes; the bound turns a broken
          // invariant (stale state) into a reported fault instead of a hung GPU
          u32 spins = 0;
          do {
            s = __hip_atomic_load(&status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          } while (Op::flag(s) == 0 && ++spins < kSpinBound);
          if (Op::flag(s) == 0) {
            raise_scan_fault(fault, kFaultLookbackSpin);
            s = Op::pack(kFlagInclusive, Op::identity());
          }
        }
        const u64 incl = __ballot(Op::flag(s) == kFlagInclusive);
        const int first = incl ? __ffsll((unsigned long long)incl) - 1 : 63;
        T v = lane <= first ? Op::value(s) : Op::identity();
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) v = Op::op(v, shfl_xor_t<Op>(v, m));
        prefix = Op::op(v, prefix);
        if (incl) break;
        base -= 64;
      }
      if (lane == 0) __hip_atomic_store(&status[tile], Op::pack(kFlagInclusive, Op::op(prefix, total)),
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) s_prefix = prefix;
  }
  __syncthreads();
  T run = Op::op(s_prefix, Op::op(wpre, excl));
#pragma unroll
  for (int j = 0; j < ITEMS; j++) {
    const T v = x[j];
    x[j] = run;
    run = Op::op(run, v);
  }
}

// Tiles of message (s, L): its extended length L + (s & 15) in 8 KiB tiles (0 if L = 0)
// (crc_ragged.hip: a message is read from the 16-B block holding its first byte).
__device__ __forceinline__ u64 msg_tiles(u64 s, u64 len) { return len ? (len + (s & 15) + 8191) >> 13 : 0; }

// Per message: tile count, scanned into tile_base (count + 1 entries); zero-length messages
// get their result, every other output word is zeroed. `offsets`/`lengths` are read with an
// element stride (1 for plain arrays, 3 for the payload/size fields of subspace_crc_slot).
__global__ __launch_bounds__(kScanThreads) void crc32_ragged_count_scan_kernel(
    const u64* __restrict__ offsets, u32 ostride, const u64* __restrict__ lengths, u32 lstride, u64 count, u32 init,
    u32 final_xor, u64* __restrict__ tile_base, u32* __restrict__ out, u32* __restrict__ zero_word,
    u64* __restrict__ status, u32* __restrict__ ticket, u32* __restrict__ wide, FaultRef fault) {
  __shared__ u64 sx[kCountTile];  // striped (coalesced) global order <-> per-thread runs
  bool stale;
  const u64 tile = scan_ticket(ticket, fault, &stale, true);
  if (stale) return;
  const u64 base = tile * kCountTile;
  const int tid = threadIdx.x;
#pragma unroll
  for (int j = 0; j < kCountItems; j++) {
    const u64 i = base + (u64)(j * kScanThreads + tid);
    u64 nt = 0;
    if (i < count) {
      const u64 so = offsets[i * ostride];
      nt = msg_tiles(so, lengths[i * lstride]);
      out[i] = nt == 0 ? init ^ final_xor : 0u;
      // a tile the 8-B descriptor cannot hold (crc_ragged.hip TileDesc8): the call keeps 16 B
      if (nt && ((((so & ~(u64)15) + ((nt - 1) << 13)) >> kDesc8StartBits) | ((nt - 1) >> kDesc8AfterBits)))
        *wide = 1u;
    } else if (i == count && zero_word) {
      *zero_word = 0u;  // a slot batch's mismatch count (no separate memset)
    }
    sx[j * kScanThreads + tid] = nt;
  }
  __syncthreads();
  u64 x[kCountItems];
#pragma unroll
  for (int j = 0; j < kCountItems; j++) x[j] = sx[tid * kCountItems + j];
  scan_tile_lookback<SumOp, kCountItems>(x, tile, status, fault);  // synchronises before returning
#pragma unroll
  for (int j = 0; j < kCountItems; j++) sx[tid * kCountItems + j] = x[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kCountItems; j++) {
    const u64 i = base + (u64)(j * kScanThreads + tid);
    if (i <= count) tile_base[i] = sx[j * kScanThreads + tid];
  }
}

// The tile-count scan and the 8-B descriptors in one kernel, for batches whose arena (the bytes
// from the base every message lies in) is at most 2^37 bytes, so every tile fits the 8-B form
// (crc_desc.h). 1,024 threads x 4 messages per workgroup (the same 4,096-message scan tiles as
// crc32_ragged_count_scan_kernel, whose work this does first); after the look-back each wave
// writes the descriptors of its 4 x 64 messages (desc8_wave), which saves the separate
// descriptor kernel's launch, its reloads and half its latency-bound rounds.
// A message outside the 8-B range (a caller's arena bound broken) sets overflow[2]: the main
// kernel then locates every tile by search (correct for any batch).
constexpr int kFusedThreads = 1024;
constexpr int kFusedItems = (int)(kCountTile / kFusedThreads);
static_assert(kCountTile % kFusedThreads == 0, "fused scan: whole items per thread");
// WIDE (round 6): batches of absolute addresses (slot lists of 32 KiB slots:
// subspace_crc32_slots past the small kernel's 4 KiB) get the same fused scan with 16-B
// descriptors (descw_wave) and flag the batch wide (overflow[1]) for the main kernel, instead of
// the separate tile-count scan and descriptor kernels (S_large: 15.5 + 18.9 us per call).
template <bool WIDE>
__device__ __forceinline__ void count_desc_body(const u64* __restrict__ offsets, u32 ostride,
                                                const u64* __restrict__ lengths, u32 lstride, u64 count, u32 init,
                                                u32 final_xor, u64* __restrict__ tile_base, u32* __restrict__ out,
                                                u32* __restrict__ zero_word, u64* __restrict__ status,
                                                u32* __restrict__ ticket, u64 capacity, void* __restrict__ desc,
                                                u32* __restrict__ overflow, FaultRef fault) {
  __shared__ u64 sx[kCountTile];
  __shared__ u32 sw[WIDE ? 1 : kFusedThreads / 64][kDesc8WaveWords][64];
  bool stale;
  const u64 tile = scan_ticket(ticket, fault, &stale, true);
  if (stale) return;
  const u64 base = tile * kCountTile;
  const int tid = threadIdx.x;
  if (WIDE && tid == 0) overflow[1] = 1u;  // (the final kernel clears it for the next call)
  u64 so[kFusedItems], L[kFusedItems], nt[kFusedItems];
  bool bad = false;
#pragma unroll
  for (int j = 0; j < kFusedItems; j++) {
    const u64 i = base + (u64)(j * kFusedThreads + tid);
    so[j] = L[j] = nt[j] = 0;
    if (i < count) {
      so[j] = offsets[i * ostride];
      L[j] = lengths[i * lstride];
      nt[j] = msg_tiles(so[j], L[j]);
      out[i] = nt[j] == 0 ? init ^ final_xor : 0u;
      if (!WIDE && nt[j] &&
          ((((so[j] & ~(u64)15) + ((nt[j] - 1) << 13)) >> kDesc8StartBits) | ((nt[j] - 1) >> kDesc8AfterBits)))
        bad = true;
    } else if (i == count && zero_word) {
      *zero_word = 0u;  // a slot batch's mismatch count (no separate memset)
    }
    sx[j * kFusedThreads + tid] = nt[j];
  }
  if (bad) overflow[2] = 1u;
  __syncthreads();
  u64 x[kFusedItems];
#pragma unroll
  for (int j = 0; j < kFusedItems; j++) x[j] = sx[tid * kFusedItems + j];
  scan_tile_lookback<SumOp, kFusedItems, kFusedThreads>(x, tile, status, fault);  // synchronises before returning
#pragma unroll
  for (int j = 0; j < kFusedItems; j++) sx[tid * kFusedItems + j] = x[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kFusedItems; j++) {
    const u64 i = base + (u64)(j * kFusedThreads + tid);
    const u64 tb = sx[j * kFusedThreads + tid];
    if (i <= count) tile_base[i] = tb;
    if (i == count) overflow[0] = tb > capacity ? 1u : 0u;
    // the wave's 64 consecutive messages i (j fixed): their descriptors below the capacity
    if constexpr (WIDE)
      descw_wave(static_cast<TileDesc*>(desc), capacity, tb, nt[j], so[j], L[j]);
    else
      desc8_wave(static_cast<TileDesc8*>(desc), capacity, tb, nt[j], so[j], L[j], 0u, 64u, sw[tid >> 6], true);
  }
}

__global__ __launch_bounds__(kFusedThreads) void crc32_ragged_count_desc_kernel(
    const u64* __restrict__ offsets, u32 ostride, const u64* __restrict__ lengths, u32 lstride, u64 count, u32 init,
    u32 final_xor, u64* __restrict__ tile_base, u32* __restrict__ out, u32* __restrict__ zero_word,
    u64* __restrict__ status, u32* __restrict__ ticket, u64 capacity, TileDesc8* __restrict__ desc8,
    u32* __restrict__ overflow, FaultRef fault) {
  count_desc_body<false>(offsets, ostride, lengths, lstride, count, init, final_xor, tile_base, out, zero_word, status,
                         ticket, capacity, desc8, overflow, fault);
}

__global__ __launch_bounds__(kFusedThreads) void crc32_ragged_count_desc16_kernel(
    const u64* __restrict__ offsets, u32 ostride, const u64* __restrict__ lengths, u32 lstride, u64 count, u32 init,
    u32 final_xor, u64* __restrict__ tile_base, u32* __restrict__ out, u32* __restrict__ zero_word,
    u64* __restrict__ status, u32* __restrict__ ticket, u64 capacity, TileDesc* __restrict__ desc,
    u32* __restrict__ overflow, FaultRef fault) {
  count_desc_body<true>(offsets, ostride, lengths, lstride, count, init, final_xor, tile_base, out, zero_word, status,
                        ticket, capacity, desc, overflow, fault);
}

// Tiles present: the batch's total (device value, ragged path) or a host count (long path),
// bounded by the workspace capacity.
__device__ __forceinline__ u64 tiles_present(const u64* total_ptr, u64 n) {
  if (total_ptr) {
    const u64 t = *total_ptr;
    return t < n ? t : n;
  }
  return n;
}

// Tile values -> per-segment inclusive XOR scans (local) and the XOR of every segment (segx,
// before its scan). Block (a, b) is the 64 x 64 block of k in [64a, +64), w in [64b, +64): it
// reads tilecrc's 16 KiB block (w-major) and writes local's (k-major), both contiguous
// (crc_device.h tilecrc_index / local_index); wave q scans the rows k = 64a + q + 4i.
__global__ __launch_bounds__(256) void tile_segment_scan_kernel(const u32* __restrict__ in, u32 nw, u32 nkmax,
                                                                u32 nwb, const u64* __restrict__ total_ptr, u64 n_cap,
                                                                u32* __restrict__ local, u32* __restrict__ segx) {
  __shared__ u32 t[64][65];
  __shared__ u32 s2[64][64 + 4];  // the scanned block, k-major (16-B aligned rows)
  const u64 n = tiles_present(total_ptr, n_cap);
  const u32 k0 = blockIdx.x * 64u, w0 = blockIdx.y * 64u;
  if ((u64)k0 * nw + w0 >= n) return;  // every tile of the block is past the batch
  const u64 blk = ((u64)blockIdx.x * nwb + blockIdx.y) * 4096u;
  const u32 x = threadIdx.x & 63u, y0 = threadIdx.x >> 6;
  // 16 B per lane: thread (y4, x4) loads columns 4 x4 .. +3 of rows y4 + 16 i
  {
    const u32 x4 = threadIdx.x & 15u, y4 = threadIdx.x >> 4;
    u32x4 v[4];
#pragma unroll
    for (u32 i = 0; i < 4u; i++) v[i] = *reinterpret_cast<const u32x4*>(in + blk + 64u * (y4 + 16u * i) + 4u * x4);
#pragma unroll
    for (u32 i = 0; i < 4u; i++) {
      const u32 y = y4 + 16u * i, w = w0 + y;
#pragma unroll
      for (u32 c = 0; c < 4u; c++) {
        const u32 k = k0 + 4u * x4 + c;
        t[y][4u * x4 + c] = (w < nw && k < nkmax) ? v[i][c] : 0u;
      }
    }
  }
  __syncthreads();
#pragma unroll 4
  for (u32 i = 0; i < 16u; i++) {  // row k = k0 + y: tiles tau = k*nw + w0 + x
    const u32 y = y0 + 4u * i, k = k0 + y;
    u32 v = t[x][y];  // 0 past nw
    // inclusive XOR scan over the 64 lanes: DPP row shifts within each 16-lane row (source
    // lanes out of the row read as 0), then rows 1, 3 take lane 15 of rows 0, 2 and rows
    // 2, 3 take lane 31 (VALU only, no LDS round trip)
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    if (k < nkmax) {
      s2[y][x] = v;
      if (x == 63u) segx[(u64)k * nwb + blockIdx.y] = v;
    }
  }
  {
    // the block of local[] (k-major) as 16-B stores; entries past the batch or past nw hold
    // values no reader uses (the allocation covers whole blocks)
    __syncthreads();
    const u32 x4 = threadIdx.x & 15u, y4 = threadIdx.x >> 4;
#pragma unroll
    for (u32 i = 0; i < 4u; i++) {
      const u32 y = y4 + 16u * i;
      if (k0 + y < nkmax)
        *reinterpret_cast<u32x4*>(local + blk + 64u * y + 4u * x4) =
            u32x4{s2[y][4u * x4], s2[y][4u * x4 + 1u], s2[y][4u * x4 + 2u], s2[y][4u * x4 + 3u]};
    }
  }
}

// Exclusive XOR scan of the segment values, in place (look-back, one pass). Workgroups past
// the last segment that holds a tile of the batch leave at once (nothing later reads them).
__global__ __launch_bounds__(kScanThreads) void segment_prefix_kernel(u32* __restrict__ segx, u64 nseg, u32 nw,
                                                                      u32 nwb, const u64* __restrict__ total_ptr,
                                                                      u64 n_cap, u64* __restrict__ status,
                                                                      u32* __restrict__ ticket, FaultRef fault) {
  bool stale;
  const u64 tile = scan_ticket(ticket, fault, &stale);
  if (stale) return;
  const u64 n = tiles_present(total_ptr, n_cap);
  if (n == 0) return;
  const u64 last = n - 1, need = (last / nw) * nwb + (last % nw) / 64u + 1;  // segments up to the last tile
  const u64 lim = need < nseg ? need : nseg;
  if (tile * kScanTile >= lim) return;  // workgroup-uniform
  const u64 i0 = tile * kScanTile + (u64)threadIdx.x * kScanItems;
  u32 x[kScanItems];
#pragma unroll
  for (int j = 0; j < kScanItems; j++) x[j] = i0 + j < lim ? segx[i0 + j] : 0u;
  scan_tile_lookback<XorOp, kScanItems>(x, tile, status, fault);
#pragma unroll
  for (int j = 0; j < kScanItems; j++)
    if (i0 + j < lim) segx[i0 + j] = x[j];
}

}  // namespace subspace_amd
