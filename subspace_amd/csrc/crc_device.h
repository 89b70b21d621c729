// Device-side building blocks shared by the CRC32 kernels (gfx950 / CDNA4).
//
// LDS layout of every CRC kernel (one workgroup per CU):
//   [0, 128 KiB)       slice-by-4 byte tables, 32-way replicated: table k (k = 0..3 for
//                      byte k of the step word) entry e copy b at byte address
//                      ((k>>1)<<16) | (e<<8) | ((k&1)<<7) | (b<<2). Lane l reads copy
//                      (l & 31), i.e. LDS bank (l & 31), so the 4 data-dependent lookups
//                      of a step are bank-conflict-free for any data (ds_read_b32 banks
//                      lanes in two groups of 32, bank = dword address mod 32).
//   [128 KiB, +16 KiB) per-lane line-shift operators Z_{128*s}, s = 0..31, laid out
//                      [nibble k][value n][slot s]: the 32 lanes of a half read 32
//                      different banks (conflict-free for any data).
//   [144 KiB, ...)     uniform kernel: per-wave result rings; ragged kernel: 22 GF(2)
//                      operator slots, each 8 nibble tables x 16 dwords (512 B). A
//                      16-entry table spans 16 distinct banks, so nibble lookups are
//                      conflict-free without replication.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace subspace_amd {

using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
using u32x2 = __attribute__((ext_vector_type(2))) unsigned int;

constexpr u32 kLdsTables = 0;
constexpr u32 kLdsOps = 128u * 1024u;  // operator area; opmul slot s = 512 B at kLdsOps + 512*s

// Uniform-kernel layout: tables, the per-lane line-shift operators (kLaneOpWords, see
// crc32_uniform4k_kernel), the opmul slot Z_4096 (slot variant), then a per-wave ring of
// results awaiting their store (the device operator array d_laneops holds the same
// kUniOpSlots slots).
constexpr int kLaneOpWords = 8 * 16 * 32;  // [nibble k][value n][lane slot s]: 16 KiB
constexpr int kUniSlotOpZ4096 = kLaneOpWords * 4 / 512;  // opmul slot 32
// slots 33..36: Z_64 as a nibble table replicated 4x, [nibble k][value n][copy c], lane l
// reading copy l & 3 (conflict-free): the join of a line's two 64-B chains (two-chain line
// CRC)
constexpr int kUniSlotOpZ64 = kUniSlotOpZ4096 + 1;
constexpr int kUniOpSlots = kUniSlotOpZ64 + 4;
constexpr int kUniOpSlotsOneChain = kUniSlotOpZ4096 + 1;
constexpr u32 kUniRing = kLdsOps + kUniOpSlots * 512u;
// results per wave ring: 256 (128 tiles), or 128 where 16 waves' rings would not fit
constexpr int uni_ring_results(int waves) { return kUniRing + (u32)waves * 1024u <= 160u * 1024u ? 256 : 128; }
constexpr size_t uniform_lds_bytes(int waves) { return kUniRing + (size_t)waves * 4u * uni_ring_results(waves); }
static_assert(uniform_lds_bytes(16) <= 160u * 1024u && uniform_lds_bytes(8) <= 160u * 1024u,
              "uniform kernel LDS exceeds 160 KiB");
// Slot variant (crc_uniform.hip, SLOT = true): each wave's results go to a ring of
// kSlotRingRounds tiles (2 tagged 8-B entries per tile: CRC | tile index << 32; a workgroup is
// one ring window: the host gives no wave more tiles), read after the tile loop by the
// workgroup's kSlotFinishers finishing waves; then the workgroup's mismatch word.
constexpr u32 kUniSlotRing = kUniRing;
constexpr int kSlotRingRounds = 32;
constexpr int kSlotFinishers = 4;  // waves 0-3: the older wave of each SIMD pair
constexpr u32 kSlotRingBytesPerWave = 2u * 8u * kSlotRingRounds;
constexpr u32 uniform_slot_mism_word(int waves) { return kUniSlotRing + (u32)waves * kSlotRingBytesPerWave; }
constexpr size_t uniform_slot_lds_bytes(int waves) { return uniform_slot_mism_word(waves) + 16u; }
static_assert(uniform_slot_lds_bytes(8) <= 160u * 1024u, "slot kernel LDS exceeds 160 KiB");

// Fused slot checksums of the uniform 4 KiB kernel: the message-slot layout of
// subspace_crc32_slots_strided with metadata_size 0 (crc_uniform.hip, crc_slots.hip).
struct SlotArgs {
  u64 prefix_size;     // payload = prefix + prefix_size; the kernel's base points at payload 0
  u32 mode;            // SUBSPACE_CRC_SLOT_CALCULATE (0) / _VERIFY (1)
  u32* status;         // optional, per slot
  u32* crc_out;        // optional (CALCULATE): stored checksum per slot
  u32* error_count;    // optional (VERIFY): mismatches of this call
  u64* counter;        // context counter entry (kCountWords words, add_call_mismatches); 0 between calls
  u64* probe;          // PROBE instantiation only: per-wave timestamps (tools/wave_timeline.py)
  u32* fault;          // context fault word (kFault* bits), read by subspace_crc_ctx_check
  u32 checksum_size;   // span 1 = prefix[48 + checksum_size, + metadata_size) (common/channel.h:527-542)
  u32 metadata_size;   // <= kSlotFusedMaxMeta
};
constexpr u32 kSlotFusedMaxMeta = 64;  // metadata bytes the fused slot kernel folds in (more: two-kernel path)

// Context fault word: set by a kernel whose bounded wait gave up (a broken invariant: stale
// state, or a call racing another on the same context). The kernel finishes instead of hanging
// the GPU, and the host reports the call as failed (subspace_crc_ctx_check) instead of OK.
constexpr u32 kFaultLookbackSpin = 1u;  // a look-back scan predecessor never published
constexpr u32 kFaultTicket = 2u;        // a look-back scan ticket beyond the grid (stale ticket)
constexpr u32 kFaultSlotRing = 4u;      // a slot finishing wave waited too long for a payload CRC
__device__ __forceinline__ void raise_fault(u32* fault, u32 bit) {
  if (fault) __hip_atomic_fetch_or(fault, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The look-back scans' faults (kFaultTicket, kFaultLookbackSpin) also mark the call they
// happened in: word[1] of the fault words takes the call's generation (a per-context counter,
// never 0), so the kernels of that call that would index with its untrusted tile_base do
// nothing, while a later call on the context -- whose kernels reset the scan state as usual --
// runs normally even when nobody has called subspace_crc_ctx_check in between (ADVICE r03:
// the accumulated word[0] alone made every later call skip and return the previous CRCs).
struct FaultRef {
  u32* word;  // the context's fault words: [0] kFault* bits (ctx_check), [1] generation
  u32 gen;    // this call's generation
};
__device__ __forceinline__ void raise_scan_fault(FaultRef f, u32 bit) {
  if (f.word) {
    __hip_atomic_fetch_or(f.word, bit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(f.word + 1, f.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// A look-back scan of this call gave up: its tile_base is not to be trusted.
__device__ __forceinline__ bool scan_faulted(FaultRef f) {
  // a plain load: the word is written by an earlier kernel of the call (a look-back scan that
  // gave up), and the kernel boundary orders it
  return f.word && f.word[1] == f.gen;
}
// Spin bound of every bounded wait, far beyond any real one: the look-back scans poll an
// uncached status word up to 2^20 times without sleeping (~1 s, tests/test_gpu_fault.py); the
// fused slot kernel's finishing waves poll their LDS ring up to 2^20 times with s_sleep(2)
// between polls (~0.1 s).
constexpr u32 kSpinBound = 1u << 20;
// Per-wave probe record of the uniform kernel's PROBE instantiation: realtime clock (100 MHz)
// at entry, after the LDS fill + barrier, after the tile loop, at exit, after the table and
// tile-0 loads were issued; then XCC_ID | tile count << 32; the wave's HW_ID register (wave
// slot [3:0], SIMD [5:4], CU [11:8], SE [14:13]) | the low 32 bits of the clock when a slot
// finishing wave began (else 0) << 32; when the wave's first tile had landed.
constexpr int kProbeWords = 8;

// Ragged-kernel layout: tables, the same line-shift operators, then opmul slots Z_4096 and
// Z_{8192 * 2^k}, k = 0..20 (8 KiB .. 8 GiB), and Z_64 (4 slots). The device operator array continues with
// Z_{8192 * 2^k}, k = 21..30, read from global memory (messages of 16 GiB and more), and
// the padding inverses Z_{2^b}^{-1}, b = 0..12, of the ragged final kernel.
constexpr int kNumTileOps = 21;
constexpr int kRagOpZ4096 = kLaneOpWords * 4 / 512;  // opmul slot 32
constexpr int kRagOpZTile = kRagOpZ4096 + 1;
// then Z_64 replicated 4x (the two-chain line CRC's join, as in the uniform kernel)
constexpr int kRagZ64Words = kLaneOpWords + (1 + kNumTileOps) * 128;
constexpr int kRagLdsOpWords = kRagZ64Words + 512;
constexpr int kRagHighOps = kRagLdsOpWords;  // word offset of Z_{8192 * 2^21} in the device array
constexpr int kNumInvOps = 13;
constexpr int kRagInvOps = kRagHighOps + (31 - kNumTileOps) * 128;  // word offset of Z_1^{-1}
// then the ragged final kernel's nibble inverses Z_{d 16^k}^{-1}, k = 0..2, d = 1..15 (slot
// 15 k + d - 1): a padding p < 8192 is undone in at most four steps, its three low nibbles and
// then bit 12 (Z_4096^{-1}, the last bit inverse)
constexpr int kRagNibInvOps = kRagInvOps + kNumInvOps * 128;
constexpr int kNumNibInvOps = 45;
constexpr int kRagOpWords = kRagNibInvOps + kNumNibInvOps * 128;
constexpr size_t ragged_lds_bytes() { return kLdsOps + (size_t)kRagLdsOpWords * 4u; }
static_assert(ragged_lds_bytes() <= 160u * 1024u, "ragged kernel LDS exceeds 160 KiB");

// Small-message kernel layout (crc_small.hip): the uniform kernel's operator slots (line
// shifts, Z_4096, Z_64 x4), then the padding inverses Z_{2^b}^{-1}, b = 0..11 (a message of
// at most 4 KiB is padded by fewer than 4,096 bytes), then a 16-B word (the workgroup's
// mismatch count). The device array d_laneops holds all kSmallOpSlots slots (the uniform kernel loads
// the first kUniOpSlots).
constexpr int kSmallOpInv = kUniOpSlots;
constexpr int kSmallInvOps = 12;
constexpr int kSmallOpSlots = kSmallOpInv + kSmallInvOps;
// one more LDS slot: Z_C for the packed forms' capacity C = 128 G < 4096 (the slot finish's
// Z_C(H)), copied per launch from d_laneops slot kSmallOpZC + log2(G) (G = 1..16)
constexpr int kSmallOpZC = kSmallOpSlots;
constexpr int kSmallLaneOpSlots = kSmallOpZC + 5;  // d_laneops slots
constexpr u32 kSmallMaxExt = 4096;  // extended bytes (length + offset & 15) of one half-tile
constexpr u32 kSmallRing = kLdsOps + (u32)(kSmallOpSlots + 1) * 512u;  // per-wave result rings
constexpr u32 kSmallRingTiles = 32;                               // tiles per ring window
constexpr u32 kSmallRingBytesPerWave = kSmallRingTiles * 2u * 8u;  // (value | code << 32) per message
// Workgroup repack of the slot kernel (crc_small.hip SLOT, G = 32, REPACK2), in the same area as
// the per-wave rings (a workgroup runs one or the other): the workgroup's entries (8 waves x 32
// messages; the host gives no slot wave more than 16 tiles) -- each wave's first Q lines its
// own local tiles (Q: the workgroup's least wave, rounded down to whole tiles, at least 64), the
// other lines laid out back to back over the workgroup's shared packed tiles, which its 8 waves
// take from an LDS ticket.
constexpr u32 kRp2Entries = 256;
constexpr u32 kRp2MaxTiles = kRp2Entries * 32u / 64u;           // every entry at most 32 lines
// the entries with lines, by rank: u64 first byte | ring entry << 56 (offsets and addresses are
// below 2^56), u32 E | first line << 13
constexpr u32 kRp2EntS = kSmallRing;
constexpr u32 kRp2EntM = kRp2EntS + 8u * kRp2Entries;
constexpr u32 kRp2Ring = kRp2EntM + 4u * kRp2Entries;           // u64: value (XOR of parts) | code << 32
constexpr u32 kRp2Starts = kRp2Ring + 8u * kRp2Entries;         // u64 per packed tile: lines that start a message
constexpr u32 kRp2First = kRp2Starts + 8u * kRp2MaxTiles;       // u32 per packed tile: rank of its line 0's entry
// u32 [0, 8) lines per wave, [8, 16) votes (not FAST), [24] ticket; u64 [14, 22) each wave's local
// start marks; then per wave 16 bytes: its entries with lines past 64 (i + 1), i = 0..15
constexpr u32 kRp2Misc = kRp2First + 4u * kRp2MaxTiles;
constexpr u32 kRp2Counts = kRp2Misc + 176u;
constexpr u32 kRp2Bytes = kRp2Counts + 128u - kSmallRing;
constexpr u32 kSmallShared = 8u * kSmallRingBytesPerWave > kRp2Bytes ? 8u * kSmallRingBytesPerWave : kRp2Bytes;
constexpr size_t small_lds_bytes() { return kSmallRing + kSmallShared; }
static_assert(small_lds_bytes() + 16u <= 160u * 1024u, "small-message kernel LDS (+ mismatch word) exceeds 160 KiB");
constexpr u32 kRp2MaxTilesPerWave = 16;  // slot waves (G = 32): the host's grid rule (capi.hip small_run)

// Small-message kernel arguments (crc_small.hip; one struct: read with scalar loads).
struct SmallArgs {
  const uint8_t* base;
  const u64* offsets;   // message m's first byte: base + offsets[m * ostride]
  const u64* lengths;   // its length: lengths[m * lstride]
  const u64* prefixes;  // SLOT: its MessagePrefix at base + prefixes[m * pstride] - pdelta
  u64 count;
  u64 pdelta;
  u32 ostride, lstride, pstride;
  u32 init, final_xor;
  u32 mode, checksum_size, metadata_size;  // SLOT: both sizes <= kSlotFusedMaxMeta (lanes
                                           // without a slot read their spans from the 4 KiB
                                           // step table)
  u32* out;          // !SLOT: the CRC of every message
  u32* status;       // SLOT, optional: per-slot status
  u32* crc_out;      // SLOT, optional: the stored checksum (CALCULATE)
  u32* error_count;  // SLOT, optional: this call's mismatches (0 for CALCULATE)
  u64* counter;      // SLOT: context counter entry (kCountWords words, add_call_mismatches); 0 between calls
  u32* zero_word;    // !SLOT, optional: zeroed at the end (the next kernel's mismatch count)
  const u32* rops;   // the ragged operator array (Z_8192; Z_4096^{-1}, the 13th padding inverse)
  const u32* pow2;   // SLOT: Z_{2^k}, k < 64 (a long message's Z_L)
  u64 max_len;       // SLOT: a larger message size is SUBSPACE_CRC_SLOT_OVERSIZE (strided layouts:
                     // the slot's payload area); ~0 for slot lists
  u64* probe;        // experiment hook (subspace_crc_testutil_probe), else null: kProbeWords realtime
                     // stamps per wave, stored at exit (tools/small_timeline.py)
  u64 ustride, ulen;  // offsets == null (a uniform batch): message m at base + m * ustride, ulen bytes
};

// Segments per workgroup of the segment-prefix look-back scan (crc_combine.hip, 256 threads)
#ifndef SUBSPACE_SCAN_TILE
#define SUBSPACE_SCAN_TILE 2048
#endif
constexpr u64 kScanTile = SUBSPACE_SCAN_TILE;
// Messages per workgroup of the tile-count scan (crc_combine.hip, 256 threads)
#ifndef SUBSPACE_COUNT_TILE
#define SUBSPACE_COUNT_TILE 4096
#endif
constexpr u64 kCountTile = SUBSPACE_COUNT_TILE;
// 8-B tile descriptors (crc_ragged.hip TileDesc8) hold tile starts below 2^37 bytes (128 GiB)
// and up to 2^25 - 1 tiles after a tile; a batch with any tile beyond that keeps 16 B (the
// tile-count scan flags it) or, through the fused count + descriptor kernel, is searched.
// hi word: start bits 36.. [kD8StartHiBits), mis [4), the first-tile flag, then X (26 bits):
// the tiles after the tile, or kLastTile8 | the last tile's bytes.
constexpr u32 kDesc8StartBits = 37;
constexpr u32 kDesc8AfterBits = 25;
constexpr u32 kD8StartHiBits = kDesc8StartBits - 36;
constexpr u32 kD8MisShift = kD8StartHiBits;
constexpr u32 kD8FirstBit = 1u << (kD8MisShift + 4);
constexpr u32 kD8XShift = kD8MisShift + 5;
static_assert(kD8XShift + kDesc8AfterBits + 1 == 32, "8-B descriptor fields fill 64 bits");

// Ragged kernel head seeds of one call: v[r] = Z_r^{-1}(init), r = 0..15 (a kernel argument).
struct HeadSeeds {
  u32 v[16];
};

typedef __attribute__((address_space(3))) u32 lds_u32_t;
typedef __attribute__((address_space(3))) u64 lds_u64_t;
typedef __attribute__((address_space(3))) u32x4 lds_u32x4_t;

// v_readfirstlane as an unsigned dword (the builtin returns int: widening it directly to
// 64 bits would sign-extend the low half of a byte offset >= 2 GiB)
__device__ __forceinline__ u32 rfl(u32 v) { return (u32)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ u64 rfl64(u32 lo, u32 hi) { return ((u64)rfl(hi) << 32) | (u64)rfl(lo); }

// Buffer-resource word 3 for raw (unformatted, unswizzled) gfx950 buffer loads.
constexpr int kBufferRsrcFlags = 0x00020000;

// Position of wave `wid` of workgroup `b` (of G) in a sweep front: consecutive pairs of
// front slots go to consecutive workgroups, i.e. round-robin over the 8 XCDs.
__device__ __forceinline__ u64 front_slot(u32 b, u32 G, u32 wid) {
  return ((u64)b + (u64)G * (wid >> 1)) * 2 + (wid & 1u);
}

__device__ __forceinline__ u32 lds_ld(u32 addr) { return *reinterpret_cast<const lds_u32_t*>((uintptr_t)addr); }
__device__ __forceinline__ void lds_st(u32 addr, u32 v) { *reinterpret_cast<lds_u32_t*>((uintptr_t)addr) = v; }
// one ds_read_b64 / ds_write_b64 (8-B aligned: single-copy atomic, so a tagged entry is
// never seen half-written by another wave)
__device__ __forceinline__ u64 lds_ld64(u32 addr) { return *reinterpret_cast<const volatile lds_u64_t*>((uintptr_t)addr); }
__device__ __forceinline__ void lds_st64(u32 addr, u64 v) { *reinterpret_cast<lds_u64_t*>((uintptr_t)addr) = v; }
__device__ __forceinline__ u32 lds_ld_volatile(u32 addr) {
  return *reinterpret_cast<const volatile lds_u32_t*>((uintptr_t)addr);
}
__device__ __forceinline__ u32x4 lds_ld4(u32 addr) { return *reinterpret_cast<const lds_u32x4_t*>((uintptr_t)addr); }
__device__ __forceinline__ void lds_st4(u32 addr, u32x4 v) { *reinterpret_cast<lds_u32x4_t*>((uintptr_t)addr) = v; }

#ifndef SUBSPACE_FILL_ROTATE
#define SUBSPACE_FILL_ROTATE 1  // conflict-free table fill (0: the round-3 store order, for A/B builds)
#endif
// Fill of the replicated step tables and the first NOPS operator slots, split into a
// load phase and a store phase so a kernel can issue its first tile's global loads in
// between: vmcnt retires in issue order, so the table loads (older) can be waited for
// while the tile loads (younger) stay in flight across the LDS stores and the barrier.
// gtab: 4 x 256 dwords, gtab[k*256 + b] = CRC of byte b followed by k zero bytes.
// gops: kNumOps * 128 dwords of nibble tables.
template <int WG, int NOPS>
struct LdsFill {
  static constexpr int kTabIters = (1024 + WG - 1) / WG;
  static constexpr int kOpWords = NOPS * 128;
  static constexpr int kOpIters = (kOpWords + WG - 1) / WG;
  u32 tv[kTabIters], ov[kOpIters];

  __device__ __forceinline__ void load(const u32* __restrict__ gtab, const u32* __restrict__ gops) {
    // Unconditional loads (indices clamped; surplus values are never stored): a load in a
    // divergent branch would make hipcc wait vmcnt(0) here instead of a counted wait.
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < kTabIters; i++) {
      const int t = min(tid + i * WG, 1023);
      // step-table k serves byte k of the word, i.e. the byte followed by 3-k zero bytes
      tv[i] = gtab[(3 - (t & 3)) * 256 + (t >> 2)];
    }
#pragma unroll
    for (int i = 0; i < kOpIters; i++) ov[i] = gops[min(tid + i * WG, kOpWords - 1)];
  }

  __device__ __forceinline__ void store(u32 sbase) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < kTabIters; i++) {
      const int t = tid + i * WG;
      if (t < 1024) {
        const int k = t & 3, e = t >> 2;
        const u32x4 vv = {tv[i], tv[i], tv[i], tv[i]};
        const u32 dst = sbase + (((u32)(k >> 1) << 16) | ((u32)e << 8) | ((u32)(k & 1) << 7));
        // A lane writes its entry's 32 copies as 8 x 16 B, starting at chunk (lane & 7): every
        // entry row is 128-B aligned, so without the rotation all lanes of a ds_write_b128 lane
        // group (8 consecutive lanes) hit the same 4 banks, an 8-way conflict (64 instead of 8
        // LDS cycles per store: ~7,200 cycles per CU per launch, 78 % of the uniform kernel's
        // SQ_LDS_BANK_CONFLICT, profiles/r04/ledger).
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const u32 jj = SUBSPACE_FILL_ROTATE ? ((u32)(j + tid) & 7u) : (u32)j;
          lds_st4(dst + 16u * jj, vv);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kOpIters; i++) {
      const int t = tid + i * WG;
      if (t < kOpWords) lds_st(sbase + kLdsOps + 4 * t, ov[i]);
    }
    // Consume every fill load on every path: otherwise hipcc's waitcnt pass treats the
    // skipped ones as possibly pending at the main loop's header and drains the tile
    // prefetch with vmcnt(0) on every iteration.
#pragma unroll
    for (int i = 0; i < kTabIters; i++) asm volatile("" ::"v"(tv[i]));
#pragma unroll
    for (int i = 0; i < kOpIters; i++) asm volatile("" ::"v"(ov[i]));
  }
};

// One slice-by-4 step: crc_raw(0, LE bytes of x) = T4(x), via 4 conflict-free lookups.
// lc0 = sbase | (lane&31)<<2, lc1 = lc0 + 64 KiB. v_perm_b32 builds each address in one
// instruction: byte0 = lane bank offset, byte1 = the data byte, byte2 = region, byte3 = 0.
__device__ __forceinline__ u32 step4(u32 x, u32 lc0, u32 lc1) {
  const u32 a0 = __builtin_amdgcn_perm(x, lc0, 0x0c020400u);
  const u32 a1 = __builtin_amdgcn_perm(x, lc0, 0x0c020500u);
  const u32 a2 = __builtin_amdgcn_perm(x, lc1, 0x0c020600u);
  const u32 a3 = __builtin_amdgcn_perm(x, lc1, 0x0c020700u);
  return lds_ld(a0) ^ lds_ld(a1 + 128) ^ lds_ld(a2) ^ lds_ld(a3 + 128);
}

// The same step with the next data word folded in: T4(x) ^ next, the four lookups and
// `next` joined by two 3-input XORs (v_bitop3_b32 0x96) instead of four v_xor_b32.
__device__ __forceinline__ u32 step4n(u32 x, u32 lc0, u32 lc1, u32 next) {
  const u32 a0 = __builtin_amdgcn_perm(x, lc0, 0x0c020400u);
  const u32 a1 = __builtin_amdgcn_perm(x, lc0, 0x0c020500u);
  const u32 a2 = __builtin_amdgcn_perm(x, lc1, 0x0c020600u);
  const u32 a3 = __builtin_amdgcn_perm(x, lc1, 0x0c020700u);
  const u32 t = __builtin_amdgcn_bitop3_b32(lds_ld(a0), lds_ld(a1 + 128), lds_ld(a2), 0x96);
  return __builtin_amdgcn_bitop3_b32(t, lds_ld(a3 + 128), next, 0x96);
}

// Z_64 of v from the 4x replicated nibble table at z64 (= its base + 4 * (lane & 3)).
__device__ __forceinline__ u32 opmul_z64(u32 z64, u32 v) {
  u32 t[8];
#pragma unroll
  for (int k = 0; k < 8; k++) t[k] = lds_ld(z64 + 256u * k + (((v >> (4 * k)) & 15u) << 4));
  const u32 a = __builtin_amdgcn_bitop3_b32(t[0], t[1], t[2], 0x96);
  const u32 b = __builtin_amdgcn_bitop3_b32(a, t[3], t[4], 0x96);
  const u32 c = __builtin_amdgcn_bitop3_b32(b, t[5], t[6], 0x96);
  return c ^ t[7];
}

// The same CRC as two independent 16-step chains (bytes 0..63 from `init`, 64..127 from 0)
// joined by linearity: crc_raw(init, A || B) = Z_64(crc_raw(init, A)) ^ crc_raw(0, B).
__device__ __forceinline__ u32 line_crc32_2chain(const u32x4 (&d)[8], u32 init, u32 lc0, u32 lc1, u32 z64) {
  u32 x = init ^ d[0][0], y = d[4][0];
#pragma unroll
  for (int w = 0; w < 16; w++) {
    x = step4n(x, lc0, lc1, w < 15 ? d[(w + 1) >> 2][(w + 1) & 3] : 0u);
    y = step4n(y, lc0, lc1, w < 15 ? d[(w + 17) >> 2][(w + 17) & 3] : 0u);
  }
  return opmul_z64(z64, x) ^ y;
}

// The same for a line whose bytes 64..127 are zero (their chain from 0 stays 0): one 16-step
// chain, Z_64 of it.
__device__ __forceinline__ u32 line_crc32_lo(const u32x4 (&d)[8], u32 init, u32 lc0, u32 lc1, u32 z64) {
  u32 x = init ^ d[0][0];
#pragma unroll
  for (int w = 0; w < 16; w++) x = step4n(x, lc0, lc1, w < 15 ? d[(w + 1) >> 2][(w + 1) & 3] : 0u);
  return opmul_z64(z64, x);
}

// CRC of one 128-B line (8 x 16 B), from state `init`: 32 steps of step4n.
__device__ __forceinline__ u32 line_crc32(const u32x4 (&d)[8], u32 init, u32 lc0, u32 lc1) {
  u32 x = init ^ d[0][0];
#pragma unroll
  for (int w = 0; w < 32; w++) x = step4n(x, lc0, lc1, w < 31 ? d[(w + 1) >> 2][(w + 1) & 3] : 0u);
  return x;
}

// Per-lane line-shift operator applied to a line CRC: 8 nibble lookups in the table laid
// out [nibble k][value n][lane slot] (lop = this lane's slot), joined by 3-input XORs.
__device__ __forceinline__ u32 lane_shift(u32 lop, u32 crc) {
  u32 t[8];
#pragma unroll
  for (int j = 0; j < 8; j++) t[j] = lds_ld(lop + 2048u * j + (((crc >> (4 * j)) & 15u) << 7));
  const u32 a = __builtin_amdgcn_bitop3_b32(t[0], t[1], t[2], 0x96);
  const u32 b = __builtin_amdgcn_bitop3_b32(a, t[3], t[4], 0x96);
  const u32 c = __builtin_amdgcn_bitop3_b32(b, t[5], t[6], 0x96);
  return c ^ t[7];
}

// Apply GF(2) operator `slot` to v: 8 conflict-free nibble lookups.
__device__ __forceinline__ u32 opmul(u32 sbase, int slot, u32 v) {
  const u32 op = sbase + kLdsOps + 512u * (u32)slot;
  u32 r = lds_ld(op + ((v << 2) & 0x3Cu));
#pragma unroll
  for (int k = 1; k < 8; k++) r ^= lds_ld(op + 64u * k + ((v >> (4 * k - 2)) & 0x3Cu));
  return r;
}

// Nibble operator read from global memory (operators not staged in LDS: the ragged kernel's
// tile shifts for messages of 16 GiB and more; the small kernel's long-message path).
__device__ __forceinline__ u32 opmul_global(const u32* __restrict__ op, u32 v) {
  u32 r = op[v & 15u];
#pragma unroll
  for (int k = 1; k < 8; k++) r ^= op[16 * k + ((v >> (4 * k)) & 15u)];
  return r;
}

// Keep the bytes of a 128-B line window at positions [lo, hi) (0 <= lo, hi <= 128).
__device__ __forceinline__ void keep_bytes(u32x4 (&d)[8], u32 lo, u32 hi) {
#pragma unroll
  for (int b = 0; b < 8; b++) {
#pragma unroll
    for (int x = 0; x < 4; x++) {
      const u32 p = 16u * b + 4u * x;
      u32 keep = 0u;
      if (p + 4u <= hi) keep = 0xFFFFFFFFu;
      else if (p < hi) keep = 0xFFFFFFFFu >> (8u * (p + 4u - hi));
      if (p + 4u <= lo) keep = 0u;
      else if (p < lo) keep &= 0xFFFFFFFFu << (8u * (lo - p));
      d[b][x] &= keep;
    }
  }
}

// keep_bytes for a line window loaded by clamped block loads (blocks past the message end
// hold copies of its last block): bytes [lo, 16) of block 0 (lo <= 15, the head's offset), the
// blocks before the one holding `hi` whole, that block's first hi & 15 bytes, nothing after.
// ~3 VALU per dword against keep_bytes' general [lo, hi) test per dword (the small kernel's
// repack loop over random 1..4096-B messages 51.8 -> 48.2 us per 65,536 slots, r05bv).
__device__ __forceinline__ void keep_sel(u32x4 (&d)[8], u32 lo, u32 hi) {
  const u32 r = hi & 15u, be = hi >> 4;
  u32 m[4];
#pragma unroll
  for (int x = 0; x < 4; x++) {
    const int n = min(max((int)r - 4 * x, 0), 4);
    m[x] = n >= 4 ? 0xFFFFFFFFu : (1u << (8 * n)) - 1u;
  }
#pragma unroll
  for (int b = 0; b < 8; b++) {
    const bool past = 16u * (u32)b >= hi;
    const u32 other = (u32)b == be ? 0u : 0xFFFFFFFFu;
#pragma unroll
    for (int x = 0; x < 4; x++) d[b][x] = past ? 0u : (d[b][x] & (m[x] | other));
  }
#pragma unroll
  for (int x = 0; x < 4; x++) {
    const int n = min(max((int)lo - 4 * x, 0), 4);
    d[0][x] &= n >= 4 ? 0u : (0xFFFFFFFFu << (8 * n));
  }
}

// Byte step with the k=3 step table (plain byte table): crc = (crc >> 8) ^ T[(crc ^ b) & 0xFF].
__device__ __forceinline__ u32 step1(u32 crc, u32 b, u32 lc1) {
  const u32 x = (crc ^ b) & 0xFFu;
  return (crc >> 8) ^ lds_ld(__builtin_amdgcn_perm(x, lc1, 0x0c020400u) + 128);
}

// Wait until every vector-memory access of this wave has completed. Issued right before a
// tile's loads, so a wave never has more than one tile of loads outstanding. Inline asm
// is invisible to hipcc's waitcnt pass, which keeps its own (weaker) waits.
__device__ __forceinline__ void drain_before_issue() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Issue priority around a tile's wait and load issue (every streaming loop: uniform, ragged,
// long, small): a wave raises its priority to SUBSPACE_ISSUE_PRIO while it waits for its tile
// and issues the next one's loads, then drops back to 0 for the lookups. The two waves of a
// SIMD otherwise issue oldest first, so a younger wave whose tile has landed waits behind its
// partner's lookups before its next loads go out. Config B 44.6-45.3 vs 44.9-45.5 us, the
// stride-4,160 plain kernel 45.7 vs 46.4 (interleaved, r03s15/r03s16; profiles/DESIGN_r01-r03.md 4.1).
#ifndef SUBSPACE_ISSUE_PRIO
#define SUBSPACE_ISSUE_PRIO 1
#endif
// The next tile's address computed before the wait for the current one and pinned there
// (uniform and long kernels), so only the load instructions follow the landing: config B
// 45.2-45.7 vs 45.8-45.9 us, slot publish / verify -0.3 / -0.4 us (interleaved, r03s18). The
// ragged and small kernels' next addresses come from records loaded one tile ahead, which
// land with the tile, so theirs cannot move. 0: left to hipcc (A/B builds).
#ifndef SUBSPACE_ADDR_EARLY
#define SUBSPACE_ADDR_EARLY 1
#endif
__device__ __forceinline__ void issue_prio_hi() {
  if constexpr (SUBSPACE_ISSUE_PRIO > 0) __builtin_amdgcn_s_setprio(SUBSPACE_ISSUE_PRIO);
}
__device__ __forceinline__ void issue_prio_lo() {
  if constexpr (SUBSPACE_ISSUE_PRIO > 0) __builtin_amdgcn_s_setprio(0);
}

// Inclusive XOR prefix, in tile order tau = k*nw + w, of the per-tile values at tile tau:
// the XOR of every segment before tau's (segx, exclusive) and of tau's segment up to tau
// (local). A segment is 64 consecutive tiles of one sweep row, s = k*nwb + w/64
// (crc_combine.hip). tau < 2^32 (workspace capacities are bounded on the host).
// Blocked layout of the per-tile values (tilecrc, written by the main kernels' flushes) and of
// their segment prefixes (local, crc_combine.hip): 64 x 64 blocks of (wave w, sweep row k),
// block (k >> 6, w >> 6) at (k >> 6) * nwb + (w >> 6), 16 KiB each. tilecrc holds a block
// w-major (a flush of 64 tiles of one wave is 256 contiguous bytes), local k-major (a segment,
// 64 tiles of one row, is 256 contiguous bytes): the segment scan reads and writes whole 16 KiB
// blocks (tile order and wave-major order cost it 256-B runs at 8-30 KiB strides, r04q).
__device__ __forceinline__ u64 tilecrc_index(u64 w, u64 k, u32 nwb) {
  return ((((k >> 6) * nwb + (w >> 6)) << 6 | (w & 63)) << 6) | (k & 63);
}
__device__ __forceinline__ u64 local_index(u64 w, u64 k, u32 nwb) {
  return ((((k >> 6) * nwb + (w >> 6)) << 6 | (k & 63)) << 6) | (w & 63);
}
__device__ __forceinline__ u32 tile_prefix(const u32* __restrict__ local, const u32* __restrict__ segx, u32 nw,
                                           u32 nwb, u64 tau) {
  const u32 t = (u32)tau, k = t / nw, w = t - k * nw;
  return segx[(u64)k * nwb + (w >> 6)] ^ local[local_index(w, k, nwb)];
}

// Zero a look-back scan's status words and ticket (grid-stride) from a kernel that runs
// after that scan in the same call, leaving the state ready for the next call (or graph
// replay) without a memset (crc_combine.hip).
__device__ __forceinline__ void reset_scan_state(u64* status, u64 nwords, u32* ticket) {
  const u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x, stride = (u64)gridDim.x * blockDim.x;
  for (u64 i = g; i < nwords; i += stride) __hip_atomic_store(&status[i], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (g == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A slot call's mismatch count over its workgroups, without a memset and without one hot word:
// the call's entry of the context's counter ring holds a top word and kCountGroups group words
// (u64, all 0 between calls). Workgroup b adds (1 << 32) | n to group word b % kCountGroups; the
// workgroup that finds the rest of its group done adds the group's total to the top word and
// resets its group word; the one that finds every other group done writes the call's total and
// resets the top word. SUBSPACE_COUNT_GROUPS = 1 (the product): one word, one atomic per
// workgroup -- the two-level form (8) did not shorten the ~2.5 us exit tail of a 65,536-slot
// S_short call (tools/small_timeline.py, r06b vs r06h) and puts a second dependent atomic on the
// last workgroup.
#ifndef SUBSPACE_COUNT_GROUPS
#define SUBSPACE_COUNT_GROUPS 1
#endif
constexpr u32 kCountGroups = SUBSPACE_COUNT_GROUPS;
constexpr u32 kCountWords = 16;  // per call entry: one 128-B line
__device__ __forceinline__ void add_call_mismatches(u64* counter, u32 n, u32* error_count) {
  if constexpr (kCountGroups == 1) {  // one word: the workgroup that sees G - 1 done writes the total
    const u64 old = atomicAdd(reinterpret_cast<unsigned long long*>(counter), (1ull << 32) | (u64)n);
    if ((u32)(old >> 32) == gridDim.x - 1u) {
      *error_count = (u32)old + n;
      __hip_atomic_store(counter, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  const u32 G = gridDim.x, g = blockIdx.x % kCountGroups;
  const u32 ng = (G - g + kCountGroups - 1u) / kCountGroups;  // workgroups of group g
  const u64 old = atomicAdd(reinterpret_cast<unsigned long long*>(counter + 1 + g), (1ull << 32) | (u64)n);
  if ((u32)(old >> 32) == ng - 1u) {
    const u32 tot = (u32)old + n;
    __hip_atomic_store(counter + 1 + g, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const u32 groups = G < kCountGroups ? G : kCountGroups;
    const u64 o2 = atomicAdd(reinterpret_cast<unsigned long long*>(counter), (1ull << 32) | (u64)tot);
    if ((u32)(o2 >> 32) == groups - 1u) {
      *error_count = (u32)o2 + tot;
      __hip_atomic_store(counter, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace subspace_amd
