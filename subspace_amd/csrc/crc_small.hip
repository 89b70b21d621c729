// Small-message kernel: one CRC32 per message of at most 4 KiB, 64 / G messages per 8 KiB tile
// (G = 1 .. 32 lanes per message, the host's choice from the call's length bound; the text
// below describes G = 32, two messages per tile, and the packed forms differ only in the
// counts: message slot mj = lane / G, line li = lane % G, capacity C = 128 G, ring window G
// tiles) -- the slot-list and per-slot-size paths (subspace_crc32_slots with max_message_size <=
// 4096, subspace_crc32_slots_strided with per-slot sizes in slots of <= 4 KiB) and uniform
// batches of messages shorter than 4 KiB. It replaces the ragged pipeline (tile-count scan,
// descriptors, ragged kernel, segment scans, final kernel, slot finish: seven launches,
// ~118 us for 65,536 slots of 4 KiB) with one kernel, because a message of at most one
// half-tile needs neither a tile index nor a cross-tile combine.
//
// Decomposition:
//  * Message m = bytes [s, s + L) of base (s = offsets[m*ostride], L = lengths[m*lstride]),
//    mis = s & 15, extended length E = L + mis. With E <= 4096 it fills one half of a tile:
//    lane l of half h owns the 128-B line [s0 + 128 l, +128) of message 2 tau + h, s0 = s -
//    mis -- the uniform kernel's access shape (64 consecutive lines per load instruction when
//    the two messages are adjacent) and the ragged kernel's alignment rule (whole 16-B
//    blocks from the block holding s; the first mis bytes and the bytes from E on masked).
//  * Waves sweep the tiles like the uniform kernel (order-0 front). A tile's two records
//    are loaded one tile ahead of its lines (vector loads, retired in order with the line
//    loads, as the ragged kernel's descriptors), so line addresses never wait on a record.
//    The host gives no wave more than 32 tiles (more workgroups for longer batches): for G =
//    32 one ring window, so the in-loop flush below never runs; the packed forms flush every G
//    tiles (64 messages) right after the next tile's loads are issued. (Round 4: the same
//    kernel with the flush moved out of the loop -- 0 SGPR spills, no full drain in the loop
//    -- measured 2.3-3.4 us slower per 65,536-slot list, with or without loop padding:
//    profiles/r04/README.md.)
//  * G = 32: a wave whose window holds only whole aligned 4 KiB messages runs the FAST loop
//    (the uniform kernel's loads). Slot lists: a workgroup with any other wave packs all 256 of
//    its messages as one stream of exact 128-B lines (n = ceil(E / 128) per message) that its
//    8 waves share (REPACK2, below; the padding left is p = 128 n - E < 128). Other batches: a
//    wave packs its own window by message size, 2^c lanes per message (REPACK).
//  * Every line load stays inside its message: block b of lane l is read from s0 +
//    min(128 l + 16 b, last block), so the lanes past the end re-read the last block (one
//    cache line) instead of branching around loads, and a half with nothing to read (no
//    message, an empty one, or one too long for this kernel) reads a 16-B block of the step
//    table. Loads never touch a 16-B block that holds no byte of the message (the uniform
//    FAST form excepted: it reads a message's C bytes, the next messages' beyond L, never past
//    the batch; tests/test_kernel_address_model.py).
//  * Line 0 starts from seed = Z_mis^{-1}(init), every other line from 0, so each half gives
//      V = crc_raw(seed, 0^mis || D || 0^p) = Z_p(crc_raw(init, D)),   p = 4096 - E;
//    each message's value and code are parked in a per-wave LDS ring (32 tiles), and every 32
//    tiles (in practice once, after the loop) each lane takes one message of the ring, undoes
//    its padding with p's bits over the inverse operators Z_{2^b}^{-1}, b < 12 (LDS), and
//    stores the CRC.
//  * SLOT: the message-slot checksum (client/checksum.h:29-47 over common/channel.h:527-542's
//    spans) in the same flush, from init 0: with H = crc_raw(~0, span 0 || span 1) from the
//    prefix (the flag set first for a publish, client/publisher.cc:664-675),
//      Z_p(crc_raw(H, payload)) = Z_{p+L}(H) ^ V = Z_4096(Z_mis^{-1}(H)) ^ V,
//    so the padding inverses that finish a plain CRC finish the checksum too; then flag +
//    checksum are stored (publish) or compared (verify: client/client.cc:1346-1356), with no
//    second kernel. The first window's prefix words are loaded in the prologue ahead of tile
//    0's lines and hashed under tile 0's flight (round 4: no prefix round trip in the tail).
//    Strided slots: a size beyond the slot's payload area (a.max_len) is
//    SUBSPACE_CRC_SLOT_OVERSIZE: nothing read, stored or compared.
//  * A message with E > 4096 (longer than the caller's max_message_size bound, or a 4 KiB
//    payload that does not start on a 16-B boundary) is parked as such and computed by the
//    wave's next flush, one at a time by the whole wave, in 8 KiB chunks (acc = Z_8192(acc) ^
//    chunk, the last chunk's padding undone; SLOT: finished as Z_L(H) ^ crc_raw(0, payload)),
//    behind a wave-uniform branch the common case never takes. No list, no second kernel, no
//    code in the tile loop, and a batch of long messages still spreads over every wave.
//  * SLOT verify: mismatches are summed per workgroup by one LDS atomic per wave and over
//    workgroups by one relaxed 64-bit atomic per workgroup on a context counter word that also
//    counts finished workgroups; the last one writes the call's total and resets the word
//    (the fused uniform slot kernel's scheme: no fences, no memset).
#include "crc_device.h"

// Timing-only investigation builds (tools/ab_lib.sh -DSUBSPACE_AB_BUILD -DSUBSPACE_SMALL_VARIANT=n;
// the product is 0, the others compute nothing valid): 1 no prologue span loads / hash; 2 no
// flush; 3 no prefix reload in later windows; 4 no byte masking in the repack loop. A variant
// outside an A/B build is a build error (a stray -D must not ship wrong CRCs).
#ifndef SUBSPACE_SMALL_VARIANT
#define SUBSPACE_SMALL_VARIANT 0
#endif
#ifndef SUBSPACE_SMALL_EARLY_TILE0
#define SUBSPACE_SMALL_EARLY_TILE0 0
#endif
#if (SUBSPACE_SMALL_VARIANT != 0 || SUBSPACE_SMALL_EARLY_TILE0 != 0 || defined(SUBSPACE_RP2_DEBUG) || \
     defined(SUBSPACE_PROBE_PREBAR)) &&                                                                 \
    !defined(SUBSPACE_AB_BUILD)
#error "timing / debug A/B knobs build only with tools/ab_lib.sh (which defines SUBSPACE_AB_BUILD)"
#endif

namespace subspace_amd {

template <int WG, bool SLOT, bool PROBE, int G>
__global__ __launch_bounds__(WG) void crc32_small_kernel(const u32* __restrict__ gtab, const u32* __restrict__ gops,
                                                         SmallArgs a) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  constexpr int NPW = WG / 64;
  // G lanes per message (one 128-B line each): M = 64 / G messages per tile, each of at most
  // C = 128 G extended bytes; a ring window (64 messages) is W = G tiles. G = 32 is the
  // half-tile form (two messages per tile); smaller G packs short messages.
  static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16 || G == 32, "lanes per message");
  constexpr u32 M = 64u / (u32)G, C = 128u * (u32)G, W = (u32)G;
  const u32 sbase = (u32)(uintptr_t)smem;
  const u32 smism = sbase + (u32)small_lds_bytes();  // SLOT: the workgroup's mismatch word
  // experiment hook: realtime stamps (entry, window records landed, barrier, tile 0 landed,
  // loop end, flush end, exit), stored at exit by lanes 0-7 (no store inside the stream)
  u64 pt[7] = {0, 0, 0, 0, 0, 0, 0};
  constexpr bool probe = PROBE;
  if constexpr (probe) pt[0] = __builtin_amdgcn_s_memrealtime();
  LdsFill<WG, kSmallOpSlots> fill;

  const int lane = threadIdx.x & 63;
  const u32 wid = rfl(threadIdx.x >> 6);
  const u32 l = (u32)lane & 31u, h = (u32)lane >> 5;
  const u32 li = (u32)lane % (u32)G, mj = (u32)lane / (u32)G;  // line in its message, message in its tile
  const u32 sring = sbase + kSmallRing + wid * kSmallRingBytesPerWave;  // this wave's result ring
  const u32 lc0 = sbase + (l << 2), lc1 = lc0 + 0x10000u;
  const u32 lop = sbase + kLdsOps + 4u * (31u - l);  // this lane's line-shift operator (G = 32)
  // Z_{128 (G-1-li)}: the lines after this one in its message (slot s of the table is Z_{128 s})
  const u32 lopg = sbase + kLdsOps + 4u * ((u32)G - 1u - li);
  const u32 z64 = sbase + kLdsOps + 512u * (u32)kUniSlotOpZ64 + 4u * (u32)(lane & 3);
  const u64 count = a.count;
  const uint8_t* const base = a.base;
  const u64 ntiles = (count + M - 1) / M;
  const u64 nw = (u64)gridDim.x * NPW;
  const u64 t0 = front_slot(blockIdx.x, gridDim.x, wid);
  const u32 nk = t0 < ntiles ? (u32)((ntiles - t0 + nw - 1) / nw) : 0u;  // tiles tau = t0 + k*nw
  const uint8_t* safe = reinterpret_cast<const uint8_t*>(gtab);  // 16 readable bytes
  const bool calc = a.mode == 0u;

  // this lane's message in tile k (present: k < nk and m < count)
  auto msg_of = [&](u32 k) __attribute__((always_inline)) { return M * (t0 + (u64)k * nw) + (u64)mj; };
  // Lane i's message of the first window (tile i / M, message i % M): the flush's message, and
  // the record lane i holds for the tile loop (clamped into the batch like every record load)
  const u64 fm = M * (t0 + (u64)((u32)lane / M) * nw) + ((u32)lane % M);
  const bool flive = ((u32)lane / M) < nk && fm < count;
  const u64 fmc = fm < count ? fm : count - 1;
  // Message m's record: offset and length from the arrays, or (a uniform batch: no offsets)
  // m * ustride and ulen (a kernel-argument branch)
  auto record = [&](u64 m, u64& s, u64& L) __attribute__((always_inline)) {
    if (a.offsets) {
      const u64* po = a.offsets + m * a.ostride;
      const u64* pl = a.lengths + m * a.lstride;
      s = *po;
      L = *pl;
      asm volatile("" ::"v"(po), "v"(pl));  // (addresses live past the loads: load_at)
    } else {
      s = m * a.ustride;
      L = a.ulen;
    }
  };
  // The record of this lane's message in tile k, clamped into the batch (every record load reads
  // a real record; whether the lane's slot holds a message is decided from k and m when used).
  auto fetch = [&](u32 k, u64& s, u64& L) __attribute__((always_inline)) {
    const u32 kk = k < nk ? k : (nk ? nk - 1 : 0u);
    u64 m = nk ? msg_of(kk) : 0;
    m = m < count ? m : count - 1;
    record(m, s, L);
  };
  // The window's records, loaded once in the prologue (lane i: message i of the first window),
  // and tile k's record for this lane's half broadcast from them (k < 32; clamped as fetch's)
  u64 wS = 0, wL = 0;
  auto readlane64 = [&](u64 v, int i) __attribute__((always_inline)) {
    return ((u64)(u32)__builtin_amdgcn_readlane((int)(u32)(v >> 32), i) << 32) |
           (u64)(u32)__builtin_amdgcn_readlane((int)(u32)v, i);
  };
  auto win_rec = [&](u32 k, u64& s, u64& L) __attribute__((always_inline)) {
    u32 kk = k < nk ? k : (nk ? nk - 1 : 0u);
    kk = kk < kSmallRingTiles ? kk : kSmallRingTiles - 1u;
    const int i0 = (int)(2u * kk);
    const u64 s0 = readlane64(wS, i0), s1 = readlane64(wS, i0 + 1);
    const u64 L0 = readlane64(wL, i0), L1 = readlane64(wL, i0 + 1);
    s = h ? s1 : s0;
    L = h ? L1 : L0;
  };
  // Extended bytes this kernel reads for tile k's half as a half-tile (0: nothing -- no
  // message, an empty one, or one longer than a half-tile, computed apart: long_crc).
  auto ext = [&](u32 k, u64 s, u64 L) __attribute__((always_inline)) -> u32 {
    const u64 E = L + (s & 15u);
    return (k < nk && msg_of(k) < count && L != 0 && E <= C && (!SLOT || L <= a.max_len)) ? (u32)E : 0u;
  };
  auto load_lines_at = [&](u32x4 (&D)[8], u64 s, u32 E, u32 line) __attribute__((always_inline)) {
    const uint8_t* p0 = E ? base + (s & ~(u64)15) : safe;
    const u32 lastb = E ? (E - 1u) & ~15u : 0u;  // the block holding the message's last byte
    const u32x4* q[8];
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const u32 off = 128u * line + 16u * (u32)b;
      q[b] = reinterpret_cast<const u32x4*>(p0 + (off < lastb ? off : lastb));
      D[b] = *q[b];
    }
    // (the addresses live past the loads: none of their VGPRs becomes a load's destination,
    // load_at)
#pragma unroll
    for (int b = 0; b < 8; b++) asm volatile("" ::"v"(q[b]));
    // keep the loads at this point, in order (hipcc otherwise sinks them into the compute)
    __builtin_amdgcn_sched_barrier(0);
  };
  auto load_lines = [&](u32x4 (&D)[8], u64 s, u32 E) __attribute__((always_inline)) { load_lines_at(D, s, E, li); };
#ifdef SUBSPACE_RP2_DEBUG
  // (A/B debug builds) REPACK2: the line this lane is about to load must be line li < n of the
  // message of ring entry q (wave q / 32's window message q % 32); else print and load nothing
  auto rp2_check = [&](const char* where, u64 s, u32& E, u32 li, u32 q) __attribute__((always_inline)) {
    if (E == 0u) return;
    const u32 w2 = q >> 5, i2 = q & 31u;
    const u64 t02 = front_slot(blockIdx.x, gridDim.x, w2);
    const u64 m2 = 2u * (t02 + (u64)(i2 >> 1) * nw) + (i2 & 1u);
    u64 rs = 0, rL = 0;
    if (m2 < count) record(m2, rs, rL);
    const u32 n2 = (E + 127u) >> 7;
    if (m2 >= count || rs != s || rL + (rs & 15u) != E || li >= n2) {
      printf("RP2 %s wg %u wave %u lane %d: q %u m %llu s %llx rec %llx E %u rec %llu li %u\n", where, blockIdx.x, wid,
             lane, q, (unsigned long long)m2, (unsigned long long)s, (unsigned long long)rs, E,
             (unsigned long long)rL, li);
      E = 0u;
    }
  };
#endif
  // FAST path: the tile's line offset from base, computed (and pinned) before the wait for
  // the previous tile, then 8 loads at immediate offsets (the uniform kernel's issue)
  auto fast_off = [&](u32 k) __attribute__((always_inline)) {
    u64 s, L;
    win_rec(k, s, L);
    u64 off = s + 128u * l;
    asm volatile("" : "+v"(off));
    return off;
  };
  auto load_at = [&](u32x4 (&D)[8], u64 off) __attribute__((always_inline)) {
    const u32x4* q = reinterpret_cast<const u32x4*>(base + off);
#pragma unroll
    for (int b = 0; b < 8; b++) D[b] = q[b];
    // the address stays live past the last load: hipcc otherwise hands its (dead) VGPRs to that
    // load as its destination, and the loop ran ~8 us slower per 65,536-slot call (r05,
    // tools/load_overlap.py)
    asm volatile("" ::"v"(q));
    __builtin_amdgcn_sched_barrier(0);
  };
  // Z_{2^b}^{-1} applied for the set bits of `bits` (b < nb <= 12; wave-uniform loop over the
  // bits any lane has): Z_mis^{-1} and the padding inverses Z_p^{-1}
  // (an operator only where some lane has the bit: a batch of one size has one padding, and
  // its bits cost one opmul each instead of every bit below the highest)
  auto inv_bits = [&](u32 x, u32 bits, int nb) __attribute__((always_inline)) {
    for (int b = 0; b < nb && __any(bits != 0u); b++) {
      if (__any((bits & 1u) != 0u)) {
        const u32 xm = opmul(sbase, kSmallOpInv + b, x);
        x = (bits & 1u) ? xm : x;
      }
      bits >>= 1;
    }
    return x;
  };

  // SLOT: the prefix terms of a slot: H = crc_raw(~0, span 0 || span 1) with the flag word as
  // stored (kMessageHasChecksum set first for a publish), the flag word F, the stored checksum
  // S (prefix + 48) and whether the flag was set. Prefixes are 8-B aligned (the C ABI's rule):
  // 8-B loads.
  constexpr u32 kW = kSlotFusedMaxMeta / 4 + 2;
  auto span_load = [&](const uint8_t* pfx, u32 (&w)[14]) __attribute__((always_inline)) {
    const u64* q = reinterpret_cast<const u64*>(pfx);
#pragma unroll
    for (int i = 0; i < 7; i++) {
      const u64 x = q[i];
      w[2 * i] = (u32)x;
      w[2 * i + 1] = (u32)(x >> 32);
    }
    asm volatile("" ::"v"(q));  // (the address lives past the loads: no load's destination, load_at)
  };
  // (span 1, the metadata, is loaded by the hash itself: the prologue keeps only the 14 prefix
  // words live across its barrier; r06: with kW more, the slot kernel spilled VGPRs to scratch
  // and the reload after the barrier waited for every load, tile 0's lines included)
  auto span_hash = [&](const uint8_t* pfx, u32 (&w)[14], u32& F, u32& S, bool& has) __attribute__((always_inline))
      -> u32 {
    // w[0] (the padding) and w[13] (not hashed) stay live until here: hipcc reuses a dead
    // destination of a pending prefix load for other values, and the reuse waits for that load
    // (r05: a vmcnt wait that put the prefix round trip in front of tile 0's lines)
    asm volatile("" ::"v"(w[0]), "v"(w[13]));
    has = (w[8] & 4u) != 0u;  // kMessageHasChecksum (common/channel.h:62-70)
    F = calc ? (w[8] | 4u) : w[8];
    w[8] = F;
    S = w[12];
    u32 hh = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 1; i < 12; i++) hh = step4(hh ^ w[i], lc0, lc1);
    if (a.metadata_size) {  // wave-uniform: span 1 after the checksum area (crc_uniform.hip),
                            // realigned with a uniform byte shift; full words by step4, the tail by bytes
      const u32 o1 = 48u + a.checksum_size, sh = o1 & 3u, ms = a.metadata_size;
      const u32 nwords = (sh + ms + 3u) >> 2;
      const u32* p1 = reinterpret_cast<const u32*>(pfx + (o1 & ~3u));
      u32 W1[kW];
#pragma unroll
      for (u32 j = 0; j < kW; j++) W1[j] = j < nwords ? p1[j] : 0u;
      u32 tail = 0;
#pragma unroll
      for (u32 j = 0; j + 1 < kW; j++) {
        const u32 x = __builtin_amdgcn_alignbyte(W1[j + 1], W1[j], sh);
        if (j < (ms >> 2)) hh = step4(hh ^ x, lc0, lc1);
        if (j == (ms >> 2)) tail = x;
      }
      for (u32 b = 0; b < (ms & 3u); b++) hh = step1(hh, (tail >> (8u * b)) & 0xFFu, lc1);
    }
    return hh;
  };
  auto span_crc = [&](const uint8_t* pfx, u32& F, u32& S, bool& has) __attribute__((always_inline)) -> u32 {
    u32 w[14];
    span_load(pfx, w);
    return span_hash(pfx, w, F, S, has);
  };

  // A message longer than a half-tile, by the whole wave (s, L, P wave-uniform): 8 KiB chunks
  // as the ragged kernel's tiles (lines, line shifts, halves joined by Z_4096), acc =
  // Z_8192(acc) ^ chunk, the last chunk's padding p = 8192 nt - E < 8192 undone (b < 12 from
  // LDS, b = 12 from global memory). Returns crc_raw(init, D); SLOT: crc_raw(~0, spans || D),
  // i.e. Z_L(H) ^ crc_raw(0, D) with L's bits over Z_{2^k} (global).
  auto long_crc = [&](u64 s, u64 L, u64 P) __attribute__((always_inline)) -> u32 {
    const u32 mis = (u32)s & 15u;
    const u64 E = L + mis, nt = (E + 8191) >> 13;
    const uint8_t* p0 = base + (s & ~(u64)15);
    const u32 seed = inv_bits(a.init, mis, 4);
    u32 acc = 0;
    for (u64 j = 0; j < nt; j++) {
      const u64 rest = E - (j << 13);
      const u32 len = rest < 8192 ? (u32)rest : 8192u;
      const u32 lastb = (len - 1u) & ~15u;
      const uint8_t* pj = p0 + (j << 13);
      u32x4 d[8];
      const u32x4* q[8];
#pragma unroll
      for (int b = 0; b < 8; b++) {
        const u32 off = 128u * (u32)lane + 16u * (u32)b;
        q[b] = reinterpret_cast<const u32x4*>(pj + (off < lastb ? off : lastb));
        d[b] = *q[b];
      }
#pragma unroll
      for (int b = 0; b < 8; b++) asm volatile("" ::"v"(q[b]));  // (load_lines)
      const bool hd = j == 0 && mis != 0u && lane == 0;
      if (__any(hd || len < 8192u)) {
        const int v0 = (int)len - 128 * lane;
        const u32 hi = v0 <= 0 ? 0u : (v0 >= 128 ? 128u : (u32)v0);
        keep_bytes(d, hd ? mis : 0u, hi);
      }
      const u32 crc = line_crc32_2chain(d, (j == 0 && lane == 0) ? seed : 0u, lc0, lc1, z64);
      u32 v = lane_shift(lop, crc);  // lanes 0-31: bytes 0..4095 of the chunk, 32-63: the rest
      v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
      v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
      v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
      v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
      v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
      const u32 h0 = (u32)__builtin_amdgcn_readlane((int)v, 31), h1 = (u32)__builtin_amdgcn_readlane((int)v, 63);
      const u32 c = opmul(sbase, kUniSlotOpZ4096, h0) ^ h1;
      acc = j ? opmul_global(a.rops + kLaneOpWords + 128, acc) ^ c : c;  // Z_8192: the first tile shift
    }
    const u32 pad = (u32)((nt << 13) - E);
    acc = inv_bits(acc, pad & 0xFFFu, kSmallInvOps);
    if (pad & 0x1000u) acc = opmul_global(a.rops + kRagInvOps + 128 * 12, acc);
    if constexpr (SLOT) {
      u32 F, S;
      bool has;
      u32 R = span_crc(base + P - a.pdelta, F, S, has);
      for (int b = 0; b < 64 && (L >> b); b++)
        if ((L >> b) & 1u) R = opmul_global(a.pow2 + 128 * b, R);
      acc ^= R;
    }
    return acc;
  };

  // SLOT: store flag + checksum (publish) or the status (verify) of slot m; counts mismatches
  u32 mism = 0;
  auto slot_store = [&](bool live, bool oversize, u64 m, const uint8_t* pfx, u32 F, u32 S, bool has, u32 R)
                        __attribute__((always_inline)) {
    const u32 res = ~R;  // *reinterpret_cast<uint32_t*>(checksum.data()) = ~crc (client/checksum.h:36)
    if (oversize && a.status) a.status[m] = 4u;  // SUBSPACE_CRC_SLOT_OVERSIZE
    if (calc) {
      if (live) {
        u32* pw = reinterpret_cast<u32*>(const_cast<uint8_t*>(pfx));
        pw[8] = F;     // SetHasChecksum()
        pw[12] = res;
        if (a.status) a.status[m] = 0u;
        if (a.crc_out) a.crc_out[m] = res;
      }
    } else {
      const u32 st = !has ? 2u : (res == S ? 0u : 1u);  // client/checksum.h:46
      if (live && a.status) a.status[m] = st;
      mism += (u32)__builtin_popcountll(__ballot(live && st == 1u));
    }
  };

  // Each message's value and code are parked in the wave's LDS ring, entry 2 (k & 31) + h.
  // Code: p = 4096 - E (bits 0-11) | mis << 12 for a half-tile message (value: Z_p(crc_raw(
  // init, D))); kCodeLong for a longer one (computed by the flush: long_crc); kCodeEmpty for
  // length 0 (CRC init ^ final_xor; a checksum over the spans only); kCodeSkip for no message;
  // SLOT: kCodeOversize for a size beyond the slot's payload area (nothing read or stored).
  constexpr u32 kCodeOversize = 0x10000000u, kCodeLong = 0x20000000u, kCodeEmpty = 0x40000000u,
                kCodeSkip = 0x80000000u;
  // A message's value from its lines' CRCs: line li -> Z_{128 (G-1-li)}(line), XOR over the
  // message's G lanes (DPP). G = 32: row_shr 1/2/4/8 + row_bcast:15 leave each half's total in
  // its last lane (31, 63); G <= 16: a butterfly (quad_perm xor 1, xor 2, row_half_mirror,
  // row_mirror) leaves the group's total in every lane of the group.
  auto msg_value = [&](u32 crc) __attribute__((always_inline)) -> u32 {
    if constexpr (G == 32) {
      u32 v = lane_shift(lop, crc);
      v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
      v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
      v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
      v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
      v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
      return v;
    } else {
      u32 v = G == 1 ? crc : lane_shift(lopg, crc);
      if constexpr (G >= 2) v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
      if constexpr (G >= 4) v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
      if constexpr (G >= 8) v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
      if constexpr (G >= 16) v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false); // row_mirror
      return v;
    }
  };
  // Inclusive scan over the wave's 64 lanes (XOR or add): row_shr 1/2/4/8 within rows, then
  // row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3) across them
  auto wave_scan = [&](u32 x, bool xr) __attribute__((always_inline)) -> u32 {
    auto op = [&](u32 y) { x = xr ? (x ^ y) : (x + y); };
    op((u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false));  // row_shr:1
    op((u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false));  // row_shr:2
    op((u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false));  // row_shr:4
    op((u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false));  // row_shr:8
    op((u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));  // row_bcast:15
    op((u32)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));  // row_bcast:31
    return x;
  };
  auto process = [&](const u32x4 (&cur)[8], u64 s, u64 L, u32 k) __attribute__((always_inline)) {
    const u32 mis = (u32)s & 15u;
    const u32 E = ext(k, s, L);
    u32x4 d[8];
#pragma unroll
    for (int b = 0; b < 8; b++) d[b] = cur[b];
    // Head: line 0's first mis bytes precede the message. Tail: bytes from E on (the
    // re-read last block included). Each lane keeps only its line's message bytes.
    const bool head = E != 0u && mis != 0u && li == 0u;
    if (__any(head || E < C)) {
      const int v0 = (int)E - 128 * (int)li;
      const u32 hi = v0 <= 0 ? 0u : (v0 >= 128 ? 128u : (u32)v0);
      // (slot kernels: keep_sel, r05bw; the non-slot instantiation measured slower with it on
      // uniform 4,000-B batches, 57.0 -> 61.5 us per 256 MiB, and keeps keep_bytes)
      if constexpr (SLOT)
        keep_sel(d, head ? mis : 0u, hi);
      else
        keep_bytes(d, head ? mis : 0u, hi);
    }
    u32 seed = a.init;  // Z_mis^{-1}(init): after the mis masked bytes the state is init
    if (seed != 0u && __any(head)) seed = inv_bits(seed, mis, 4);
    // (G = 1, every message of the tile within 64 bytes: the line's second half is zeros)
    const u32 crc = G == 1 && __all(E <= 64u) ? line_crc32_lo(d, seed, lc0, lc1, z64)
                                              : line_crc32_2chain(d, li == 0u ? seed : 0u, lc0, lc1, z64);
    const u32 v = msg_value(crc);
    const u64 m = msg_of(k);
    const bool present = k < nk && m < count;
    const bool over = present && L + mis > C;
    const u32 code = !present              ? kCodeSkip
                   : SLOT && L > a.max_len ? kCodeOversize
                   : over                  ? kCodeLong
                   : L == 0                ? kCodeEmpty
                                           : (C - E) | (mis << 12);
    // the message's last lane: its value and code, one 8-B LDS store
    if (li == (u32)G - 1u) lds_st64(sring + 8u * ((k & (W - 1u)) * M + mj), (u64)v | ((u64)code << 32));
  };
  // FAST: a whole 16-B-aligned 4 KiB message per half (mis = 0, no padding: code 0); line 0 from
  // init itself
  auto process_fast = [&](const u32x4 (&cur)[8], u32 k) __attribute__((always_inline)) {
    const u32 crc = line_crc32_2chain(cur, l == 0u ? a.init : 0u, lc0, lc1, z64);
    u32 v = lane_shift(lop, crc);
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    const u32 code = (k < nk && msg_of(k) < count) ? 0u : kCodeSkip;
    if (l == 31u) lds_st64(sring + 8u * (2u * (k & (kSmallRingTiles - 1u)) + h), (u64)v | ((u64)code << 32));
  };
  auto bperm = [&](u32 e, u32 v) __attribute__((always_inline)) {  // lane e's v
    return (u32)__builtin_amdgcn_ds_bpermute((int)(e << 2), (int)v);
  };
  // UNIFORM FAST (no slots; G = 32 too since r05ca: 2-4 KiB messages 14-20 % faster than the
  // repack loop): a uniform batch of messages of L <= C bytes on 16-B
  // boundaries -- the tile's address from m * stride, one address and 8 immediate-offset loads
  // (reading C bytes per message: past L they are the next messages' bytes, masked), one padding
  // p = C - L for every message, no codes. A tile holding a message whose C bytes would reach
  // past the batch (the last few) takes the clamped loads instead.
  const u64 uL = a.ulen;
  const u32 upad = C - (u32)(uL < C ? uL : C);
  // the last message whose C-byte read stays inside the batch (none: -1)
  const int64_t usafe = upad == 0u ? (int64_t)count - 1
                        : a.ustride == 0 ? -1
                                         : (int64_t)count - 1 - (int64_t)((upad + a.ustride - 1) / a.ustride);
  auto u_off = [&](u32 k) __attribute__((always_inline)) {
    const u32 kk = k < nk ? k : (nk ? nk - 1 : 0u);
    u64 m = msg_of(kk);
    m = m < count ? m : count - 1;
    u64 off = m * a.ustride + 128u * li;
    asm volatile("" : "+v"(off));
    return off;
  };
  auto u_safe = [&](u32 k) __attribute__((always_inline)) {  // wave-uniform: the tile's last message
    const u32 kk = k < nk ? k : (nk ? nk - 1 : 0u);
    return (int64_t)(M * (t0 + (u64)kk * nw) + M - 1) <= usafe;
  };
  auto u_load = [&](u32x4 (&D)[8], u32 k, u64 q) __attribute__((always_inline)) {
    if (u_safe(k)) {
      load_at(D, q);
    } else {
      const u32 kk = k < nk ? k : (nk ? nk - 1 : 0u);
      u64 m = msg_of(kk);
      m = m < count ? m : count - 1;
      load_lines(D, m * a.ustride, (u32)uL);
    }
  };
  auto process_u = [&](const u32x4 (&cur)[8], u32 k) __attribute__((always_inline)) {
    u32x4 d[8];
#pragma unroll
    for (int b = 0; b < 8; b++) d[b] = cur[b];
    if (upad != 0u) {  // (uniform) the bytes from L on
      const int v0 = (int)uL - 128 * (int)li;
      keep_bytes(d, 0u, v0 <= 0 ? 0u : (v0 >= 128 ? 128u : (u32)v0));
    }
    const u32 crc = G == 1 && uL <= 64u ? line_crc32_lo(d, a.init, lc0, lc1, z64)
                                        : line_crc32_2chain(d, li == 0u ? a.init : 0u, lc0, lc1, z64);
    const u32 v = msg_value(crc);
    const u32 code = (k < nk && msg_of(k) < count) ? 0u : kCodeSkip;
    if (li == (u32)G - 1u) lds_st64(sring + 8u * ((k & (W - 1u)) * M + mj), (u64)v | ((u64)code << 32));
  };
  auto flush_u = [&](u32 kf, u32 nt) __attribute__((always_inline)) {
    wave_lds_sync();
    const u32 hh = (u32)lane % M, ti = (u32)lane / M;
    const u64 e = lds_ld64(sring + 8u * (u32)lane);
    const u64 m = M * (t0 + (u64)(kf + ti) * nw) + hh;
    const u32 r = upad ? inv_bits((u32)e, upad, kSmallInvOps) : (u32)e;
    if (ti < nt && (u32)(e >> 32) == 0u) a.out[m] = r ^ a.final_xor;
    wave_lds_sync();
  };
  // PACKED UNIFORM FAST (round 6, VERDICT r05 item 4: packed application buffers): the same loop
  // for strides that are not multiples of 16 -- message m starts mis = (m * stride) & 15 bytes
  // into its first block, one address and 8 immediate-offset loads per lane from that block
  // (C >= L + 15 from the host), its line 0 masks the mis bytes and starts from Z_mis^{-1}(init)
  // (16 seeds, one per lane, picked by ds_bpermute), its lines keep E = L + mis bytes (keep_sel:
  // the bytes past E are whatever follows, all masked) and its padding C - E travels with its
  // value to the flush (the general loop's clamped loads, record arithmetic and per-tile seed
  // inverses ran 200 / 1,000 / 1,500 / 3,000-B packed messages at 33-43 % of HBM, r05cc). The
  // 16-B-stride loop above stays as it was: sharing one body cost it 7 us per 256 MiB of 2,000 and
  // 4,000-B messages (r06k).
  u32 useed = 0;  // lane l: Z_{l & 15}^{-1}(init)
  auto u_off_p = [&](u32 k) __attribute__((always_inline)) {
    const u32 kk = k < nk ? k : (nk ? nk - 1 : 0u);
    u64 m = msg_of(kk);
    m = m < count ? m : count - 1;
    u64 off = ((m * a.ustride) & ~(u64)15) + 128u * li;
    asm volatile("" : "+v"(off));
    return off;
  };
  auto u_load_p = [&](u32x4 (&D)[8], u32 k, u64 q) __attribute__((always_inline)) {
    if (u_safe(k)) {
      load_at(D, q);
    } else {
      const u32 kk = k < nk ? k : (nk ? nk - 1 : 0u);
      u64 m = msg_of(kk);
      m = m < count ? m : count - 1;
      const u64 so = m * a.ustride;
      load_lines(D, so, (u32)uL + ((u32)so & 15u));
    }
  };
  auto process_up = [&](const u32x4 (&cur)[8], u32 k) __attribute__((always_inline)) {
    u32x4 d[8];
#pragma unroll
    for (int b = 0; b < 8; b++) d[b] = cur[b];
    const u32 mis = (u32)(msg_of(k) * a.ustride) & 15u;
    const u32 E = (u32)uL + mis;
    const int v0 = (int)E - 128 * (int)li;
    keep_sel(d, li == 0u ? mis : 0u, v0 <= 0 ? 0u : (v0 >= 128 ? 128u : (u32)v0));
    const u32 seed = bperm(mis, useed);
    const u32 crc = G == 1 && __all(E <= 64u) ? line_crc32_lo(d, seed, lc0, lc1, z64)
                                              : line_crc32_2chain(d, li == 0u ? seed : 0u, lc0, lc1, z64);
    const u32 v = msg_value(crc);
    const u32 code = (k < nk && msg_of(k) < count) ? C - E : kCodeSkip;
    if (li == (u32)G - 1u) lds_st64(sring + 8u * ((k & (W - 1u)) * M + mj), (u64)v | ((u64)code << 32));
  };
  auto flush_up = [&](u32 kf, u32 nt) __attribute__((always_inline)) {
    wave_lds_sync();
    const u32 hh = (u32)lane % M, ti = (u32)lane / M;
    const u64 e = lds_ld64(sring + 8u * (u32)lane);
    const u64 m = M * (t0 + (u64)(kf + ti) * nw) + hh;
    const u32 code = (u32)(e >> 32);
    const bool live = ti < nt && code != kCodeSkip;
    const u32 r = inv_bits((u32)e, live ? code : 0u, kSmallInvOps);
    if (live) a.out[m] = r ^ a.final_xor;
    wave_lds_sync();
  };
  // REPACK (G = 32 kernels): a wave whose window is every tile of the wave (nk <= 32) and not
  // FAST packs its window's messages into tiles by size: entry e (lane e's record, read by
  // ds_bpermute) of E = L + (s & 15) bytes in [1, 4096] gets g_e = 2^c lanes, the least power of
  // two with 128 g_e >= E; the entries are laid out by class, 32-lane ones first, so every
  // group sits on a multiple of its size and never straddles a tile (sum of g_e / 64 tiles
  // instead of nk). Lane li' of a group applies Z_{128 (31-li')} -- the value as if the message
  // filled a half-tile (its lines past g_e contribute 0) -- then the butterfly's first c steps
  // (row_bcast:15 for the 32-lane step), so the ring, codes (p = 4096 - E) and flush are the
  // general loop's. Entries without lanes (none, empty, longer than 4 KiB, SLOT oversize) have
  // their codes written to the ring in the prologue.
  // class c's first lane position | first sorted index << 16, in lane c (one VGPR: kept out of
  // the SGPRs the other loops use)
  u32 vbn = 0;
  u32 vT = 0, vS = 0, rnt = 0;  // lane positions used; sorted index (this lane) -> entry; tiles
  u32 rcmax = 0;        // the largest class present
  bool rident = false;  // uniform layout: entry = position >> rcmax (entries with lanes: rmask)
  u64 rmask = 0;
  // packed tile j, this lane: entry | line in its group << 8 | class << 16 | present << 24
  auto rp_map = [&](u32 j) __attribute__((always_inline)) -> u32 {
    const u32 P = (j << 6) + (u32)lane;
    if (rident) {  // (wave-uniform) entry e at lanes e 2^rcmax .. (a channel's common case)
      const u32 e = P >> rcmax;
      const bool pres = P < vT && ((rmask >> (e & 63u)) & 1ull);
      return (pres ? e : 0u) | ((P & ((1u << rcmax) - 1u)) << 8) | (rcmax << 16) | ((u32)pres << 24);
    }
    u32 c = 5u, b0 = 0u, n0 = 0u;
#pragma unroll
    for (int q = 4; q >= 0; q--) {
      const u32 bq = (u32)__builtin_amdgcn_readlane((int)vbn, q);
      const bool in = P >= (bq & 0xFFFFu);
      c = in ? (u32)q : c;
      b0 = in ? (bq & 0xFFFFu) : b0;
      n0 = in ? (bq >> 16) : n0;
    }
    const u32 off = P - b0;
    const bool pres = P < vT;
    const u32 e = bperm(pres ? n0 + (off >> c) : 0u, vS);
    return e | ((off & ((1u << c) - 1u)) << 8) | (c << 16) | ((u32)pres << 24);
  };
  auto rp_rec = [&](u32 map, u64& s, u64& L) __attribute__((always_inline)) {
    const u32 e = map & 0xFFu;
    s = ((u64)bperm(e, (u32)(wS >> 32)) << 32) | (u64)bperm(e, (u32)wS);
    L = (u64)bperm(e, (u32)wL);
  };
  auto rp_ext = [&](u64 s, u64 L, u32 map) __attribute__((always_inline)) -> u32 {
    return (map >> 24) ? (u32)(L + (s & 15u)) : 0u;
  };
  auto process_rp = [&](const u32x4 (&cur)[8], u64 s, u64 L, u32 map) __attribute__((always_inline)) {
    const u32 rli = (map >> 8) & 31u, c = (map >> 16) & 7u, g = 1u << c;
    const u32 mis = (u32)s & 15u;
    const u32 E = rp_ext(s, L, map);
    u32x4 d[8];
#pragma unroll
    for (int b = 0; b < 8; b++) d[b] = cur[b];
    const bool head = E != 0u && mis != 0u && rli == 0u;
    if (SUBSPACE_SMALL_VARIANT != 4 && __any(head || E < 128u * g)) {
      const int v0 = (int)E - 128 * (int)rli;
      const u32 hi = v0 <= 0 ? 0u : (v0 >= 128 ? 128u : (u32)v0);
      // (slot kernels: keep_sel, r05bw; the non-slot instantiation measured slower with it on
      // uniform 4,000-B batches, 57.0 -> 61.5 us per 256 MiB, and keeps keep_bytes)
      if constexpr (SLOT)
        keep_sel(d, head ? mis : 0u, hi);
      else
        keep_bytes(d, head ? mis : 0u, hi);
    }
    u32 seed = a.init;
    if (seed != 0u && __any(head)) seed = inv_bits(seed, mis, 4);
    const u32 crc = line_crc32_2chain(d, rli == 0u ? seed : 0u, lc0, lc1, z64);
    u32 v = lane_shift(sbase + kLdsOps + 4u * (31u - rli), crc);
    // (each step only when some group needs it: the wave-uniform largest class)
    if (rcmax >= 1u) {
      const u32 t = (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
      v ^= c >= 1u ? t : 0u;
    }
    if (rcmax >= 2u) {
      const u32 t = (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
      v ^= c >= 2u ? t : 0u;
    }
    if (rcmax >= 3u) {
      const u32 t = (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
      v ^= c >= 3u ? t : 0u;
    }
    if (rcmax >= 4u) {
      const u32 t = (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);  // row_mirror
      v ^= c >= 4u ? t : 0u;
    }
    if (rcmax >= 5u) {
      const u32 t = (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15 (rows 1, 3)
      v ^= c >= 5u ? t : 0u;
    }
    const u32 code = (kSmallMaxExt - E) | (mis << 12);
    if ((map >> 24) && rli == g - 1u) lds_st64(sring + 8u * (map & 0xFFu), (u64)v | ((u64)code << 32));
  };
  // SLOT: lane i's message of the first window (fm): its record's prefix offset, and (after
  // the barrier) the prefix terms, from words loaded in the prologue
  u64 fpre = 0;
  u32 eF = 0, eS = 0, eH = 0;
  bool ehas = false;
  // Finish and store the ring's tiles kf .. kf+nt-1 (nt <= 32): lane i takes message i of the
  // window, i.e. tile kf + i/2, half i & 1 (its value and code from the ring; a slot's prefix
  // offset from its record again).
  // SLOT, G < 32 (windows of G tiles, an in-loop flush every window): a window's prefix offsets
  // are loaded at the previous window's flush and its prefix words at its own flush before the
  // next tile's loads are issued (flush_issue), so the flush's reads wait for neither a record
  // round trip nor that tile (vmcnt retires in order); flush_any(..., true) hashes them.
  u64 Pn = 0, Pc = 0;  // the next / current window's prefix offset of this lane's entry
  u32 fw[14];
  auto win_pref = [&](u32 kf) __attribute__((always_inline)) -> u64 {
    const u32 ti = (u32)lane / M, hh = (u32)lane % M;
    const u64 m = M * (t0 + (u64)(kf + ti) * nw) + hh;
    return a.prefixes[(kf + ti < nk && m < count ? m : 0) * a.pstride];
  };
  auto flush_issue = [&](u32 kf) __attribute__((always_inline)) {
    if (kf != 0) {
      Pc = Pn;
      span_load(base + Pc - a.pdelta, fw);
    }
    Pn = win_pref(kf + W);
  };
  auto flush_any = [&](u32 kf, u32 nt, bool pre) __attribute__((always_inline)) {
    wave_lds_sync();
    const u32 hh = (u32)lane % M, ti = (u32)lane / M;
    const bool valid = ti < nt;
    const u64 e = lds_ld64(sring + 8u * (u32)lane);
    u32 v = (u32)e;
    const u32 code = valid ? (u32)(e >> 32) : kCodeSkip;
    const u64 m = M * (t0 + (u64)(kf + ti) * nw) + hh;
    const u64 mc = code != kCodeSkip ? m : 0;  // (a real record for every lane)
    // rare: messages longer than a half-tile, one at a time by the whole wave
    u64 msk = __ballot(code == kCodeLong);
    while (msk) {
      const u32 src = (u32)__builtin_ctzll(msk);
      msk &= msk - 1;
      const u64 ms = M * (t0 + (u64)(kf + src / M) * nw) + src % M;
      u64 s, L;
      record(ms, s, L);
      const u64 P = SLOT ? a.prefixes[ms * a.pstride] : 0;
      const u32 r = long_crc(s, L, P);
      v = lane == (int)src ? r : v;
    }
    const bool half = code < kCodeOversize;  // a half-tile message: Z_p undone here
    if constexpr (SLOT) {
      const bool oversize = code == kCodeOversize;
      const bool live = code != kCodeSkip && !oversize;
      // the first window's prefix terms come from the prologue (every window, under the host's
      // grid rule); a later window's are loaded here
      const uint8_t* pfx =
          (kf == 0 ? flive : live) ? base + (kf == 0 ? fpre : (pre ? Pc : a.prefixes[mc * a.pstride])) - a.pdelta
                                   : safe;  // (a read-only block)
      u32 F = eF, S = eS, H = eH;
      bool has = ehas;
      if (kf != 0 && SUBSPACE_SMALL_VARIANT != 3) H = pre ? span_hash(pfx, fw, F, S, has) : span_crc(pfx, F, S, has);
      // Z_p(crc_raw(H, payload)) = Z_C(Z_mis^{-1}(H)) ^ V, then Z_p undone
      const u32 Hm = inv_bits(H, half ? (code >> 12) & 15u : 0u, 4);
      const u32 X = opmul(sbase, G == 32 ? kUniSlotOpZ4096 : kSmallOpZC, Hm) ^ v;
      const u32 R = half ? inv_bits(X, code & 0xFFFu, kSmallInvOps) : (code == kCodeLong ? v : H);
      slot_store(live, oversize, m, pfx, F, S, has, R);
    } else {
      u32 r = inv_bits(v, half ? code & 0xFFFu : 0u, kSmallInvOps);
      if (code == kCodeEmpty) r = a.init;
      if (code != kCodeSkip) a.out[m] = r ^ a.final_xor;
    }
    wave_lds_sync();
  };
  auto flush = [&](u32 kf, u32 nt) __attribute__((always_inline)) { flush_any(kf, nt, false); };
  constexpr bool kSplit = SLOT && G < 32;
  // FAST waves' flush: one window (kf = 0), every code 0 (a whole aligned 4 KiB message: no
  // padding, no mis) or none -- no long messages, no inverses, no prefix reload (r05y: 0.5-0.7 us
  // per 65,536-slot list against the general flush).
  auto flush_fast = [&](u32 nt) __attribute__((always_inline)) {
    wave_lds_sync();
    const u32 hh = (u32)lane & 1u, ti = (u32)lane >> 1;
    const u64 e = lds_ld64(sring + 8u * (u32)lane);
    const u32 v = (u32)e;
    const bool live = ti < nt && (u32)(e >> 32) == 0u;
    const u64 m = 2 * (t0 + (u64)ti * nw) + hh;
    if constexpr (SLOT) {
      const uint8_t* pfx = flive ? base + fpre - a.pdelta : safe;
      // Z_0(crc_raw(H, payload)) = Z_4096(H) ^ V (mis = 0, p = 0)
      const u32 R = opmul(sbase, kUniSlotOpZ4096, eH) ^ v;
      slot_store(live, false, m, pfx, eF, eS, ehas, R);
    } else {
      if (live) a.out[m] = v ^ a.final_xor;
    }
  };
  constexpr u32 kWinMask = W - 1u;

  // Prologue: table loads, the window's records (and SLOT its prefix offsets); the LDS fill while
  // the records are in flight; then the first window's prefix words and tile 0's lines, the
  // barrier (tile 0's latency hides behind it), and the span terms hashed under tile 0's flight.
  // (SUBSPACE_SMALL_EARLY_TILE0, an A/B build: the records first and the fill after tile 0's
  // issue -- measured slower on config S's list, 61.7 vs 63.0 %, r06i.)
  if constexpr (!SUBSPACE_SMALL_EARLY_TILE0) fill.load(gtab, gops);
  if constexpr (G == 32) {
    record(fmc, wS, wL);
  }
  if constexpr (SLOT) {
    const u64* pp = a.prefixes + (flive ? fm : 0) * a.pstride;
    fpre = *pp;
    asm volatile("" ::"v"(pp));
  }
  if constexpr (SUBSPACE_SMALL_EARLY_TILE0) {
    fill.load(gtab, gops);
  } else {
    fill.store(sbase);
  }
  if constexpr (SLOT && G < 32) {  // Z_C into its LDS slot
    if (threadIdx.x < 128u)
      lds_st(sbase + kLdsOps + 512u * (u32)kSmallOpZC + 4u * threadIdx.x,
             gops[128 * (kSmallOpZC + __builtin_ctz((u32)G)) + threadIdx.x]);
  }
  if (SLOT && threadIdx.x == 0) lds_st64(smism, 0ull);
  // FAST (wave-uniform): the window is every tile of the wave (at most 32: small_run's grid) and
  // each of its messages is a whole 4 KiB payload on a 16-B boundary (SLOT: within max_len) --
  // the fixed-size channel drain. Its loop is the uniform kernel's: the next tile's address from
  // the window's records before the wait, one address and 8 loads at immediate offsets, no
  // clamps, codes or records in the loop. (Config S's channel as a shuffled slot list: 53.0 against
  // the general loop's 60.8 us per 65,536 slots, compute only 36.5 against 45.7 us -- its address
  // and code arithmetic, 6,759 VALU instructions per wave against the uniform kernel's 4,508;
  // r05z)
  const bool conf = !flive || (wL == (u64)kSmallMaxExt && (wS & 15u) == 0 && (!SLOT || wL <= a.max_len));
  const bool fast = G == 32 && nk <= kSmallRingTiles && __ballot(!conf) == 0;
  const bool ua = (a.ustride & 15u) == 0 && ((uintptr_t)base & 15u) == 0;  // 16-B strides
  const bool fastu = !SLOT && a.offsets == nullptr && a.ulen != 0 && a.ulen + (ua ? 0u : 15u) <= (u64)C;
  bool repack = false;
  u32 rcode0 = 0;  // (REPACK) this lane's entry's code when it has no lanes, written after tile 0's loads
  // REPACK2 (slot kernel, G = 32; grid-uniform: the host gives no slot wave more than
  // kRp2MaxTilesPerWave tiles, i.e. 32 messages). Lane i of each wave classifies message i of its
  // window: a code, its extended bytes E and its lines ceil(E / 128), laid out back to back in
  // lane order (r2x: the lines before it). The wave's first 64 lines are its local tile, mapped
  // and loaded before the barrier (its latency hides behind the LDS fill, as the FAST loop's tile
  // 0 does); the wave's line total and its vote (not FAST) go to LDS for the workgroup's shared
  // stream of the remaining lines.
  const bool wg2 = SLOT && G == 32 && ntiles <= (u64)kRp2MaxTilesPerWave * nw;
  u32 r2n = 0, r2x = 0, r2E = 0, r2code = 0;  // lines, lines of the wave's earlier entries, E, code
  // the entries with lines by rank (lane order) -> their lanes (ds_permute: rank k's lane to lane k)
  u32 r2l = 0;
  bool runi = false;  // the wave's entries with lines are lanes 0, 1, ... and have one line count
  auto rank_lanes = [&]() __attribute__((always_inline)) {
    const bool wl = r2n != 0u;
    const u64 mwl = __ballot(wl);
    const u32 rk = (u32)__builtin_popcountll(mwl & ((1ull << lane) - 1ull));
    r2l = (u32)__builtin_amdgcn_ds_permute((int)((wl ? rk : 32u + ((u32)lane & 31u)) << 2), lane);
    const u32 n0 = (u32)__builtin_amdgcn_readfirstlane((int)r2n);
    runi = (mwl & (mwl + 1ull)) == 0ull && __ballot(wl && r2n != n0) == 0ull;
  };
  // Local tile j of the wave (lines 64 j .. 64 j + 63 of its own stream, those below nloc), this
  // lane: its entry's lane, line in the entry, E (0: none), first byte, and the lane where the
  // entry's part in this tile starts. The entry is the one of rank k - 1, k = the entries with
  // lines starting before the tile + the tile's start marks up to this lane (an LDS word per
  // wave); one line count throughout (a fixed-size channel): rank = line / n.
  auto local_map = [&](u32 j, u32 nloc, u32& src, u64& s_, u32& E_, u32& li_, u32& st_) __attribute__((always_inline)) {
    const u32 P = 64u * j + (u32)lane;
    u32 k, x;
    if (runi) {  // entry = line / n, its first line = entry * n (no rank map, no marks)
      const u32 n0 = (u32)__builtin_amdgcn_readfirstlane((int)r2n);
      const u32 e0 = n0 ? P / n0 : 0u;
      src = e0 < 31u ? e0 : 31u;
      k = n0 ? 1u : 0u;
      x = src * n0;
    } else {
      const u32 slm = sbase + kRp2Misc + 112u + 8u * wid;
      const bool mk = r2n != 0u && (r2x >> 6) == j;
      if (lane == 0) lds_st64(slm, 0ull);
      if (mk)
        __hip_atomic_fetch_or(reinterpret_cast<lds_u64_t*>((uintptr_t)slm), 1ull << (r2x & 63u), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_WORKGROUP);
      const u64 Sl = lds_ld64(slm);
      k = (u32)__builtin_popcountll(__ballot(r2n != 0u && r2x < 64u * j)) +
          (u32)__builtin_popcountll(Sl & ((2ull << lane) - 1ull));
      src = bperm(k ? k - 1u : 0u, r2l) & 31u;
      x = bperm(src, r2x);
    }
    s_ = ((u64)bperm(src, (u32)(wS >> 32)) << 32) | (u64)bperm(src, (u32)wS);
    const u32 E = bperm(src, r2E);
    li_ = P - x;
    E_ = P < nloc && k ? E : 0u;
    st_ = x > 64u * j ? x - 64u * j : 0u;
  };
  // the local tile 0 (mapped, and loaded, before the barrier)
  u32 lsrc = 0, lli = 0, lE = 0, lst = 0;
  u64 ls = 0;
  // A wave's line total and its entries with lines past Q = 64 (i + 1), i = 0..15 (the workgroup
  // picks Q after the barrier), one byte each, for the others (the ballots outside the one-lane
  // branch: inside it only lane 0 would vote)
  auto r2_publish = [&](u32 incl) __attribute__((always_inline)) {
    u32 cnt[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (u32 i = 0; i < 16; i++)
      cnt[i >> 2] |= (u32)__builtin_popcountll(__ballot(r2n != 0u && r2x + r2n > 64u * (i + 1u))) << (8u * (i & 3u));
    if (lane == 63) lds_st(sbase + kRp2Misc + 4u * wid, incl);
    if (lane == 0) lds_st4(sbase + kRp2Counts + 16u * wid, u32x4{cnt[0], cnt[1], cnt[2], cnt[3]});
  };
  // a FAST wave's entries: every live one a whole aligned 4 KiB payload, 32 lines, live lanes first
  auto r2_fast = [&]() __attribute__((always_inline)) {
    r2code = flive ? 0u : kCodeSkip;
    r2E = flive ? kSmallMaxExt : 0u;
    r2n = flive ? 32u : 0u;
    r2x = 32u * (u32)__builtin_popcountll(__ballot(flive) & ((1ull << lane) - 1ull));
    r2_publish(r2x + r2n);
  };
  if constexpr (SLOT && G == 32) {
    if (wg2) {
      __builtin_amdgcn_sched_barrier(0);
      // every wave votes; a FAST wave does nothing else here (its bookkeeping only if the
      // workgroup repacks: r2_fast after the barrier), the config-S list's prologue stays short
      if (lane == 0) lds_st(sbase + kRp2Misc + 32u + 4u * wid, fast ? 0u : 1u);
      // the shared tiles' start marks and the tile ticket, zeroed before any wave sets them
      // (after the barrier; the FAST waves' rings, the only other users of this LDS, start after
      // it too and do not overlap them)
      if (threadIdx.x < 2u * kRp2MaxTiles) lds_st(sbase + kRp2Starts + 4u * threadIdx.x, 0u);
      if (threadIdx.x == 0) lds_st(sbase + kRp2Misc + 96u, 0u);
      if (!fast) {
        u32 incl;
        const u64 Ew = wL + (wS & 15u);
        r2code = !flive                 ? kCodeSkip
               : wL > a.max_len         ? kCodeOversize
               : Ew > (u64)kSmallMaxExt ? kCodeLong
               : wL == 0                ? kCodeEmpty
                                        : 0u;
        r2E = r2code ? 0u : (u32)Ew;
        r2n = (r2E + 127u) >> 7;
        incl = wave_scan(r2n, false);
        r2x = incl - r2n;
        r2_publish(incl);
        rank_lanes();
        const u32 tot = (u32)__builtin_amdgcn_readlane((int)incl, 63);
        local_map(0u, tot < 64u ? tot : 64u, lsrc, ls, lE, lli, lst);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if constexpr (G == 32 && !SLOT) {
    if (__builtin_expect(!fast && !fastu && nk <= kSmallRingTiles, 0)) {
      // (fenced off from the FAST path's prologue; measured neutral, r05bm, kept as validated)
      __builtin_amdgcn_sched_barrier(0);
      repack = true;
      const u64 Ew = wL + (wS & 15u);
      const u32 code0 = !flive                          ? kCodeSkip
                      : SLOT && wL > a.max_len          ? kCodeOversize
                      : Ew > (u64)kSmallMaxExt          ? kCodeLong
                      : wL == 0                         ? kCodeEmpty
                                                        : 0u;
      const u32 nl = ((u32)Ew + 127u) >> 7;  // (1 .. 32 when code0 == 0)
      const int cls = code0 ? -1 : (nl <= 1u ? 0 : 32 - __builtin_clz(nl - 1u));
      // the common case first: every placed entry in one class, the placed entries lanes 0 .. n-1
      const u64 mpl = __ballot(cls >= 0);
      const int c0 = mpl ? __builtin_amdgcn_readlane(cls, (int)__builtin_ctzll(mpl)) : 0;
      rident = (mpl & (mpl + 1ull)) == 0ull && __ballot(cls >= 0 && cls != c0) == 0ull;
      rmask = mpl;
      if (rident) {
        rcmax = (u32)c0;
        vT = (u32)__builtin_popcountll(mpl) << c0;
      } else {  // per class: lane positions and sorted indices; each entry's sorted index; inverse
        u32 base = 0, sorted = 0, ncls = 0;
        u64 mqs[6];
#pragma unroll
        for (int q = 5; q >= 0; q--) {
          const u64 mq = __ballot(cls == q);
          mqs[q] = mq;
          vbn = lane == q ? base | (sorted << 16) : vbn;
          base += (u32)__builtin_popcountll(mq) << q;
          sorted += (u32)__builtin_popcountll(mq);
          if (mq) {
            rcmax = ncls ? rcmax : (u32)q;
            ncls++;
          }
        }
        vT = base;
        // every entry up to the last placed one at 2^rcmax lanes (the uniform layout, no sort)
        // unless sorting saves tiles: two, or one of four or more (r05bo, r05bp: for a window of
        // one or two tiles the sort's prologue costs more than the tile it saves)
        const u32 nu = (u32)(64 - __builtin_clzll(mpl)) << rcmax;
        const u32 tu = (nu + 63u) >> 6, ts = (vT + 63u) >> 6;
        if (!(ts < tu && (tu >= 4u || ts + 2u <= tu))) {
          rident = true;
          vT = nu;
        } else {
          const u64 below = (1ull << lane) - 1ull;
          u32 pos = sorted + (u32)__builtin_popcountll(~mpl & below);
#pragma unroll
          for (int q = 5; q >= 0; q--)
            if (cls == q) pos = ((u32)__builtin_amdgcn_readlane((int)vbn, q) >> 16) + (u32)__builtin_popcountll(mqs[q] & below);
          vS = (u32)__builtin_amdgcn_ds_permute((int)(pos << 2), lane);
        }
      }
      rnt = (vT + 63u) >> 6;
      rcode0 = cls < 0 ? code0 : 0u;
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#ifndef SUBSPACE_PROBE_PREBAR
  if constexpr (probe) pt[1] = __builtin_amdgcn_s_memrealtime();
#endif
  u64 sA, LA, sB, LB;
  if constexpr (G == 32) {
    win_rec(0, sA, LA);
    win_rec(1, sB, LB);
  } else {
    fetch(0, sA, LA);
    fetch(1, sB, LB);
  }
  u32 pwords[14];
  if constexpr (SLOT) {
    if (SUBSPACE_SMALL_VARIANT != 1) span_load(flive ? base + fpre - a.pdelta : safe, pwords);
    __builtin_amdgcn_sched_barrier(0);
  }
  u32x4 A[8], B[8];
  u64 sc = sA, Lc = LA;
  u32 pc = 0;  // (REPACK: packed tile 0's map)
  if (repack) {
    pc = rp_map(0u);
    rp_rec(pc, sc, Lc);
    load_lines_at(A, sc, rp_ext(sc, Lc, pc), (pc >> 8) & 31u);
    if (rcode0) lds_st64(sring + 8u * (u32)lane, (u64)rcode0 << 32);
  } else {
    // REPACK2: the wave's local tile; else tile 0 (FAST: the same addresses as load_at's). (One
    // load site with selected arguments measured slower on config S's list: 54.8 against 53.3 us
    // per call, r06n)
    if (wg2 && !fast) {
#ifdef SUBSPACE_RP2_DEBUG
      rp2_check("local", ls, lE, lli, 32u * wid + lsrc);
#endif
      load_lines_at(A, ls, lE, lli);
    } else {
      load_lines(A, sc, ext(0, sc, Lc));
    }
  }
  if constexpr (SUBSPACE_SMALL_EARLY_TILE0) fill.store(sbase);
#ifdef SUBSPACE_PROBE_PREBAR  // (A/B timelines: stamp 1 = the wave reaches the barrier)
  if constexpr (probe) pt[1] = __builtin_amdgcn_s_memrealtime();
#endif
  __syncthreads();
  // (nothing hoisted above the barrier: hipcc otherwise moved the span hash's first step there,
  // with a wait for tile 0's lines, so every wave of the workgroup waited for the slowest
  // wave's tile 0 -- ~1 us per slot-list call, r05bm)
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (probe) pt[2] = __builtin_amdgcn_s_memrealtime();
  if constexpr (SLOT && SUBSPACE_SMALL_VARIANT != 1) eH = span_hash(flive ? base + fpre - a.pdelta : safe, pwords, eF, eS, ehas);
  if (fastu && !ua) useed = inv_bits(a.init, (u32)lane & 15u, 4);  // the 16 head seeds, one per lane

  // REPACK2 after the barrier: a workgroup whose waves are not all FAST packs its messages as one
  // stream of 128-B lines (message after message, every wave's entries in order; a message's
  // lines may straddle two packed tiles) and its 8 waves take the packed tiles from an LDS
  // ticket, so the work of a workgroup is shared whatever its messages' sizes and whichever wave
  // of a SIMD pair the hardware favours (round 5's per-wave repack: waves' loops ended 24 to 45
  // us into a 48 us mixed-size drain, tools/small_timeline.py). Each lane of a packed tile holds
  // line li of a message of n = ceil(E / 128) lines and applies Z_{128 (n-1-li)} to its line CRC;
  // an inclusive XOR scan over the tile and the scan value before the message's first lane in
  // the tile give the message's part in this tile, which the part's last lane XORs into the
  // message's LDS ring entry (two parts when the message straddles tiles). The entry then holds
  // V = Z_p(crc_raw(init, D)) with p = 128 n - E < 128, one padding for 7 bits at most.
  bool rp2 = false, allv = false;  // (allv: every wave voted, none is FAST)
  u32 r2tiles = 0;  // (PROBE) packed tiles this wave computed
  if constexpr (SLOT && G == 32) {
    if (wg2) {
      const u32x4 va = lds_ld4(sbase + kRp2Misc + 32u), vb = lds_ld4(sbase + kRp2Misc + 48u);
      rp2 = rfl(va.x | va.y | va.z | va.w | vb.x | vb.y | vb.z | vb.w) != 0u;
      allv = rfl((u32)(va.x && va.y && va.z && va.w && vb.x && vb.y && vb.z && vb.w)) != 0u;
    }
  }
  // PROBE: tile 0 landed (the first wait of whichever loop form runs; stamped once)
  auto stamp_tile0 = [&]() __attribute__((always_inline)) {
    if constexpr (probe)
      if (pt[3] == 0) pt[3] = __builtin_amdgcn_s_memrealtime();
  };
  u32 k = 0;
  if (rp2) {
    if constexpr (SLOT && G == 32) {
      auto process2 = [&](const u32x4 (&cur)[8], u64 ms, u32 mE, u32 mli, u32 me, u32 mst)
                          __attribute__((always_inline)) {
        const u32 mis = (u32)ms & 15u;
        u32x4 d[8];
#pragma unroll
        for (int b = 0; b < 8; b++) d[b] = cur[b];
        const bool head = mE != 0u && mis != 0u && mli == 0u;
        const int v0 = (int)mE - 128 * (int)mli;
        const u32 hi = v0 <= 0 ? 0u : (v0 >= 128 ? 128u : (u32)v0);
        if (__any(head || hi < 128u)) keep_sel(d, head ? mis : 0u, hi);
        u32 seed = a.init;
        if (seed != 0u && __any(head)) seed = inv_bits(seed, mis, 4);
        const u32 crc = line_crc32_2chain(d, mli == 0u ? seed : 0u, lc0, lc1, z64);
        const u32 n = (mE + 127u) >> 7;
        u32 v = lane_shift(sbase + kLdsOps + 4u * ((n - 1u - mli) & 31u), crc);
        v = mE ? v : 0u;
        const u32 P = wave_scan(v, true);
        const u32 pv = bperm(mst ? mst - 1u : 0u, P);
        const u32 seg = P ^ (mst ? pv : 0u);
        if (mE != 0u && (mli == n - 1u || lane == 63))
          __hip_atomic_fetch_xor(reinterpret_cast<lds_u32_t*>((uintptr_t)(sbase + kRp2Ring + 8u * me)), seg,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      };
      // the FAST waves' bookkeeping, now that the workgroup repacks; every wave's ring entries
      // (codes, values 0) and its local tile 0 (loaded before the barrier; a FAST wave's is its
      // FAST tile 0, mapped here; Q >= 64, so the tile does not depend on Q)
      if (fast) {
        r2_fast();
        rank_lanes();
      }
      const u32 tot0 = (u32)__builtin_amdgcn_readlane((int)(r2x + r2n), 63);  // the wave's lines
      if (fast) local_map(0u, tot0 < 64u ? tot0 : 64u, lsrc, ls, lE, lli, lst);
      if (lane < 32) {
        const u32 code = r2code ? r2code : ((128u * r2n - r2E) | (((u32)wS & 15u) << 12) | (r2n << 16));
        lds_st64(sbase + kRp2Ring + 8u * (32u * wid + (u32)lane), (u64)code << 32);
      }
      // Q: every wave computes its first Q lines itself (local tiles), Q = the workgroup's least
      // wave rounded down to whole tiles, at least one tile (or its largest wave rounded up, when
      // that is at most one tile more); the rest of every wave's lines form the shared stream,
      // wave after wave. Known now when every wave voted (their totals and
      // counts went to LDS before the prologue barrier); else after the FAST waves' bookkeeping
      // barrier below.
      u32 tw[8], Q = 64u;
      auto read_q = [&]() __attribute__((always_inline)) {
        const u32x4 ta = lds_ld4(sbase + kRp2Misc), tb = lds_ld4(sbase + kRp2Misc + 16u);
        tw[0] = rfl(ta.x), tw[1] = rfl(ta.y), tw[2] = rfl(ta.z), tw[3] = rfl(ta.w);
        tw[4] = rfl(tb.x), tw[5] = rfl(tb.y), tw[6] = rfl(tb.z), tw[7] = rfl(tb.w);
        u32 tmin = tw[0], tmax = tw[0];
#pragma unroll
        for (u32 w = 1; w < 8; w++) {
          tmin = tw[w] < tmin ? tw[w] : tmin;
          tmax = tw[w] > tmax ? tw[w] : tmax;
        }
        Q = tmin >= 128u ? tmin & ~63u : 64u;
        // no shared stream when no wave has more than one tile beyond Q: its tables, barrier and
        // a shared tile's round trip after them cost more than one wave's extra local tile
        const u32 tm = (tmax + 63u) & ~63u;
        if (tm <= Q + 64u) Q = tm > 64u ? tm : 64u;
      };
      if (allv) read_q();
      // local tile 1 (the wave's lines 64 .. 127): its loads go out before tile 0's compute, as the
      // loop's next tile does -- known local when every wave voted (Q >= 128), else on speculation
      // for a wave with more than one tile of lines (local iff Q >= 128, known after the barrier)
      bool use1 = tot0 > 64u && (!allv || Q >= 128u);
      u32 s1src = 0, E1 = 0, li1 = 0, st1 = 0;
      u64 s1 = 0;
      if (use1) {
        local_map(1u, tot0 < 128u ? tot0 : 128u, s1src, s1, E1, li1, st1);
#ifdef SUBSPACE_RP2_DEBUG
        rp2_check("local1", s1, E1, li1, 32u * wid + s1src);
#endif
      }
      issue_prio_hi();
      drain_before_issue();
      stamp_tile0();
      if (use1) load_lines_at(B, s1, E1, li1);
      issue_prio_lo();
      process2(A, ls, lE, lli, 32u * wid + lsrc, lst);
      r2tiles++;
      if (!allv) {
        __syncthreads();  // the FAST waves' totals and counts
        read_q();
        use1 = use1 && Q >= 128u;
      }
      // An entry's shared part (its lines from local position Q on) gets a rank among the entries
      // with one, its record, its first shared position and the line it starts with; the shared
      // tiles' start marks and first entries (by rank).
      const u32 qi = (Q >> 6) - 1u;  // (<= 15: a wave has at most 32 x 32 lines)
      u32 wbase = 0, T = 0, rbase = 0, NR = 0;
#pragma unroll
      for (u32 w = 0; w < 8; w++) {
        const u32 sh = tw[w] > Q ? tw[w] - Q : 0u;
        const u32 cw = (lds_ld(sbase + kRp2Counts + 16u * w + (qi & ~3u)) >> (8u * (qi & 3u))) & 0xFFu;
        wbase += w < wid ? sh : 0u;
        T += sh;
        rbase += w < wid ? cw : 0u;
        NR += cw;
      }
      const u32 a0 = r2x > Q ? r2x : Q;  // the entry's first local position in the shared stream
      const u32 shn = r2x + r2n > Q ? r2x + r2n - a0 : 0u;
      const u32 start = wbase + a0 - Q;
      const u32 r = rbase + (u32)__builtin_popcountll(__ballot(shn != 0u) & ((1ull << lane) - 1ull));
      if (lane < 32) {
        const u32 q = 32u * wid + (u32)lane;
        if (shn) {
          lds_st64(sbase + kRp2EntS + 8u * r, wS | ((u64)q << 56));
          lds_st(sbase + kRp2EntM + 4u * r, r2E | (start << 13) | ((a0 - r2x) << 26));
          __hip_atomic_fetch_or(reinterpret_cast<lds_u64_t*>((uintptr_t)(sbase + kRp2Starts + 8u * (start >> 6))),
                                1ull << (start & 63u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const u32 jb = (start + 63u) >> 6;  // the shared tile whose line 0 is in this part, if any
          if (64u * jb < start + shn) lds_st(sbase + kRp2First + 4u * jb, r);
        }
      }
      const u32 tot = tw[wid];
      const u32 nloc = tot < Q ? tot : Q, nlt = (nloc + 63u) >> 6;  // local lines, tiles
      const u32 ntl = (T + 63u) >> 6;  // shared tiles of the workgroup
      if (ntl) __syncthreads();       // the shared tables
      const u32 tick = sbase + kRp2Misc + 96u;
      // the wave's next tile: its local tiles 1 .. nlt - 1, then shared tiles from the ticket; v
      // false: none left (E 0: the loads read the step table)
      u32 jl = use1 ? 2u : 1u;  // (use1: B holds local tile 1)
      auto next = [&](bool& v, u64& ms, u32& mE, u32& mli, u32& me, u32& mst) __attribute__((always_inline)) {
        if (jl < nlt) {
          u32 src;
          local_map(jl, nloc, src, ms, mE, mli, mst);
          me = 32u * wid + src;
#ifdef SUBSPACE_RP2_DEBUG
          rp2_check("local", ms, mE, mli, me);
#endif
          jl++;
          v = true;
          return;
        }
        u32 j = ntl;
        if (ntl) {
          u32 t = 0;
          if (lane == 0)
            t = __hip_atomic_fetch_add(reinterpret_cast<lds_u32_t*>((uintptr_t)tick), 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
          j = (u32)__builtin_amdgcn_readlane((int)t, 0);
        }
        v = j < ntl;
        if (!v) {  // (wave-uniform: none left -- no table reads; the caller loads nothing)
          ms = 0;
          mE = mli = me = mst = 0u;
          return;
        }
        // shared tile j, this lane: its entry's record and ring entry, its line, the entry's E,
        // and the lane where the entry's part in this tile starts
        const u32 jj = j;
        const u64 Sj = lds_ld64(sbase + kRp2Starts + 8u * jj);
        const u32 fe = lds_ld(sbase + kRp2First + 4u * jj);
        u32 e = fe + (u32)__builtin_popcountll(Sj & ((2ull << lane) - 1ull)) - (u32)(Sj & 1ull);
        e = e < NR ? e : (NR ? NR - 1u : 0u);
        const u32 m = lds_ld(sbase + kRp2EntM + 4u * e);
        const u64 sq = lds_ld64(sbase + kRp2EntS + 8u * e);
        ms = sq & ((1ull << 56) - 1ull);
        const u32 P = 64u * jj + (u32)lane, st = (m >> 13) & 0x1FFFu;
        const bool live = v && P < T;
        mE = live ? (m & 0x1FFFu) : 0u;
        mli = live ? P - st + (m >> 26) : 0u;
        me = (u32)(sq >> 56);
        mst = st > 64u * jj ? st - 64u * jj : 0u;
#ifdef SUBSPACE_RP2_DEBUG
        rp2_check("shared", ms, mE, mli, me);
#endif
      };
      bool va = false, vb = use1;
      u64 s_a = 0, s_b = s1;
      u32 E_a = 0, li_a = 0, e_a = 0, st_a = 0, E_b = E1, li_b = li1, e_b = 32u * wid + s1src, st_b = st1;
      if (!use1) {  // (B's lines, if loaded, are the shared stream's: dropped)
        next(va, s_a, E_a, li_a, e_a, st_a);
        if (va) load_lines_at(A, s_a, E_a, li_a);
      }
      // the ping-pong (entered at its second half when B holds local tile 1); a wave's last tile
      // is computed after the loop with no load in flight (loading an empty tile instead put an
      // L2 round trip in front of every wave's flush)
      bool inB = use1, last = false, lastA = false;
      for (;;) {
        if (!inB) {
          if (!va) break;
          next(vb, s_b, E_b, li_b, e_b, st_b);
          issue_prio_hi();
          drain_before_issue();
          if (!vb) {
            last = lastA = true;
            break;
          }
          load_lines_at(B, s_b, E_b, li_b);
          issue_prio_lo();
          process2(A, s_a, E_a, li_a, e_a, st_a);
          r2tiles++;
        }
        inB = false;
        next(va, s_a, E_a, li_a, e_a, st_a);
        issue_prio_hi();
        drain_before_issue();
        if (!va) {
          last = true;
          break;
        }
        load_lines_at(A, s_a, E_a, li_a);
        issue_prio_lo();
        process2(B, s_b, E_b, li_b, e_b, st_b);
        r2tiles++;
      }
      issue_prio_lo();
      if (last) {
        u32x4 L[8];
#pragma unroll
        for (int b = 0; b < 8; b++) L[b] = lastA ? A[b] : B[b];
        process2(L, lastA ? s_a : s_b, lastA ? E_a : E_b, lastA ? li_a : li_b, lastA ? e_a : e_b,
                 lastA ? st_a : st_b);
        r2tiles++;
      }
      drain_before_issue();
      if constexpr (probe) pt[4] = __builtin_amdgcn_s_memrealtime();
      // every part is in the ring (without a shared stream every entry is its own wave's alone)
      if (ntl)
        __syncthreads();
      else
        wave_lds_sync();
      // the flush: lane i finishes message i of the wave's window (entry 32 wid + i), as flush_any
      // with p < 128 and Z_{128 n} for the entry's n lines
      {
        const u64 ev = lds_ld64(sbase + kRp2Ring + 8u * (32u * wid + ((u32)lane & 31u)));
        u32 v = (u32)ev;
        const u32 code = lane < 32 ? (u32)(ev >> 32) : kCodeSkip;
        u64 msk = __ballot(code == kCodeLong);
        while (msk) {  // rare: messages longer than 4 KiB, one at a time by the whole wave
          const u32 src = (u32)__builtin_ctzll(msk);
          msk &= msk - 1;
          const u64 mm = 2u * (t0 + (u64)(src >> 1) * nw) + (src & 1u);
          u64 ls, lL;
          record(mm, ls, lL);
          const u32 r = long_crc(ls, lL, a.prefixes[mm * a.pstride]);
          v = lane == (int)src ? r : v;
        }
        const bool half = code < kCodeOversize, oversize = code == kCodeOversize;
        const bool live = code != kCodeSkip && !oversize;
        const u32 n = (code >> 16) & 63u;
        const u32 Hm = inv_bits(eH, half ? (code >> 12) & 15u : 0u, 4);
        u32 Z = 0;
        if (__any(half && n == 32u)) Z = opmul(sbase, kUniSlotOpZ4096, Hm);
        if (__any(half && n < 32u)) {
          const u32 Zs = lane_shift(sbase + kLdsOps + 4u * (n & 31u), Hm);
          Z = n == 32u ? Z : Zs;
        }
        // Z_p(crc_raw(H, payload)) = Z_{128 n}(Z_mis^{-1}(H)) ^ V, then Z_p undone (p < 128)
        const u32 R = half ? inv_bits(Z ^ v, code & 0x7Fu, 7) : (code == kCodeLong ? v : eH);
        slot_store(live, oversize, fm, flive ? base + fpre - a.pdelta : safe, eF, eS, ehas, R);
      }
      if constexpr (probe) pt[5] = __builtin_amdgcn_s_memrealtime();
    }
  } else if (fast) {
    // ping-pong, unrolled by two, one tile in flight (crc_uniform.hip's loop)
    for (; k + 1 < nk; k += 2) {
      const u64 qB = fast_off(k + 1);
      issue_prio_hi();
      drain_before_issue();  // tile k's lines
      stamp_tile0();
      load_at(B, qB);
      issue_prio_lo();
      process_fast(A, k);
      const u64 qA = fast_off(k + 2);
      issue_prio_hi();
      drain_before_issue();
      stamp_tile0();
      load_at(A, qA);
      issue_prio_lo();
      process_fast(B, k + 1);
    }
    if (k < nk) {
      drain_before_issue();
      stamp_tile0();
      process_fast(A, k);
    }
  } else if (repack) {
    // the general loop's ping-pong over the wave's rnt packed tiles
    u32 j = 0;
    for (; j + 1 < rnt; j += 2) {
      const u32 p1 = rp_map(j + 1);
      u64 s1, L1;
      rp_rec(p1, s1, L1);
      issue_prio_hi();
      drain_before_issue();  // tile j's lines
      stamp_tile0();
      load_lines_at(B, s1, rp_ext(s1, L1, p1), (p1 >> 8) & 31u);
      issue_prio_lo();
      process_rp(A, sc, Lc, pc);
      const u32 p2 = rp_map(j + 2);
      u64 s2, L2;
      rp_rec(p2, s2, L2);
      issue_prio_hi();
      drain_before_issue();
      stamp_tile0();
      load_lines_at(A, s2, rp_ext(s2, L2, p2), (p2 >> 8) & 31u);
      issue_prio_lo();
      process_rp(B, s1, L1, p1);
      sc = s2;
      Lc = L2;
      pc = p2;
    }
    if (j < rnt) {
      drain_before_issue();
      stamp_tile0();
      process_rp(A, sc, Lc, pc);
    }
  } else if (fastu && ua) {
    // the general loop's schedule (windows of W tiles) with the FAST loop's loads and compute
    for (; k + 1 < nk; k += 2) {
      const u64 qB = u_off(k + 1);
      issue_prio_hi();
      drain_before_issue();  // tile k's lines
      stamp_tile0();
      u_load(B, k + 1, qB);
      issue_prio_lo();
      if (k && (k & kWinMask) == 0u) flush_u(k - W, W);
      process_u(A, k);
      const u64 qA = u_off(k + 2);
      issue_prio_hi();
      drain_before_issue();
      stamp_tile0();
      u_load(A, k + 2, qA);
      issue_prio_lo();
      if constexpr (W == 1) flush_u(k, 1u);
      process_u(B, k + 1);
    }
    if (k < nk) {
      drain_before_issue();
      stamp_tile0();
      if (k && (k & kWinMask) == 0u) flush_u(k - W, W);
      process_u(A, k);
    }
  } else if (fastu && !ua) {
    // (packed strides: the same schedule)
    for (; k + 1 < nk; k += 2) {
      const u64 qB = u_off_p(k + 1);
      issue_prio_hi();
      drain_before_issue();  // tile k's lines
      stamp_tile0();
      u_load_p(B, k + 1, qB);
      issue_prio_lo();
      if (k && (k & kWinMask) == 0u) flush_up(k - W, W);
      process_up(A, k);
      const u64 qA = u_off_p(k + 2);
      issue_prio_hi();
      drain_before_issue();
      stamp_tile0();
      u_load_p(A, k + 2, qA);
      issue_prio_lo();
      if constexpr (W == 1) flush_up(k, 1u);
      process_up(B, k + 1);
    }
    if (k < nk) {
      drain_before_issue();
      stamp_tile0();
      if (k && (k & kWinMask) == 0u) flush_up(k - W, W);
      process_up(A, k);
    }
  } else {
    // Ping-pong line buffers, loop unrolled by two, records one tile ahead of the lines; the
    // ring is finished whenever it holds W tiles (64 messages), right after the next tile's
    // loads are issued (so the stores retire during that tile's compute), and at the end
    // (crc_ragged.hip's loop, without descriptors). Nothing else lives across the loop
    // (register-parked values, 64-tile windows and a flush only after the loop
    // each measured slower).
    for (; k + 1 < nk; k += 2) {
      issue_prio_hi();       // (crc_device.h)
      drain_before_issue();  // tile k's lines and tile k+1's record
      stamp_tile0();
      const bool wb = k && (k & kWinMask) == 0u;
      if constexpr (kSplit) {
        if (wb) flush_issue(k - W);
      }
      const u64 s1 = sB, L1 = LB;
      fetch(k + 2, sA, LA);
      load_lines(B, s1, ext(k + 1, s1, L1));
      issue_prio_lo();
      if (wb) flush_any(k - W, W, kSplit);
      process(A, sc, Lc, k);
      issue_prio_hi();
      drain_before_issue();
      stamp_tile0();
      if constexpr (kSplit && W == 1) flush_issue(k);
      const u64 s2 = sA, L2 = LA;
      fetch(k + 3, sB, LB);
      load_lines(A, s2, ext(k + 2, s2, L2));
      issue_prio_lo();
      if constexpr (W == 1) flush_any(k, 1u, kSplit);  // (one-tile windows: tile k before tile k + 1)
      process(B, s1, L1, k + 1);
      sc = s2;
      Lc = L2;
    }
    if (k < nk) {
      drain_before_issue();
      stamp_tile0();
      if (k && (k & kWinMask) == 0u) flush(k - (kWinMask + 1u), kWinMask + 1u);
      process(A, sc, Lc, k);
    }
  }
  if constexpr (probe)
    if (!rp2) pt[4] = __builtin_amdgcn_s_memrealtime();
  if (nk && !rp2 && SUBSPACE_SMALL_VARIANT != 2) {
    if (fast) {
      flush_fast(nk);
    } else if (fastu) {
      const u32 kf = (nk - 1u) & ~kWinMask;
      if (ua)
        flush_u(kf, nk - kf);
      else
        flush_up(kf, nk - kf);
    } else {
      const u32 kf = (nk - 1u) & ~kWinMask;  // the last window, not flushed yet
      flush(kf, nk - kf);
    }
  }
  if constexpr (probe)
    if (!rp2) pt[5] = __builtin_amdgcn_s_memrealtime();
  if constexpr (SLOT) {
    if (a.error_count && lane == 0) {
      if (calc) {
        if (blockIdx.x == 0 && wid == 0) *a.error_count = 0u;  // a publish has no mismatches
      } else {
        // the workgroup's count: one 64-bit LDS atomic per wave, (1 << 40) | its count; the
        // last wave of the workgroup adds the workgroup's total to the call's counter entry
        // (crc_device.h add_call_mismatches)
        const u64 o = __hip_atomic_fetch_add(reinterpret_cast<lds_u64_t*>((uintptr_t)smism), (1ull << 40) | mism,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if ((u32)(o >> 40) == (u32)NPW - 1u)
          add_call_mismatches(a.counter, (u32)((o & ((1ull << 40) - 1)) + mism), a.error_count);
      }
    }
  } else {
    // a word the caller's next kernel accumulates into (a slot batch's mismatch count)
    if (a.zero_word != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *a.zero_word = 0u;
  }
  if constexpr (probe) {
    pt[6] = __builtin_amdgcn_s_memrealtime();
    u64* r = a.probe + ((u64)blockIdx.x * NPW + wid) * kProbeWords;
    const u64 xcc = (u64)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    const u64 v = lane == 0 ? pt[0] : lane == 1 ? pt[1] : lane == 2 ? pt[2] : lane == 3 ? pt[3]
                : lane == 4 ? pt[4] : lane == 5 ? pt[5] : lane == 6 ? pt[6]
                : (xcc | ((u64)nk << 32) | ((u64)(fast && !rp2) << 48) | ((u64)(repack || rp2) << 49) |
                   ((u64)(rp2 ? r2tiles : rnt) << 52));
    if (lane < kProbeWords) r[lane] = v;
  }
}

// The product instantiations (devtools.hip includes this file for its PROBE instantiation
// only: libsubspace_crc_dev.so)
#ifndef SUBSPACE_DEV_TU
#define SUBSPACE_SMALL_INST(G)                                                                          \
  template __global__ void crc32_small_kernel<512, false, false, G>(const u32*, const u32*, SmallArgs); \
  template __global__ void crc32_small_kernel<512, true, false, G>(const u32*, const u32*, SmallArgs);
SUBSPACE_SMALL_INST(1)
SUBSPACE_SMALL_INST(2)
SUBSPACE_SMALL_INST(4)
SUBSPACE_SMALL_INST(8)
SUBSPACE_SMALL_INST(16)
SUBSPACE_SMALL_INST(32)
#undef SUBSPACE_SMALL_INST
#endif

}  // namespace subspace_amd
