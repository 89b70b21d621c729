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
//    ds_read_b32 + 4 v_perm + 2 v_bitop3 per word), as two 16-step chains (bytes 0..63,
//    64..127) joined by a 4x-replicated Z_64 nibble table (crc_device.h line_crc32_2chain).
//  * Combine, per tile: lane l of half h holds line l's CRC; the message CRC is
//      crc(msg) = XOR_l Z_{128*(31-l)}(line_l)      (crc_raw linearity)
//    Each lane applies its own operator Z_{128*(31-l)} from nibble tables laid out
//    [nibble k][value n][lane slot], so the 32 lanes of a half read 32 different banks
//    (conflict-free, 8 ds_read_b32, one LDS round trip), and the XOR over the half is a
//    DPP reduction (row_shr 1/2/4/8 + row_bcast15: VALU only). Lanes 31 and 63 end with
//    the two messages' CRCs.
//  * Results go to a per-wave LDS ring and are stored to HBM only when the ring is full
//    (every 128 tiles) and at the end. vmcnt counts stores with the loads, in order, so
//    a store in the stream makes the wait for the next tile's loads wait for the store's
//    write-back too: a store every 4 tiles cost ~10 % of a streaming kernel's rate
//    (tools/ubench/streamread.hip lines_store: 6.0 vs 6.6 TB/s).
//  * SLOT = true: the message-slot checksums of a contiguous channel layout
//    (subspace_crc32_slots_strided, metadata_size 0) in the same pass, no second kernel.
//    Message i's payload is at base + i*stride, its MessagePrefix prefix_size bytes before.
//    The checksum (client/checksum.h:29-37 over common/channel.h:527-542's spans) is
//      ~crc_raw(~0, span0 || payload) = ~( Z_4096(crc_raw(~0, span0)) ^ crc_raw(0, payload) )
//    with span0 = prefix[4, 48). The payload term is the message CRC from init 0. The waves
//    run exactly the plain kernel's stream -- no prefix load, slot store or slot register in
//    the tile loop -- and leave each message CRC in an LDS ring, tagged with its tile index.
//    Every workgroup is one ring window (<= kSlotRingRounds tiles per wave; the host launches
//    more workgroups for longer channels). After its tiles, each of waves 0-3 -- the older
//    wave of each SIMD pair, which runs ~1.3 us ahead of its partner (profiles/DESIGN_r01-r03.md 4.4) --
//    finishes a quarter of the workgroup's messages: it loads their prefix lines (one per
//    lane), computes crc_raw(~0, span0) (11 steps; for a publish with the kMessageHasChecksum
//    bit set first, as SetHasChecksum() precedes the checksum: client/publisher.cc:664-675) and
//    one Z_4096 opmul, waits for the tagged ring entries of waves 4-7, and stores flag +
//    checksum (publish) or the status (verify: client/client.cc:1346-1356; no
//    kMessageHasChecksum -> unchecked). Mismatches are summed per workgroup with one LDS
//    atomic per finishing wave and over workgroups by one 64-bit global atomic per workgroup
//    that also counts finished workgroups; the last one writes the call's total.
#include "crc_device.h"

// Timing-only investigation builds of the slot finishing (tools/ubench/build_variants.sh
// passes -DSUBSPACE_SLOT_VARIANT=n; the product build is 0): 12 no prefix stores; 13 no prefix
// loads (zeros). The other variants measured in round 3 are in profiles/DESIGN_r01-r03.md 4.4.
#ifndef SUBSPACE_SLOT_VARIANT
#define SUBSPACE_SLOT_VARIANT 0
#endif
#if SUBSPACE_SLOT_VARIANT != 0 && !defined(SUBSPACE_AB_BUILD)
#error "SUBSPACE_SLOT_VARIANT is a timing-only A/B knob (define SUBSPACE_AB_BUILD)"
#endif

namespace subspace_amd {

template <int WG, bool SLOT, bool PROBE>
__global__ __launch_bounds__(WG) void crc32_uniform4k_kernel(
    const uint8_t* __restrict__ base, u64 stride, u64 count, const u32* __restrict__ gtab,
    const u32* __restrict__ gops, u32 init, u32 final_xor, u32* __restrict__ out, int order,
    u32* __restrict__ zero_word, SlotArgs sa) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  constexpr int NPW = WG / 64;  // waves
  const u32 sbase = (u32)(uintptr_t)smem;
  u64 pt[4] = {0, 0, 0, 0};  // PROBE: timestamps, stored at exit (no store inside the stream)
  if constexpr (PROBE) pt[0] = __builtin_amdgcn_s_memrealtime();
  // Prologue: every kernel argument in one scalar round trip, then the table
  // loads first of all (they need only gtab/gops), then tile 0's loads once its address is
  // known; the LDS stores and the barrier follow, under tile 0's latency.
  asm volatile("" ::"s"(base), "s"(stride), "s"(count), "s"(init), "s"(final_xor), "s"(out), "s"(order),
               "s"(gridDim.x));
  // Two 64-B lookup chains per line, joined by Z_64 (crc_device.h line_crc32_2chain): half
  // the dependent chain per tile for 8 more conflict-free lookups per line; config B 45.36 ->
  // 45.10 us (r02c17, slot_gap interleaved) and 45.4-45.8 -> 45.0-45.4 us (r02c18, sweep A/B,
  // four pairs); bit-exact.
  constexpr bool kTwoChain = true;  // (false: the one-chain line CRC, for A/B builds)
  // step tables, per-lane operators, Z_4096 and Z_64 (the two-chain line CRC's join)
  LdsFill<WG, kTwoChain ? kUniOpSlots : kUniOpSlotsOneChain> fill;
  fill.load(gtab, gops);

  const int lane = threadIdx.x & 63;
  // wave-uniform (SGPR) wave index: keeps the tile loop a scalar loop, so hipcc's waitcnt
  // bookkeeping stays exact (a divergent loop makes it drain the prefetch every iteration)
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u32 lc0 = sbase + ((u32)(lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  constexpr int kRing = uni_ring_results(NPW);
  const u32 ring = sbase + kUniRing + (u32)wid * (4u * kRing);
  // SLOT: this wave's tagged result ring; the workgroup's mismatch word
  const u32 sring = sbase + kUniSlotRing + (u32)wid * kSlotRingBytesPerWave;
  const u32 smism = sbase + uniform_slot_mism_word(NPW);
  const u32 lop = sbase + kLdsOps + 4u * (u32)(31 - (lane & 31));  // this lane's operator slot
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
  // (The slot finishing replays order 0's mapping: the host launches SLOT with order 0.)
  constexpr u64 wpb = NPW;
  const u64 nw = (u64)gridDim.x * wpb;
  u64 t0, tstep, tend;
  // order 3 needs whole XCD groups: 8 | G and 16 | (G/8)*wpb; otherwise it is order 0
  if (order == 3 && ((gridDim.x & 7u) || ((((u64)gridDim.x >> 3) * wpb) & 15u))) order = 0;
  if (SLOT || order == 0) {
    t0 = front_slot(blockIdx.x, gridDim.x, (u32)wid);
    tstep = nw;
    tend = ntiles;
  } else if (order == 3) {
    // Sweep in XCD groups: each aligned group of 16 front slots (16 tiles = 32 messages =
    // one 128-B line of results) lands on one XCD (two workgroups b, b+8), groups rotating
    // over the 8 XCDs, so every output line is written from a single L2.
    const u32 x = blockIdx.x & 7u, local = (blockIdx.x >> 3) * (u32)wpb + (u32)wid;
    t0 = ((u64)(local >> 4) * 8u + x) * 16u + (local & 15u);
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
  // (32-bit division: every tile count here is < 2^32, as count < 2^33 messages)
  const u32 nk = t0 < tend ? ((u32)(tend - t0) + (u32)tstep - 1u) / (u32)tstep : 0u;
  const u32 s_init = (l == 0) ? init : 0u;

  // Tile k's lines. Past the wave's last tile it re-reads that tile, and the missing odd
  // message of the batch's last tile re-reads the even one (its CRC is never stored): every
  // lane issues every load, no divergent branch around loads (which forces vmcnt(0)).
  // Waves without tiles read message 0. (Buffer loads against a per-tile scalar resource,
  // which make all this address math scalar, measured 7-10 % slower: profiles/DESIGN_r01-r03.md 4.1.)
  auto tile_off = [&](u32 k) {  // byte offset of this lane's line of tile k from base
    const u32 kk = k < nk ? k : (nk ? nk - 1 : 0u);
    u64 msg = nk ? 2 * (t0 + (u64)kk * tstep) + (u64)h : 0;
    msg = msg < count ? msg : msg - 1;
    return msg * stride + (u64)l * 128;
  };
  auto load_at = [&](u32x4 (&d)[8], u64 off) {
    const u32x4* q = reinterpret_cast<const u32x4*>(base + off);
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = q[i];
    // the address live past the last load, so that its VGPRs are never that load's destination
    // (the 768- and 1,024-thread instantiations had such a load)
    asm volatile("" ::"v"(q));
    // keep the loads at this point, in order (hipcc otherwise sinks them into the compute)
    __builtin_amdgcn_sched_barrier(0);
  };
  auto load_tile = [&](u32x4 (&d)[8], u32 k) { load_at(d, tile_off(k)); };
  // The next tile's offset, computed before the wait for the current one (pinned there), so
  // only the load instructions remain between the landing and the issue
  auto addr_before_wait = [&](u32 k) {
    u64 off = tile_off(k);
#if SUBSPACE_ADDR_EARLY
    asm volatile("" : "+v"(off));
#endif
    return off;
  };

  // CRC of this lane's line of a tile (from the batch init for line 0, else from 0).
  const u32 z64 = sbase + kLdsOps + 512u * (u32)kUniSlotOpZ64 + 4u * (u32)(lane & 3);
  auto line_crc = [&](const u32x4 (&d)[8]) {
    if constexpr (kTwoChain) return line_crc32_2chain(d, s_init, lc0, lc1, z64);
    else return line_crc32(d, s_init, lc0, lc1);
  };
  // Message CRCs of tile k: into ring slots 2*(k - kf) + h (kf = first tile of the window);
  // SLOT: into the tagged ring entry 2*k + h (k < kSlotRingRounds), as CRC | k << 32.
  auto tile_result = [&](u32 crc, u32 k, u32 kf) {
    u32 v = lane_shift(lop, crc);
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    if constexpr (SLOT) {
      if (l == 31)
        lds_st64(sring + 16u * (k & (u32)(kSlotRingRounds - 1)) + 8u * (u32)h, ((u64)k << 32) | (u64)(v ^ final_xor));
    } else {
      if (l == 31) lds_st(ring + 4u * (2u * (k - kf) + (u32)h), v ^ final_xor);
    }
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
  u64 pt_args = 0;
  if constexpr (PROBE) pt_args = __builtin_amdgcn_s_memrealtime();
  u32x4 A[8], B[8];
  load_tile(A, 0);
  fill.store(sbase);
  if constexpr (SLOT) {
    // no ring entry may carry a tag before its tile is written; the mismatch word starts at 0
    constexpr u32 kEntries = (u32)NPW * kSlotRingBytesPerWave / 8u;
    for (u32 i = threadIdx.x; i < kEntries; i += WG) lds_st64(sbase + kUniSlotRing + 8u * i, ~0ull);
    if (threadIdx.x == 0) lds_st(smism, 0u);
  }
  __syncthreads();
  // Wait for tile 0 right here (the loop's first drain is then a no-op). Waves without tiles
  // run through the loop without iterations rather than returning early: the early return
  // cost 0.5 us per config-B launch (bench.py A/B, r02af), as did the waves' late start
  // when the table loads waited behind the kernel-argument math.
  u64 pt_landed = 0;
  if constexpr (PROBE) pt[1] = __builtin_amdgcn_s_memrealtime();
  drain_before_issue();
  if constexpr (PROBE) pt_landed = __builtin_amdgcn_s_memrealtime();

  // Ping-pong buffers, loop unrolled by two (no early exit: a break between the halves
  // would give the loop head a predecessor with fewer loads in flight, and hipcc's waitcnt
  // merge would drain the prefetch there); the ring is stored when full. Tile k has
  // landed before tile k+1 is issued (drain_before_issue): each wave keeps at most one
  // tile in flight, which HBM serves faster than two (45.5 vs 47.3 us per 256 MiB launch,
  // profiles/r01/ceiling.md), and tile k+1's latency still hides behind tile k's compute.
  // A full ring is stored right after the next tile's loads are issued, so the stores
  // retire during that tile's compute instead of stalling the next drain (crc_long.hip).
  // SLOT: the same loop without the ring stores (a workgroup is one ring window).
  constexpr u32 kWin = SLOT ? ~0u : (u32)(kRing / 2);
  u32 k = 0, kf = 0;
  u64 pt_finish = 0;  // PROBE, SLOT: when a finishing wave began
  for (; k + 1 < nk; k += 2) {
    const u64 qB = addr_before_wait(k + 1);
    issue_prio_hi();
    drain_before_issue();
    load_at(B, qB);
    issue_prio_lo();
    if (!SLOT && k - kf == kWin) {
      wave_lds_sync();
      flush(kf, kRing / 2);
      kf = k;
    }
    tile_result(line_crc(A), k, kf);
    const u64 qA = addr_before_wait(k + 2);
    issue_prio_hi();
    drain_before_issue();
    load_at(A, qA);
    issue_prio_lo();
    tile_result(line_crc(B), k + 1, kf);
  }
  if constexpr (PROBE) pt[2] = __builtin_amdgcn_s_memrealtime();
  if (k < nk) {  // odd last tile, already loaded
    if (!SLOT && k - kf == kWin) {
      wave_lds_sync();
      flush(kf, kRing / 2);
      kf = k;
    }
    tile_result(line_crc(A), k, kf);
  }
  wave_lds_sync();
  if constexpr (SLOT) {
    if (wid < kSlotFinishers) {
      if constexpr (PROBE) pt_finish = __builtin_amdgcn_s_memrealtime();
      // Round r: message q = r * 64 * kSlotFinishers + 64 * wid + lane of the workgroup, i.e. tile
      // q >> 4 of wave (q >> 1) & 7, half q & 1 (16 tiles per round, one message per lane).
      static_assert(NPW == 8 && kSlotRingRounds == 2 * 16, "the finishing map assumes 8 waves, 2 rounds");
      const u32 fw = ((u32)lane >> 1) & 7u, fh = (u32)lane & 1u;
      const u64 ft0 = front_slot(blockIdx.x, gridDim.x, fw);
      const u32 fnk = ft0 < ntiles ? ((u32)(ntiles - ft0) + (u32)nw - 1u) / (u32)nw : 0u;
      const u64 w0 = front_slot(blockIdx.x, gridDim.x, 0u);  // wave 0 has the most tiles
      const u32 nk0 = w0 < ntiles ? ((u32)(ntiles - w0) + (u32)nw - 1u) / (u32)nw : 0u;
      const bool calc = sa.mode == 0u;
      auto ftile = [&](u32 r) { return 16u * r + 4u * (u32)wid + ((u32)lane >> 4); };
      auto fmsg = [&](u32 r) { return 2 * (ft0 + (u64)ftile(r) * nw) + (u64)fh; };
      auto fvalid = [&](u32 r) { return ftile(r) < fnk && fmsg(r) < count; };
      // both rounds' prefix lines at once (64 B per lane and round)
      u32x4 Q[2][4];
#pragma unroll
      for (u32 r = 0; r < 2; r++) {
        const u64 m = fvalid(r) ? fmsg(r) : 0;
        const u32x4* q = reinterpret_cast<const u32x4*>(base + m * stride - sa.prefix_size);
#pragma unroll
        for (int i = 0; i < 4; i++) Q[r][i] = SUBSPACE_SLOT_VARIANT == 13 ? u32x4{0, 0, 0, 0} : q[i];
      }
      u32 mism = 0;
      bool gave_up = false;
#pragma unroll
      for (u32 r = 0; r < 2; r++) {
        if (16u * r >= nk0) break;  // wave-uniform
        // span-0 term: P = Z_4096(crc_raw(~0, prefix[4, 48)))
        u32 w[16];
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = Q[r][i >> 2][i & 3];
        const bool has = (w[8] & 4u) != 0u;  // kMessageHasChecksum (common/channel.h:62-70)
        const u32 F = calc ? (w[8] | 4u) : w[8];
        w[8] = F;
        u32 hh = 0xFFFFFFFFu;
#pragma unroll
        for (int i = 1; i < 12; i++) hh = step4(hh ^ w[i], lc0, lc1);
        if (sa.metadata_size) {  // wave-uniform: span 1, the metadata after the checksum area
          // dwords from the one holding its first byte (o1 & 3 bytes before it), realigned
          // with a uniform byte shift; full words by step4, the tail by byte steps
          const u32 o1 = 48u + sa.checksum_size, sh = o1 & 3u, ms = sa.metadata_size;
          const u32 nwords = (sh + ms + 3u) >> 2;  // >= 1
          const u64 m = fvalid(r) ? fmsg(r) : 0;
          const u32* p1 = reinterpret_cast<const u32*>(base + m * stride - sa.prefix_size + (o1 & ~3u));
          constexpr u32 kW = kSlotFusedMaxMeta / 4 + 2;
          u32 W1[kW];
#pragma unroll
          for (u32 j = 0; j < kW; j++) {  // only the words the span needs (a uniform bound)
            W1[j] = 0u;
            if (j < nwords) W1[j] = p1[j];
          }
          u32 tail = 0;
#pragma unroll
          for (u32 j = 0; j + 1 < kW; j++) {
            const u32 x = __builtin_amdgcn_alignbyte(W1[j + 1], W1[j], sh);
            if (j < (ms >> 2)) hh = step4(hh ^ x, lc0, lc1);
            if (j == (ms >> 2)) tail = x;
          }
          for (u32 b = 0; b < (ms & 3u); b++) hh = step1(hh, (tail >> (8u * b)) & 0xFFu, lc1);
        }
        const u32 P = opmul(sbase, kUniSlotOpZ4096, hh);
        const u32 S = w[12];  // the stored checksum (first 4 B of the checksum area, prefix + 48)
        const bool valid = fvalid(r);
        const u64 msg = fmsg(r);
        // the payload CRC, once its wave has written it (bounded: a broken invariant raises
        // kFaultSlotRing instead of hanging the GPU, and the wave waits no more)
        const u32 ea = sbase + kUniSlotRing + fw * kSlotRingBytesPerWave + 16u * ftile(r) + 8u * fh;
        u64 e;
        for (u32 spins = 0;; spins++) {
          e = lds_ld64(ea);
          if (gave_up || __ballot(valid && (u32)(e >> 32) != ftile(r)) == 0) break;
          if (spins == kSpinBound) {
            if (lane == 0) raise_fault(sa.fault, kFaultSlotRing);
            gave_up = true;
          }
          __builtin_amdgcn_s_sleep(2);
        }
        const u32 res = (u32)e ^ P;
        u32* pw = reinterpret_cast<u32*>(const_cast<uint8_t*>(base) + msg * stride - sa.prefix_size);
        if (calc) {
          if (valid && SUBSPACE_SLOT_VARIANT != 12) {
            pw[8] = F;     // SetHasChecksum()
            pw[12] = res;  // *reinterpret_cast<uint32_t*>(checksum.data()) = ~crc (client/checksum.h:36)
          }
          if (valid) {
            if (sa.status) sa.status[msg] = 0u;
            if (sa.crc_out) sa.crc_out[msg] = res;
          }
        } else {
          const u32 st = !has ? 2u : (res == S ? 0u : 1u);  // client/checksum.h:46
          if (valid && sa.status) sa.status[msg] = st;
          mism += (u32)__builtin_popcountll(__ballot(valid && st == 1u));
        }
      }
      if (sa.error_count && lane == 0) {
        if (calc) {
          // a publish has no mismatches: the count is 0 (include/subspace_crc.h)
          if (blockIdx.x == 0 && wid == 0) *sa.error_count = 0u;
        } else {
          // the workgroup's count: one LDS atomic per finishing wave, (1 << 24) | its count
          // (< 2^24: at most 512 messages per workgroup); the last of them adds the workgroup's
          // total to the call's counter entry (crc_device.h add_call_mismatches)
          const u32 o = __hip_atomic_fetch_add(reinterpret_cast<lds_u32_t*>((uintptr_t)smism), (1u << 24) | mism,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if ((o >> 24) == (u32)kSlotFinishers - 1u) add_call_mismatches(sa.counter, (o + mism) & 0xFFFFFFu, sa.error_count);
        }
      }
    }
  } else {
    if (nk > kf) flush(kf, nk - kf);
  }
  // a word the caller's next kernel accumulates into (a slot batch's mismatch count): zeroed
  // here, at the end, so the call needs no separate memset
  if (zero_word != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0u;
  if constexpr (PROBE) {
    {
      pt[3] = __builtin_amdgcn_s_memrealtime();
      u64* r = sa.probe + ((u64)blockIdx.x * wpb + (u64)wid) * kProbeWords;
      const u64 xcc = (u64)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
      const u64 hwid = (u64)__builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID: wave slot, SIMD, CU, SE
      const u64 v = lane == 0 ? pt[0] : lane == 1 ? pt[1] : lane == 2 ? pt[2] : lane == 3 ? pt[3]
                  : lane == 4 ? pt_args : lane == 5 ? (xcc | ((u64)nk << 32)) : lane == 6 ? (hwid | (pt_finish << 32)) : pt_landed;
      if (lane < 8) r[lane] = v;
    }
  }
}

#define INST(WGV, SL, PR)                                                                                 \
  template __global__ void crc32_uniform4k_kernel<WGV, SL, PR>(const uint8_t*, u64, u64, const u32*, const u32*, u32, \
                                                               u32, u32*, int, u32*, SlotArgs);
// The product instantiations (512 threads: the round-4/5 workgroup sweeps);
// devtools.hip includes this file for its PROBE ones (libsubspace_crc_dev.so)
#ifndef SUBSPACE_DEV_TU
INST(512, false, false)
INST(512, true, false)
#endif
#undef INST

}  // namespace subspace_amd
