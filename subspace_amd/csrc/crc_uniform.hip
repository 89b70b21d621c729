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
//    with span0 = prefix[4, 48). The payload term is this kernel's message CRC from init 0.
//    Per window of 32 tiles (64 messages, one per lane) each lane loads its message's 64-B
//    prefix line -- issued with the window's first tile loads, so it lands with them -- and at
//    the window's end computes crc_raw(~0, span0) (11 steps, flag bit set first for a
//    publish, as SetHasChecksum() precedes the checksum: client/publisher.cc:664-675) and
//    one Z_4096 opmul, XORs it into its ring slot and stores flag + checksum (publish) or
//    the status (verify: client/client.cc:1346-1356; no kMessageHasChecksum -> unchecked).
//    Mismatches are counted per workgroup and summed by one 64-bit atomic per workgroup
//    that also counts finished workgroups; the last one writes the call's total.
#include "crc_device.h"


namespace subspace_amd {

template <int WG, bool SLOT, bool PROBE>
__global__ __launch_bounds__(WG) void crc32_uniform4k_kernel(const uint8_t* __restrict__ base, u64 stride, u64 count,
                                                             const u32* __restrict__ gtab, const u32* __restrict__ gops,
                                                             u32 init, u32 final_xor, u32* __restrict__ out,
                                                             int order, u32* __restrict__ zero_word, SlotArgs sa) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
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
  // four pairs); config S publish 48.96 -> 48.70 us, verify 47.87 -> 47.62 (r02c20); bit-exact.
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
  constexpr int kRing = SLOT ? kUniSlotRingResults : uni_ring_results(WG / 64);
  const u32 ring = sbase + (SLOT ? kUniSlotRing : kUniRing) + (u32)wid * (4u * kRing);
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
  constexpr u64 wpb = WG / 64;
  const u64 nw = (u64)gridDim.x * wpb;
  u64 t0, tstep, tend;
  // order 3 needs whole XCD groups: 8 | G and 16 | (G/8)*wpb; otherwise it is order 0
  if (order == 3 && ((gridDim.x & 7u) || ((((u64)gridDim.x >> 3) * wpb) & 15u))) order = 0;
  if (order == 0) {
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
  // which make all this address math scalar, measured 7-10 % slower: DESIGN.md 4.1.)
  auto load_tile = [&](u32x4 (&d)[8], u32 k) {
    const u32 kk = k < nk ? k : (nk ? nk - 1 : 0u);
    u64 msg = nk ? 2 * (t0 + (u64)kk * tstep) + (u64)h : 0;
    msg = msg < count ? msg : msg - 1;
    const u32x4* q = reinterpret_cast<const u32x4*>(base + msg * stride + (u64)l * 128);
#pragma unroll
    for (int i = 0; i < 8; i++) d[i] = q[i];
    // keep the loads at this point, in order (hipcc otherwise sinks them into the compute)
    __builtin_amdgcn_sched_barrier(0);
  };

  // CRC of this lane's line of a tile (from the batch init for line 0, else from 0).
  const u32 z64 = sbase + kLdsOps + 512u * (u32)kUniSlotOpZ64 + 4u * (u32)(lane & 3);
  auto line_crc = [&](const u32x4 (&d)[8]) {
    if constexpr (kTwoChain) return line_crc32_2chain(d, s_init, lc0, lc1, z64);
    else return line_crc32(d, s_init, lc0, lc1);
  };
  // Message CRCs of tile k into ring slots 2*(k - kf) + h (kf = first tile of the window).
  auto tile_result = [&](u32 crc, u32 k, u32 kf) {
    u32 v = lane_shift(lop, crc);
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v ^= (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    if (l == 31) lds_st(ring + 4u * (2u * (k - kf) + (u32)h), v ^ final_xor);
  };
  // SLOT: the current window's prefix lines (lane j: message j of the window), their span-0
  // term P = Z_4096(crc_raw(~0, span0)), stored checksum S, flags word F, the flag as found.
  u32x4 Q[4];
  u32 P = 0, S = 0, F = 0, mism = 0;
  bool HAS = false;
  const bool calc = sa.mode == 0u;
  // message of lane j in the window of tiles kf.. (clamped like load_tile for the loads)
  auto win_msg = [&](u32 kf, bool clamp) {
    const u32 t = kf + ((u32)lane >> 1);
    const u32 kk = !clamp ? t : (t < nk ? t : (nk ? nk - 1 : 0u));
    u64 msg = (nk || !clamp) ? 2 * (t0 + (u64)kk * tstep) + (u64)(lane & 1) : 0;
    if (clamp) msg = msg < count ? msg : msg - 1;
    return msg;
  };
  auto load_prefix = [&](u32 kf) {
    const u32x4* q = reinterpret_cast<const u32x4*>(base + win_msg(kf, true) * stride - sa.prefix_size);
#pragma unroll
    for (int i = 0; i < 4; i++) Q[i] = q[i];
    __builtin_amdgcn_sched_barrier(0);
  };
  // After the drain that follows window 0's prefix loads: every loaded prefix word counts as
  // used here. Words the checksum never reads (bytes 0-3, the checksum area's tail) would
  // otherwise leave their registers free while the loads are in flight, and hipcc reused such
  // a register in tile 0's compute -- which then waited for the prefix loads and for tile 1's,
  // issued before them (config S publish 50.2 -> 49.6 us, verify 49.2 -> 48.4, r02c5). The
  // same hint after the loop's drains ran 8.7 us slower (r02c4): only here.
  auto prefix_landed = [&]() {
#pragma unroll
    for (int i = 0; i < 4; i++) asm volatile("" ::"v"(Q[i]));
  };
  auto prefix_pass = [&]() {
    u32 w[16];
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = Q[i >> 2][i & 3];
    HAS = (w[8] & 4u) != 0u;  // kMessageHasChecksum in MessagePrefix::flags (common/channel.h:62-70)
    F = calc ? (w[8] | 4u) : w[8];
    w[8] = F;
    u32 hh = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 1; i < 12; i++) hh = step4(hh ^ w[i], lc0, lc1);  // span 0 = prefix bytes [4, 48)
    P = opmul(sbase, kUniSlotOpZ4096, hh);
    S = w[12];  // the stored checksum (first 4 B of the checksum area, prefix + 48)
  };
  // Finish the window's messages: lane j takes ring slot j (its payload CRC, complemented)
  // and XORs in its span-0 term; then stores flag + checksum, or the status.
  auto slot_flush = [&](u32 kf, u32 nt) {
    const u64 msg = win_msg(kf, false);
    const bool valid = ((u32)lane >> 1) < nt && msg < count;
    const u32 r = lds_ld(ring + 4u * (u32)lane) ^ P;
    u32* pw = reinterpret_cast<u32*>(const_cast<uint8_t*>(base) + msg * stride - sa.prefix_size);
    if (calc) {
      if (valid) {
        pw[8] = F;   // SetHasChecksum()
        pw[12] = r;  // *reinterpret_cast<uint32_t*>(checksum.data()) = ~crc (client/checksum.h:36)
        if (sa.status) sa.status[msg] = 0u;
        if (sa.crc_out) sa.crc_out[msg] = r;
      }
    } else {
      const u32 st = !HAS ? 2u : (r == S ? 0u : 1u);  // client/checksum.h:46
      if (valid && sa.status) sa.status[msg] = st;
      mism += (u32)__builtin_popcountll(__ballot(valid && st == 1u));
    }
    wave_lds_sync();
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
  // SLOT: a window's prefix lines are loaded with its first tile's loads (window 0's with
  // tile 1's, below); the window ends right after a drain, before the next tile's loads,
  // where its span-0 terms are computed and its messages finished and stored, and the next
  // window's prefix lines are loaded.
  // (Computing the span-0 terms right after the window's first drain instead -- so that only
  // the stores remain at the end -- ran 62 vs 50 us at config S in an interleaved A/B, r02l.)
  u32 k = 0, kf = 0;
  // SLOT: window 0's prefix lines go out with tile 1's loads, not with tile 0's: 4 MiB of
  // scattered 64-B reads in the kernel's first flood delayed every wave's tile 0 by 1.6 us
  // (tools/wave_timeline.py --mode publish, r02ai; config S publish 49.65 -> 49.42 us, verify
  // 48.67 -> 48.45 us, tools/session_slotab.sh r02ak). The pair is peeled so that the wait for
  // tile 0 counts the prefix loads exactly (inside the loop, a conditional load would make
  // hipcc's merged count wait for the next tile's loads before computing the current one).
  if constexpr (SLOT) {
    if (k + 2 < nk) {
      load_tile(B, 1);
      load_prefix(0);
      tile_result(line_crc(A), 0, 0);
      drain_before_issue();
      prefix_landed();
      load_tile(A, 2);
      tile_result(line_crc(B), 1, 0);
      k = 2;
    } else {
      load_prefix(0);
    }
  }
  // SLOT: the loop stops before the wave's last pair, which follows it: the last window's
  // span-0 terms are computed while the wave's last tile is in flight
  for (; SLOT ? k + 2 < nk : k + 1 < nk; k += 2) {
    drain_before_issue();
    if constexpr (SLOT) {
      if (k - kf == (u32)(kRing / 2)) {
        prefix_pass();
        wave_lds_sync();
        slot_flush(kf, kRing / 2);
        load_prefix(k);
        kf = k;
      }
      load_tile(B, k + 1);
    } else {
      load_tile(B, k + 1);
      if (k - kf == (u32)(kRing / 2)) {
        wave_lds_sync();
        flush(kf, kRing / 2);
        kf = k;
      }
    }
    tile_result(line_crc(A), k, kf);
    drain_before_issue();
    load_tile(A, k + 2);
    tile_result(line_crc(B), k + 1, kf);
  }
  if constexpr (PROBE) pt[2] = __builtin_amdgcn_s_memrealtime();
  bool pdone = false;  // SLOT: the current window's span-0 terms are computed
  if constexpr (SLOT) {
    if (k + 1 < nk) {  // the last pair: tile k loaded, tile k+1 the wave's last
      drain_before_issue();
      if (k - kf == (u32)(kRing / 2)) {
        prefix_pass();
        wave_lds_sync();
        slot_flush(kf, kRing / 2);
        load_prefix(k);
        kf = k;
      }
      load_tile(B, k + 1);
      if (k != kf) {  // the window's prefix lines landed a tile ago: overlap with tile k+1's loads
        prefix_pass();
        pdone = true;
      }
      tile_result(line_crc(A), k, kf);
      drain_before_issue();
      tile_result(line_crc(B), k + 1, kf);
      k += 2;
    }
  }
  if (k < nk) {  // odd last tile, already loaded
    if (k - kf == (u32)(kRing / 2)) {
      if constexpr (SLOT) {
        prefix_pass();
        wave_lds_sync();
        slot_flush(kf, kRing / 2);
        load_prefix(k);
      } else {
        wave_lds_sync();
        flush(kf, kRing / 2);
      }
      kf = k;
    }
    tile_result(line_crc(A), k, kf);
  }
  wave_lds_sync();
  u64 pt_flush = 0;
  if constexpr (SLOT) {
    if (!pdone) prefix_pass();
    if constexpr (PROBE) pt_flush = __builtin_amdgcn_s_memrealtime();
    slot_flush(kf, nk > kf ? nk - kf : 0u);
    // the call's mismatch count: one 64-bit atomic per workgroup adds (1 << 32) | its count;
    // the workgroup that sees G - 1 finished before it writes the total and resets the word
    if (!calc && sa.error_count) {
      const u32 mring = sbase + kUniSlotRing + (u32)wid * (4u * kRing);
      if (lane == 0) lds_st(mring, mism);
      __syncthreads();
      if (threadIdx.x == 0) {
        u32 n = 0;
#pragma unroll
        for (int q = 0; q < WG / 64; q++) n += lds_ld(sbase + kUniSlotRing + (u32)q * (4u * kRing));
        const u64 old = atomicAdd(reinterpret_cast<unsigned long long*>(sa.counter), (1ull << 32) | (u64)n);
        if ((u32)(old >> 32) == gridDim.x - 1u) {
          *sa.error_count = (u32)old + n;
          __hip_atomic_store(sa.counter, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
    pt[3] = __builtin_amdgcn_s_memrealtime();
    u64* r = sa.probe + ((u64)blockIdx.x * wpb + (u64)wid) * kProbeWords;
    const u64 xcc = (u64)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
    const u64 v = lane == 0 ? pt[0] : lane == 1 ? pt[1] : lane == 2 ? pt[2] : lane == 3 ? pt[3]
                : lane == 4 ? pt_args : lane == 5 ? (xcc | ((u64)nk << 32)) : lane == 6 ? pt_flush : pt_landed;
    if (lane < 8) r[lane] = v;
  }
}

#define INST(WGV, SL, PR)                                                                                 \
  template __global__ void crc32_uniform4k_kernel<WGV, SL, PR>(const uint8_t*, u64, u64, const u32*, const u32*, u32, \
                                                               u32, u32*, int, u32*, SlotArgs);
INST(256, false, false)
INST(512, false, false)
INST(768, false, false)
INST(1024, false, false)
INST(512, true, false)
INST(512, false, true)
INST(512, true, true)
#undef INST

}  // namespace subspace_amd
