// Tile descriptors of the ragged path: the 16-B form, the 8-B form and the expansion that
// writes a wave's messages' 8-B descriptors (crc_ragged.hip descriptor kernel,
// crc_combine.hip fused tile-count scan + descriptor kernel). DESIGN.md 4.3.
#pragma once
#include "crc_device.h"

namespace subspace_amd {

// 16 B per tile: one vector load and four readfirstlanes per tile in the main kernel.
struct TileDesc {
  u64 tile_start;  // absolute offset (from base) of the tile's first byte (16-B aligned)
  u32 after;       // tiles after this one in the message | kFirstTile for its first tile
  u32 len;         // bytes of the extended message in the tile (1..8192) | mis << 16
};
static_assert(sizeof(TileDesc) == 16, "TileDesc is 16 B");
constexpr u32 kFirstTile = 0x80000000u;

// 8 B per tile, the form of every batch whose tile starts lie below 2^37 bytes and whose
// messages have at most 2^25 tiles (crc_device.h kDesc8*): lo = bits 4..35 of the tile start;
// hi = bit 36 of it, mis, the first-tile flag and X = the tiles after this one or, for a
// message's last tile, kLastTile8 | its bytes (only a last tile can be short; 14 bits). Half
// the descriptor kernel's stores and the main kernel's descriptor loads.
struct TileDesc8 {
  u32 lo, hi;
};
static_assert(sizeof(TileDesc8) == 8, "TileDesc8 is 8 B");
constexpr u32 kLastTile8 = 1u << kDesc8AfterBits;

__device__ __forceinline__ TileDesc8 pack_desc8(const TileDesc& d) {
  const u64 s16 = d.tile_start >> 4;
  const u32 after = d.after & ~kFirstTile, len = d.len & 0xFFFFu, mis = d.len >> 16;
  const u32 x = (after == 0u || len == 0u) ? (kLastTile8 | len) : after;  // len 0: a defensive empty tile
  return TileDesc8{(u32)s16, ((u32)(s16 >> 32) & ((1u << kD8StartHiBits) - 1u)) | (mis << kD8MisShift) |
                                 ((d.after & kFirstTile) ? kD8FirstBit : 0u) | (x << kD8XShift)};
}
__device__ __forceinline__ TileDesc unpack_desc8(u32 lo, u32 hi) {
  TileDesc t;
  t.tile_start = ((u64)(hi & ((1u << kD8StartHiBits) - 1u)) << 36) | ((u64)lo << 4);
  const u32 x = hi >> kD8XShift;
  const bool last = (x & kLastTile8) != 0u;
  t.after = (last ? 0u : x) | ((hi & kD8FirstBit) ? kFirstTile : 0u);
  t.len = (last ? (x & 0x3FFFu) : 8192u) | (((hi >> kD8MisShift) & 15u) << 16);
  return t;
}

// The 8-B descriptors of the tiles of one wave's 64 messages, every tile below `limit`. Lane
// l holds its message's first tile t0, tile count nt (0: none), start so and length L. With
// lane_puts, each lane stores its message's first kLaneTiles tiles itself (neighbouring lanes
// hold neighbouring messages, so for small messages the stores are contiguous). The later
// tiles are numbered q = 0 .. W - 1 in message order (an exclusive wave scan of b = nt -
// kLaneTiles) and stored 64 per round, round r of row y (of ystep / 64 rows) storing q = 64 (y +
// r ystep / 64) + lane: every store has 64 useful lanes, and a wave takes W / 64 rounds instead
// of one per long message. The message of a lane's q: with one row, each message starting in
// the round marks its first position in LDS and a DPP max-scan over the lanes carries the
// marks forward from the previous round's last message (three LDS operations a round); with
// more rows a 6-step binary search over the 64 scan values. sx: the wave's kDesc8WaveWords x 64
// words of LDS. The config-C descriptor kernel took 37 us this way, against 52 us with one long
// message after the other per wave and 63-72 us tile-parallel (a shuffle search per 64-tile
// window from chunk hints), r04o-r04p.
constexpr u32 kLaneTiles = 2;  // 1, 4, 8: slower (r04o, r04p)
constexpr int kDesc8WaveWords = 9;  // excl, s16 lo, s16 hi, mis field, last, last_len, t0 lo, t0 hi, marks
__device__ __forceinline__ void desc8_wave(TileDesc8* __restrict__ desc8, u64 limit, u64 t0, u64 nt, u64 so, u64 L,
                                           u32 y, u32 ystep, u32 (*sx)[64], bool lane_puts) {
  const u32 lane = threadIdx.x & 63u;
  const u32 mis = (u32)(so & 15);
  if (lane_puts) {
#pragma unroll
    for (u32 j = 0; j < kLaneTiles; j++) {
      if (j < nt && t0 + j < limit) {
        const u64 rest = L + mis - ((u64)j << 13);
        TileDesc d;
        d.tile_start = (so & ~(u64)15) + ((u64)j << 13);
        d.after = (u32)(nt - 1 - j) | (j == 0 ? kFirstTile : 0u);
        d.len = (rest < 8192 ? (u32)rest : 8192u) | (mis << 16);
        desc8[t0 + j] = pack_desc8(d);
      }
    }
  }
  const u32 b = nt > kLaneTiles ? (u32)nt - kLaneTiles : 0u;
  u32 incl = b;
#pragma unroll
  for (u32 d = 1; d < 64; d <<= 1) {
    const u32 t = (u32)__shfl_up((int)incl, d, 64);
    if (lane >= d) incl += t;
  }
  const u32 W = (u32)__builtin_amdgcn_readlane((int)incl, 63);
  if (W == 0u) return;  // wave-uniform
  const u32 last = (u32)nt - 1u;
  const u64 s16 = so >> 4;
  const u32 ex = incl - b;
  wave_lds_sync();  // the wave's previous use of sx is done
  sx[0][lane] = ex;
  sx[1][lane] = (u32)s16;
  sx[2][lane] = (u32)(s16 >> 32);
  sx[3][lane] = mis << kD8MisShift;
  sx[4][lane] = last;
  sx[5][lane] = (u32)(L + mis - ((u64)last << 13));
  sx[6][lane] = (u32)t0;
  sx[7][lane] = (u32)(t0 >> 32);
  wave_lds_sync();
  u32 carry = (u32)__ffsll((unsigned long long)__ballot(b != 0u));  // (first long message) + 1
  for (u32 q0 = 64u * y; q0 < W; q0 += ystep) {
    const u32 q = q0 + lane;
    u32 o;
    if (ystep == 64u) {
      sx[8][lane] = 0u;
      wave_lds_sync();
      if (b != 0u && ex >= q0 && ex < q0 + 64u) sx[8][ex - q0] = lane + 1u;
      wave_lds_sync();
      u32 v = sx[8][lane];
      v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));  // row_shr:1
      v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));  // row_shr:2
      v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));  // row_shr:4
      v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));  // row_shr:8
      v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));  // row_bcast:15
      v = max(v, (u32)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));  // row_bcast:31
      v = max(v, carry);
      carry = (u32)__builtin_amdgcn_readlane((int)v, 63);
      o = v - 1u;
    } else {
      o = 0;
#pragma unroll
      for (u32 st = 32; st; st >>= 1)
        if (sx[0][o + st] <= q) o += st;
    }
    if (q < W) {
      const u32 j = kLaneTiles + q - sx[0][o];
      const u64 t16 = (((u64)sx[2][o] << 32) | sx[1][o]) + ((u64)j << 9);
      const u32 ol = sx[4][o];
      const u32 x = j == ol ? (kLastTile8 | sx[5][o]) : ol - j;
      const u64 ot0 = ((u64)sx[7][o] << 32) | sx[6][o];
      if (ot0 + j < limit)
        desc8[ot0 + j] = TileDesc8{(u32)t16, ((u32)(t16 >> 32) & ((1u << kD8StartHiBits) - 1u)) | sx[3][o] |
                                                  (x << kD8XShift)};
    }
  }
}

// The 16-B descriptors of the tiles of one wave's 64 messages (the fused tile-count scan's form
// for batches of absolute addresses, beyond the 8-B form's 2^37-byte range): each lane stores its
// message's first kLaneTilesW tiles, then longer messages one after the other, 64 tiles per
// store (as crc32_ragged_desc_kernel's wide batches). Tiles at or past `limit` are not stored.
constexpr u32 kLaneTilesW = 8;
__device__ __forceinline__ void descw_tile(TileDesc* __restrict__ desc, u64 limit, u64 so, u64 L, u64 t0, u64 nt,
                                           u64 j) {
  if (t0 + j >= limit) return;
  const u32 mis = (u32)(so & 15);
  const u64 rest = L + mis - (j << 13);
  TileDesc d;
  d.tile_start = (so & ~(u64)15) + (j << 13);
  d.after = (u32)(nt - 1 - j) | (j == 0 ? kFirstTile : 0u);
  d.len = (rest < 8192 ? (u32)rest : 8192u) | (mis << 16);
  desc[t0 + j] = d;
}
__device__ __forceinline__ void descw_wave(TileDesc* __restrict__ desc, u64 limit, u64 t0, u64 nt, u64 so, u64 L) {
  const u32 lane = threadIdx.x & 63u;
#pragma unroll
  for (u32 j = 0; j < kLaneTilesW; j++)
    if (j < nt) descw_tile(desc, limit, so, L, t0, nt, j);
  u64 big = __ballot(nt > kLaneTilesW);
  while (big) {  // wave-uniform
    const int src = __ffsll((unsigned long long)big) - 1;
    big &= big - 1;
    const u64 bt0 = __shfl(t0, src, 64), bnt = __shfl(nt, src, 64);
    const u64 bso = __shfl(so, src, 64), bL = __shfl(L, src, 64);
    for (u64 j = kLaneTilesW + lane; j < bnt; j += 64) descw_tile(desc, limit, bso, bL, bt0, bnt, j);
  }
}

}  // namespace subspace_amd
