// Host-side CRC-32 algebra used to build the device tables.
//
// Notation. The reference's raw CRC state c (client/checksum.cc:125-130) is a
// polynomial over GF(2) in the reflected representation; every quantity below is
// linear in it:
//   crc_raw(c, A || B) = Z_{|B|}(crc_raw(c, A)) ^ crc_raw(0, B)
// where Z_n(c) = crc_raw(c, n zero bytes) -- "advance the state over n zero bytes",
// multiplication by x^(8n) mod P. T4(x) = crc_raw(0, 4 LE bytes of x) = Z_4(x) is
// the slice-by-4 step. Every operator is a 32x32 GF(2) matrix (Mat32, columns).
#pragma once
#include <array>
#include <cstdint>

namespace subspace_amd {

constexpr uint32_t kPoly = 0xEDB88320u;            // reflected IEEE 802.3 (client/checksum.cc:78)
constexpr uint32_t kPolyCastagnoli = 0x82F63B78u;  // reflected CRC-32C: what _mm_crc32_* compute
                                                   // (client/checksum.cc:56-76, -msse4.2 builds)

struct Tables {
  uint32_t t[4][256];  // t[0]: byte table; t[k][b] = CRC of byte b followed by k zero bytes
};

inline Tables make_tables(uint32_t poly = kPoly) {
  Tables tb{};
  for (uint32_t b = 0; b < 256; b++) {
    uint32_t c = b;
    for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ poly : (c >> 1);
    tb.t[0][b] = c;
  }
  for (int k = 1; k < 4; k++)
    for (uint32_t b = 0; b < 256; b++) tb.t[k][b] = (tb.t[k - 1][b] >> 8) ^ tb.t[0][tb.t[k - 1][b] & 0xFF];
  return tb;
}

struct Mat32 {
  uint32_t col[32];  // col[i] = image of the basis vector 1 << i
};

inline uint32_t apply(const Mat32& m, uint32_t v) {
  uint32_t r = 0;
  for (int i = 0; i < 32; i++)
    if ((v >> i) & 1u) r ^= m.col[i];
  return r;
}
inline Mat32 mul(const Mat32& a, const Mat32& b) {  // a o b
  Mat32 r;
  for (int i = 0; i < 32; i++) r.col[i] = apply(a, b.col[i]);
  return r;
}
inline Mat32 identity() {
  Mat32 m;
  for (int i = 0; i < 32; i++) m.col[i] = 1u << i;
  return m;
}
// Z_1: advance over one zero byte.
inline Mat32 z_one(const Tables& tb) {
  Mat32 m;
  for (int i = 0; i < 32; i++) {
    const uint32_t c = 1u << i;
    m.col[i] = (c >> 8) ^ tb.t[0][c & 0xFF];
  }
  return m;
}
// Z_n by square-and-multiply.
inline Mat32 z_bytes(const Tables& tb, uint64_t n) {
  Mat32 r = identity(), p = z_one(tb);
  while (n) {
    if (n & 1) r = mul(p, r);
    p = mul(p, p);
    n >>= 1;
  }
  return r;
}
// T4 as a matrix (== z_bytes(tb, 4)).
inline Mat32 t4(const Tables& tb) {
  Mat32 m;
  for (int i = 0; i < 32; i++) {
    const uint32_t c = 1u << i;
    m.col[i] = tb.t[3][c & 0xFF] ^ tb.t[2][(c >> 8) & 0xFF] ^ tb.t[1][(c >> 16) & 0xFF] ^ tb.t[0][c >> 24];
  }
  return m;
}
// Inverse over GF(2) (Gauss-Jordan). Z_n is always invertible (P has a constant term).
inline Mat32 inverse(const Mat32& m) {
  // Work on rows: build row-major [M | I].
  uint32_t a[32], inv[32];
  for (int r = 0; r < 32; r++) {
    a[r] = 0;
    for (int c = 0; c < 32; c++) a[r] |= ((m.col[c] >> r) & 1u) << c;
    inv[r] = 1u << r;
  }
  for (int c = 0; c < 32; c++) {
    int p = c;
    while (p < 32 && !((a[p] >> c) & 1u)) p++;
    if (p == 32) return identity();  // singular: cannot happen for Z_n
    uint32_t t = a[p]; a[p] = a[c]; a[c] = t;
    t = inv[p]; inv[p] = inv[c]; inv[c] = t;
    for (int r = 0; r < 32; r++)
      if (r != c && ((a[r] >> c) & 1u)) { a[r] ^= a[c]; inv[r] ^= inv[c]; }
  }
  Mat32 out;
  for (int c = 0; c < 32; c++) {
    out.col[c] = 0;
    for (int r = 0; r < 32; r++) out.col[c] |= ((inv[r] >> c) & 1u) << r;
  }
  return out;
}
// Nibble tables of an operator: out[16*k + n] = M(n << 4k), k = 0..7 (128 dwords = 512 B).
inline void nibble_tables(const Mat32& m, uint32_t* out) {
  for (int k = 0; k < 8; k++)
    for (uint32_t n = 0; n < 16; n++) out[16 * k + n] = apply(m, n << (4 * k));
}

}  // namespace subspace_amd
