// Host SubspaceCRC32: the per-message drop-in for client/checksum.cc:125-130.
//
// Same function, same result as the reference's default x86-64 build (IEEE 802.3
// reflected polynomial 0xEDB88320, raw state in and out), computed 16 bytes per
// step (slice-by-16) instead of one table lookup per byte. The batched GPU path
// lives in crc_uniform.hip / crc_ragged.hip / crc_long.hip; this host function is what per-message callers
// (publisher.cc:673, subscriber.h:274, user callbacks such as client_test.cc:5234)
// keep calling, because a kernel launch per 4 KiB message would cost more than
// the CRC itself. SubspaceCRC32C is the same function for the CRC-32C polynomial (the
// folding below with the Castagnoli constants for bodies of 256 B or more where the CPU has
// AVX-512 VPCLMULQDQ, the SSE4.2 crc32 instruction for the rest, slice-by-16 otherwise).
//
// On x86-64 CPUs with PCLMULQDQ (every current server part; checked at run time) the
// 16-B-multiple body of an IEEE CRC of 64 bytes or more is folded with carry-less
// multiplies (4 x 128-bit lanes, then one, then a Barrett reduction to 32 bits; the
// published folding scheme for reflected CRCs, with the constants below derived for
// 0xEDB88320), the remaining bytes by slice-by-16. Where the CPU also has AVX-512 with
// VPCLMULQDQ (Zen 4/5 EPYC such as the MI355X hosts' 9575F, Ice Lake and later Xeons), bodies
// of 256 bytes or more are folded 4 x 512 bits per step first. SUBSPACE_CRC_HOST_ISA=
// vpclmul|pclmul|table caps the path (read once; tests use it to cover every path on one
// machine). tests/test_host_api.py checks every boundary of the split against zlib.
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "crc_math.h"

namespace {

struct Slice16 {
  uint32_t t[16][256];  // t[k][b] = CRC of byte b followed by k zero bytes
  explicit Slice16(uint32_t poly) {
    const subspace_amd::Tables tb = subspace_amd::make_tables(poly);
    for (int b = 0; b < 256; b++) t[0][b] = tb.t[0][b];
    for (int k = 1; k < 16; k++)
      for (int b = 0; b < 256; b++) t[k][b] = (t[k - 1][b] >> 8) ^ t[0][t[k - 1][b] & 0xFF];
  }
};

const Slice16& slice16() {
  static const Slice16 s(subspace_amd::kPoly);  // thread-safe init (C++11 magic statics)
  return s;
}

const Slice16& slice16c() {
  static const Slice16 s(subspace_amd::kPolyCastagnoli);
  return s;
}

inline uint32_t load_le32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);  // any alignment
#if defined(__BYTE_ORDER__) && __BYTE_ORDER__ == __ORDER_BIG_ENDIAN__
  v = __builtin_bswap32(v);
#endif
  return v;
}

uint32_t crc_slice16(const Slice16& s, uint32_t crc, const uint8_t* data, size_t length) {
  const auto& t = s.t;
  while (length >= 16) {
    const uint32_t a = load_le32(data) ^ crc;
    const uint32_t b = load_le32(data + 4);
    const uint32_t c = load_le32(data + 8);
    const uint32_t d = load_le32(data + 12);
    crc = t[15][a & 0xFF] ^ t[14][(a >> 8) & 0xFF] ^ t[13][(a >> 16) & 0xFF] ^ t[12][a >> 24] ^
          t[11][b & 0xFF] ^ t[10][(b >> 8) & 0xFF] ^ t[9][(b >> 16) & 0xFF] ^ t[8][b >> 24] ^
          t[7][c & 0xFF] ^ t[6][(c >> 8) & 0xFF] ^ t[5][(c >> 16) & 0xFF] ^ t[4][c >> 24] ^
          t[3][d & 0xFF] ^ t[2][(d >> 8) & 0xFF] ^ t[1][(d >> 16) & 0xFF] ^ t[0][d >> 24];
    data += 16;
    length -= 16;
  }
  while (length--) crc = (crc >> 8) ^ t[0][(crc ^ *data++) & 0xFF];
  return crc;
}

#if defined(__x86_64__)
// Raw-state CRC of len bytes (len >= 64, len % 16 == 0) by carry-less folding.
// Folding constants, bit-reflected and shifted left by one (reflected-domain products):
//   k_D    = x^(D+32), x^(D-32) mod P (low, high qword)  fold a 128-bit lane forward by D bits
//            (D = 2048: 4 x 512-bit step; 512: 4 x 128-bit step and zmm -> zmm; 128: lane -> lane)
//   k5     = x^64 mod P                                   (128 -> 64 -> 32 bits)
//   mu, p  = x^64 div P and P, reflected (33 bits), for the Barrett reduction.
// The two sets below were derived from the polynomials (tools-free: a few lines of GF(2)
// arithmetic); the CRC-32C set equals the published one for 0x82F63B78.
struct FoldConsts {
  long long k2048[2], k512[2], k128[2], k5, mu, p;
};
constexpr FoldConsts kFoldIeee = {{0x11542778all, 0x1322d1430ll}, {0x154442bd4ll, 0x1c6e41596ll},
                                  {0x1751997d0ll, 0x0ccaa009ell}, 0x163cd6124ll, 0x1f7011641ll, 0x1db710641ll};
constexpr FoldConsts kFoldCastagnoli = {{0x0dcb17aa4ll, 0x0b9e02b86ll}, {0x0740eef02ll, 0x09e4addf8ll},
                                        {0x0f20c0dfell, 0x14cd00bd6ll}, 0x0dd45aab8ll, 0x0dea713f1ll, 0x105ec76f1ll};

#define SUBSPACE_PCLMUL __attribute__((target("pclmul,sse4.1")))
SUBSPACE_PCLMUL inline __m128i ld128(const uint8_t* q) { return _mm_loadu_si128(reinterpret_cast<const __m128i*>(q)); }
SUBSPACE_PCLMUL inline __m128i fold128(__m128i x, __m128i k, __m128i next) {  // x * k (both halves) + next
  return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11)), next);
}

// Fold four 128-bit lanes (x1 oldest) and the remaining 16-B blocks into one, then reduce to
// the raw 32-bit state.
SUBSPACE_PCLMUL uint32_t finish128(const FoldConsts& c, __m128i x1, __m128i x2, __m128i x3, __m128i x4,
                                   const uint8_t* p, size_t len) {
  const __m128i k34 = _mm_set_epi64x(c.k128[1], c.k128[0]);
  const __m128i k5 = _mm_set_epi64x(0, c.k5);
  const __m128i mup = _mm_set_epi64x(c.mu, c.p);
  const __m128i mask32 = _mm_set_epi32(0, 0, 0, -1);
  x1 = fold128(x1, k34, x2);
  x1 = fold128(x1, k34, x3);
  x1 = fold128(x1, k34, x4);
  for (; len >= 16; p += 16, len -= 16) x1 = fold128(x1, k34, ld128(p));
  // 128 -> 64 bits
  x1 = _mm_xor_si128(_mm_clmulepi64_si128(x1, k34, 0x10), _mm_srli_si128(x1, 8));
  // 64 -> 32 bits
  x1 = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(x1, mask32), k5, 0x00), _mm_srli_si128(x1, 4));
  // Barrett reduction
  __m128i t = _mm_clmulepi64_si128(_mm_and_si128(x1, mask32), mup, 0x10);
  t = _mm_clmulepi64_si128(_mm_and_si128(t, mask32), mup, 0x00);
  return (uint32_t)_mm_extract_epi32(_mm_xor_si128(x1, t), 1);
}

SUBSPACE_PCLMUL uint32_t crc_pclmul(const FoldConsts& c, uint32_t crc, const uint8_t* p, size_t len) {
  const __m128i k12 = _mm_set_epi64x(c.k512[1], c.k512[0]);
  __m128i x1 = _mm_xor_si128(ld128(p), _mm_cvtsi32_si128((int)crc));
  __m128i x2 = ld128(p + 16), x3 = ld128(p + 32), x4 = ld128(p + 48);
  p += 64;
  len -= 64;
  for (; len >= 64; p += 64, len -= 64) {
    x1 = fold128(x1, k12, ld128(p));
    x2 = fold128(x2, k12, ld128(p + 16));
    x3 = fold128(x3, k12, ld128(p + 32));
    x4 = fold128(x4, k12, ld128(p + 48));
  }
  return finish128(c, x1, x2, x3, x4, p, len);
}

// The same scheme on 512-bit registers (len >= 256, len % 16 == 0): four zmm accumulators
// fold by 2,048 bits per step, then into one zmm by 512 bits, 64-B blocks likewise, and its
// four 128-bit lanes go to finish128.
#define SUBSPACE_VPCLMUL __attribute__((target("avx512f,avx512vl,vpclmulqdq,pclmul,sse4.1")))
SUBSPACE_VPCLMUL inline __m512i ld512(const uint8_t* q) { return _mm512_loadu_si512(q); }
SUBSPACE_VPCLMUL inline __m512i fold512(__m512i x, __m512i k, __m512i next) {
  return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x, k, 0x00), _mm512_clmulepi64_epi128(x, k, 0x11), next,
                                   0x96);  // a ^ b ^ c
}

SUBSPACE_VPCLMUL uint32_t crc_vpclmul(const FoldConsts& c, uint32_t crc, const uint8_t* p, size_t len) {
  const __m512i k2048 = _mm512_broadcast_i32x4(_mm_set_epi64x(c.k2048[1], c.k2048[0]));
  const __m512i k512 = _mm512_broadcast_i32x4(_mm_set_epi64x(c.k512[1], c.k512[0]));
  __m512i z0 = _mm512_xor_si512(ld512(p), _mm512_zextsi128_si512(_mm_cvtsi32_si128((int)crc)));
  __m512i z1 = ld512(p + 64), z2 = ld512(p + 128), z3 = ld512(p + 192);
  p += 256;
  len -= 256;
  for (; len >= 256; p += 256, len -= 256) {
    z0 = fold512(z0, k2048, ld512(p));
    z1 = fold512(z1, k2048, ld512(p + 64));
    z2 = fold512(z2, k2048, ld512(p + 128));
    z3 = fold512(z3, k2048, ld512(p + 192));
  }
  z0 = fold512(z0, k512, z1);
  z0 = fold512(z0, k512, z2);
  z0 = fold512(z0, k512, z3);
  for (; len >= 64; p += 64, len -= 64) z0 = fold512(z0, k512, ld512(p));
  return finish128(c, _mm512_extracti32x4_epi32(z0, 0), _mm512_extracti32x4_epi32(z0, 1),
                   _mm512_extracti32x4_epi32(z0, 2), _mm512_extracti32x4_epi32(z0, 3), p, len);
}

// CRC-32C with the SSE4.2 crc32 instruction (the same instruction the reference's
// -msse4.2 build uses, client/checksum.cc:56-76): 8 bytes per step, raw state in and out.
__attribute__((target("sse4.2"))) uint32_t crc32c_sse42(uint32_t crc, const uint8_t* p, size_t len) {
  uint64_t c = crc;
  for (; len >= 8; p += 8, len -= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
  }
  uint32_t c32 = (uint32_t)c;
  for (; len; p++, len--) c32 = _mm_crc32_u8(c32, *p);
  return c32;
}

// The crc32 instruction path of SubspaceCRC32C: the CPU's SSE4.2 alone decides (not the
// folding paths' PCLMULQDQ), unless SUBSPACE_CRC_HOST_ISA=table asks for tables only.
bool use_crc32_insn() {
  static const bool ok = [] {
    const char* e = std::getenv("SUBSPACE_CRC_HOST_ISA");
    return __builtin_cpu_supports("sse4.2") && !(e && !std::strcmp(e, "table"));
  }();
  return ok;
}

// The widest folding path this CPU has, capped by SUBSPACE_CRC_HOST_ISA: 2 = VPCLMULQDQ on
// AVX-512, 1 = PCLMULQDQ, 0 = tables only.
int host_isa() {
  static const int isa = [] {
    int v = 0;
    if (__builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1")) {
      v = 1;
      if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") &&
          __builtin_cpu_supports("vpclmulqdq"))
        v = 2;
    }
    if (const char* e = std::getenv("SUBSPACE_CRC_HOST_ISA")) {
      const int cap = !std::strcmp(e, "table") ? 0 : !std::strcmp(e, "pclmul") ? 1 : 2;
      v = v < cap ? v : cap;
    }
    return v;
  }();
  return isa;
}
#endif

}  // namespace

extern "C" uint32_t SubspaceCRC32(uint32_t crc, const uint8_t* data, size_t length) {
#if defined(__x86_64__)
  if (length >= 64 && host_isa() > 0) {
    const size_t body = length & ~(size_t)15;
    crc = body >= 256 && host_isa() == 2 ? crc_vpclmul(kFoldIeee, crc, data, body)
                                         : crc_pclmul(kFoldIeee, crc, data, body);
    data += body;
    length -= body;
  }
#endif
  return crc_slice16(slice16(), crc, data, length);
}

// CRC-32C (Castagnoli), raw state in and out: the value a -msse4.2 / -march=native x86
// build of the reference computes with _mm_crc32_u64/u32/u8 (client/checksum.cc:56-76).
extern "C" uint32_t SubspaceCRC32C(uint32_t crc, const uint8_t* data, size_t length) {
#if defined(__x86_64__)
  // bodies of 256 B or more by 4 x 512-bit folding where the CPU has it (one serial crc32
  // chain is latency-bound at ~8 B per 3 cycles), the rest by the crc32 instruction
  if (length >= 256 && host_isa() == 2) {
    const size_t body = length & ~(size_t)15;
    crc = crc_vpclmul(kFoldCastagnoli, crc, data, body);
    data += body;
    length -= body;
  }
  if (use_crc32_insn()) return crc32c_sse42(crc, data, length);
#endif
  return crc_slice16(slice16c(), crc, data, length);
}
