// Host SubspaceCRC32: the per-message drop-in for client/checksum.cc:125-130.
//
// Same function, same result as the reference's default x86-64 build (IEEE 802.3
// reflected polynomial 0xEDB88320, raw state in and out), computed 16 bytes per
// step (slice-by-16) instead of one table lookup per byte. The batched GPU path
// lives in crc_kernels.hip; this host function is what per-message callers
// (publisher.cc:673, subscriber.h:274, user callbacks such as client_test.cc:5234)
// keep calling, because a kernel launch per 4 KiB message would cost more than
// the CRC itself. SubspaceCRC32C is the same function for the CRC-32C polynomial.
#include <cstddef>
#include <cstdint>
#include <cstring>

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

}  // namespace

extern "C" uint32_t SubspaceCRC32(uint32_t crc, const uint8_t* data, size_t length) {
  return crc_slice16(slice16(), crc, data, length);
}

// CRC-32C (Castagnoli), raw state in and out: the value a -msse4.2 / -march=native x86
// build of the reference computes with _mm_crc32_u64/u32/u8 (client/checksum.cc:56-76).
extern "C" uint32_t SubspaceCRC32C(uint32_t crc, const uint8_t* data, size_t length) {
  return crc_slice16(slice16c(), crc, data, length);
}
