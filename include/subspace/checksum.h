// Drop-in replacement for dallison/subspace client/checksum.h.
//
// Same API surface, so publisher/subscriber code compiles against it unchanged:
//   - SUBSPACE_HARDWARE_CRC                    (reference client/checksum.h:14)
//   - extern "C" SubspaceCRC32(crc, data, len) (reference client/checksum.h:18-20)
//       raw-state in/out: the caller does the 0xFFFFFFFF init and the final ~,
//       chainable across spans, pure and reentrant, any alignment, len 0 = no-op.
//       Bit-exact with the reference's default x86-64 build (IEEE 802.3 reflected
//       polynomial 0xEDB88320, client/checksum.cc:78-130).
//   - ChecksumCallback                         (reference client/checksum.h:25-27)
//   - CalculateCRC32Checksum<N> / VerifyCRC32Checksum<N> (reference :29-47)
//
// The host symbol SubspaceCRC32 is exported by libsubspace_crc.so (built from
// subspace_amd/csrc/host_crc.cpp). The batched device path -- one CRC32 per message
// over a whole batch of device-resident slot payloads -- is the C ABI in
// include/subspace_crc.h.
#pragma once

#if __has_include("absl/types/span.h")
#include "absl/types/span.h"
#else
// absl is not available: provide the minimal absl::Span the reference signatures
// use (data(), size(), operator[], (ptr, len) constructor, begin/end). When absl IS
// present the real type is used, so the signatures are identical to the reference.
#include <cstddef>
namespace absl {
template <typename T>
class Span {
 public:
  using element_type = T;
  constexpr Span() noexcept : ptr_(nullptr), len_(0) {}
  constexpr Span(T* ptr, std::size_t len) noexcept : ptr_(ptr), len_(len) {}
  template <typename U, std::size_t N>
  constexpr Span(U (&a)[N]) noexcept : ptr_(a), len_(N) {}
  constexpr T* data() const noexcept { return ptr_; }
  constexpr std::size_t size() const noexcept { return len_; }
  constexpr bool empty() const noexcept { return len_ == 0; }
  constexpr T& operator[](std::size_t i) const noexcept { return ptr_[i]; }
  constexpr T* begin() const noexcept { return ptr_; }
  constexpr T* end() const noexcept { return ptr_ + len_; }

 private:
  T* ptr_;
  std::size_t len_;
};
}  // namespace absl
#endif

#include <array>
#include <cstddef>
#include <cstdint>
#include <functional>

// Undefine this if you don't want to use hardware CRC32 instructions
#define SUBSPACE_HARDWARE_CRC 1

namespace subspace {

extern "C" {
uint32_t SubspaceCRC32(uint32_t crc, const uint8_t *data, size_t length);
// CRC-32C, the function a -msse4.2 x86 build of the reference computes in SubspaceCRC32
// (client/checksum.cc:56-76). A deployment that must interoperate with such peers builds
// with -DSUBSPACE_CRC_CASTAGNOLI, which routes the templates below to it.
uint32_t SubspaceCRC32C(uint32_t crc, const uint8_t *data, size_t length);
}

#if defined(SUBSPACE_CRC_CASTAGNOLI)
#define SUBSPACE_CRC_FN SubspaceCRC32C
#else
#define SUBSPACE_CRC_FN SubspaceCRC32
#endif

// The callback receives the data to be checksummed and a writable region where
// the checksum should be stored. The default CRC32 implementation writes 4 bytes;
// custom callbacks may use the full region.
using ChecksumCallback = std::function<void(const std::array<absl::Span<const uint8_t>, 3> &data,
                                            absl::Span<std::byte> checksum)>;

template <size_t N>
void CalculateCRC32Checksum(const std::array<absl::Span<const uint8_t>, N> &data,
                            absl::Span<std::byte> checksum) {
  uint32_t crc = 0xFFFFFFFF;
  for (size_t i = 0; i < N; i++) {
    crc = SUBSPACE_CRC_FN(crc, data[i].data(), data[i].size());
  }
  *reinterpret_cast<uint32_t *>(checksum.data()) = ~crc;
}

template <size_t N>
bool VerifyCRC32Checksum(const std::array<absl::Span<const uint8_t>, N> &data,
                         absl::Span<const std::byte> checksum) {
  uint32_t crc = 0xFFFFFFFF;
  for (size_t i = 0; i < N; i++) {
    crc = SUBSPACE_CRC_FN(crc, data[i].data(), data[i].size());
  }
  return *reinterpret_cast<const uint32_t *>(checksum.data()) == ~crc;
}

}  // namespace subspace
