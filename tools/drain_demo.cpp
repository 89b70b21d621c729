// Subscriber drain through include/subspace/checksum_batch.h:
// a host shared-memory channel (memfd, 64 slots of MessagePrefix 64 B + 4 KiB payload,
// stride 4,160, common/channel.h:88-112, client/client_channel.h:130-132) is published
// in one batch (BatchChecksum::Calculate), cross-checked slot by slot with the drop-in
// header's VerifyCRC32Checksum<3> on the host, then a drain of 48 slots in shuffled order
// (a subscriber's read order across wrap-around) with ragged delivered sizes is verified
// in one call (BatchChecksum::Verify / VerifyFlags) after two payload bytes and one prefix
// byte were corrupted and one slot's checksum flag was cleared.
//
// Exit 0 when every result matches the host templates; 77 when no device context can be
// created (a CPU-only machine: the error path is what gets checked there); 1 otherwise.
// Prints one JSON line.
//   g++ -O2 -std=c++17 -Iinclude tools/drain_demo.cpp -Lsubspace_amd -lsubspace_crc
#include <sys/mman.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "subspace/checksum.h"
#include "subspace/checksum_batch.h"

namespace {

constexpr int kSlots = 64;
constexpr size_t kPrefix = 64, kSlotSize = 4096, kStride = kPrefix + kSlotSize;
constexpr int32_t kChecksumSize = 4, kMetadataSize = 0;
constexpr int64_t kHasChecksum = 4;

std::array<absl::Span<const uint8_t>, 3> spans(const uint8_t* prefix, const uint8_t* payload, size_t size) {
  return {absl::Span<const uint8_t>(prefix + 4, 44), absl::Span<const uint8_t>(prefix + 52, 0),
          absl::Span<const uint8_t>(payload, size)};
}

}  // namespace

int main() {
  const int fd = memfd_create("subspace_drain_demo", 0);
  if (fd < 0 || ftruncate(fd, kSlots * kStride) != 0) {
    std::perror("memfd");
    return 1;
  }
  auto* chan = static_cast<uint8_t*>(mmap(nullptr, kSlots * kStride, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0));
  if (chan == MAP_FAILED) {
    std::perror("mmap");
    return 1;
  }
  subspace::BatchChecksum batch(0);
  if (!batch.ok()) {
    std::printf("{\"device\": false, \"error\": \"%s\"}\n", batch.error().c_str());
    return 77;
  }
  if (batch.RegisterBuffer(chan, kSlots * kStride) != SUBSPACE_CRC_OK) {
    std::printf("{\"device\": true, \"register_error\": \"%s\"}\n", batch.error().c_str());
    return 1;
  }

  // publish: payload bytes + prefix fields as client/publisher.cc:645-653 sets them
  uint64_t rng = 0x5EED00D1ull;
  auto next = [&]() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
  };
  std::vector<uint64_t> size(kSlots);
  std::vector<subspace::ChecksumSlot> pub;
  for (int i = 0; i < kSlots; i++) {
    uint8_t* prefix = chan + i * kStride;
    uint8_t* payload = prefix + kPrefix;
    size[i] = i == 5 ? 0 : 1 + next() % kSlotSize;  // ragged, one empty message
    for (size_t k = 0; k < kSlotSize; k++) payload[k] = (uint8_t)next();
    std::memset(prefix, 0, kPrefix);
    const int32_t slot_id = i, vchan = -1;
    const uint64_t ordinal = (uint64_t)i + 1, ts = 1000ull * i;
    const int64_t flags = 0;
    const uint16_t cs = kChecksumSize, ms = kMetadataSize;
    std::memcpy(prefix + 4, &slot_id, 4);
    std::memcpy(prefix + 8, &size[i], 8);
    std::memcpy(prefix + 16, &ordinal, 8);
    std::memcpy(prefix + 24, &ts, 8);
    std::memcpy(prefix + 32, &flags, 8);
    std::memcpy(prefix + 40, &vchan, 4);
    std::memcpy(prefix + 44, &cs, 2);
    std::memcpy(prefix + 46, &ms, 2);
    pub.push_back({prefix, payload, size[i]});
  }
  int failures = 0;
  if (batch.Calculate(pub, kSlotSize, kChecksumSize, kMetadataSize) != SUBSPACE_CRC_OK) {
    std::printf("{\"device\": true, \"calculate_error\": \"%s\"}\n", batch.error().c_str());
    return 1;
  }
  for (int i = 0; i < kSlots; i++) {  // every published slot verifies on the host
    const uint8_t* prefix = chan + i * kStride;
    int64_t flags;
    std::memcpy(&flags, prefix + 32, 8);
    const bool ok = subspace::VerifyCRC32Checksum<3>(
        spans(prefix, prefix + kPrefix, size[i]),
        absl::Span<const std::byte>(reinterpret_cast<const std::byte*>(prefix + 48), 4));
    failures += !ok || !(flags & kHasChecksum);
  }

  // corruptions (all in the drain below): payload bytes of slots 7 and 40, the ordinal of
  // slot 22, the flag of slot 33
  chan[7 * kStride + kPrefix + 3] ^= 0x01;
  chan[40 * kStride + kPrefix + size[40] - 1] ^= 0x80;
  chan[22 * kStride + 16] ^= 0x10;
  int64_t f33;
  std::memcpy(&f33, chan + 33 * kStride + 32, 8);
  f33 &= ~kHasChecksum;
  std::memcpy(chan + 33 * kStride + 32, &f33, 8);

  // drain: 48 slots in a subscriber's order (wrap-around from slot 30), truncated sizes
  // on a few (a delivered size smaller than the published one fails verification too)
  std::vector<subspace::ChecksumSlot> drain;
  std::vector<subspace::SlotCheck> expect;
  for (int k = 0; k < 48; k++) {
    const int i = (30 + 3 * k) % kSlots;
    uint8_t* prefix = chan + i * kStride;
    const uint64_t delivered = (k % 11 == 10 && size[i] > 1) ? size[i] - 1 : size[i];
    drain.push_back({prefix, prefix + kPrefix, delivered});
    int64_t flags;
    std::memcpy(&flags, prefix + 32, 8);
    const bool ok = subspace::VerifyCRC32Checksum<3>(
        spans(prefix, prefix + kPrefix, delivered),
        absl::Span<const std::byte>(reinterpret_cast<const std::byte*>(prefix + 48), 4));
    expect.push_back(!(flags & kHasChecksum) ? subspace::SlotCheck::kUnchecked
                     : ok                    ? subspace::SlotCheck::kOk
                                             : subspace::SlotCheck::kMismatch);
  }
  std::vector<subspace::SlotCheck> got;
  uint32_t mismatches = 0;
  if (batch.Verify(drain, kSlotSize, kChecksumSize, kMetadataSize, &got, &mismatches) != SUBSPACE_CRC_OK) {
    std::printf("{\"device\": true, \"verify_error\": \"%s\"}\n", batch.error().c_str());
    return 1;
  }
  uint32_t want_mismatches = 0, unchecked = 0;
  for (size_t k = 0; k < drain.size(); k++) {
    failures += got[k] != expect[k];
    want_mismatches += expect[k] == subspace::SlotCheck::kMismatch;
    unchecked += expect[k] == subspace::SlotCheck::kUnchecked;
  }
  failures += mismatches != want_mismatches;
  std::vector<bool> flags;
  if (batch.VerifyFlags(drain, kSlotSize, kChecksumSize, kMetadataSize, &flags) != SUBSPACE_CRC_OK) return 1;
  for (size_t k = 0; k < drain.size(); k++) failures += flags[k] != (expect[k] == subspace::SlotCheck::kMismatch);

  const int unreg = batch.UnregisterBuffer(chan);
  failures += unreg != SUBSPACE_CRC_OK;
  // a drain over memory that is no longer registered is rejected, not read
  const int rejected = batch.Verify(drain, kSlotSize, kChecksumSize, kMetadataSize, &got);
  failures += rejected == SUBSPACE_CRC_OK;
  std::printf("{\"device\": true, \"published\": %d, \"drained\": %zu, \"mismatches\": %u, \"expected_mismatches\": %u, "
              "\"unchecked\": %u, \"unregistered_rejected\": %s, \"failures\": %d}\n",
              kSlots, drain.size(), mismatches, want_mismatches, unchecked, rejected != SUBSPACE_CRC_OK ? "true" : "false",
              failures);
  munmap(chan, kSlots * kStride);
  close(fd);
  return failures ? 1 : 0;
}
