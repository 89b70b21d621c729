// Config A (BASELINE.json configs[0]): the reference's per-message CPU path, 1 publisher x
// 1 subscriber, 4 KiB messages, checksums on -- per-message publish-checksum + verify
// latency in the reference's slot layout (client/latency_test.cc:577-608 shape).
//
// A channel of 16 slots (MessagePrefix 64 B + 4 KiB payload, stride 4,160, common/channel.h
// :88-112, client/client_channel.h:130-132) lives in a shared memory mapping (memfd, as
// the reference maps channels). For each of N messages the publisher writes the payload,
// fills the prefix as client/publisher.cc:645-653 does and calls CalculateCRC32Checksum<3>
// over GetMessageChecksumData's spans (publisher.cc:664-675); the subscriber then runs
// VerifyCRC32Checksum<3> (client/client.cc:1346-1356). calc + verify is timed per message.
//
// Two legs over identical messages:
//   "dropin":    include/subspace/checksum.h templates + libsubspace_crc.so's SubspaceCRC32
//                (slice-by-16, the product host path);
//   "reference": the same templates' chain over oracle/liboracle_crc.so's byte-table
//                restatement of client/checksum.cc:125-130 (the CPU baseline; dlopen'ed).
// Prints one JSON line: p50/p99/mean ns per message for each leg. Not a GPU program.
//   usage: tools/config_a [messages]   (default 20,000)
#include <dlfcn.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "subspace/checksum.h"

namespace {

constexpr int kSlots = 16;
constexpr size_t kPrefix = 64, kPayload = 4096, kStride = kPrefix + kPayload;

using CrcFn = uint32_t (*)(uint32_t, const uint8_t*, size_t);

// GetMessageChecksumData (common/channel.h:527-542), checksum_size 4, metadata_size 0.
std::array<absl::Span<const uint8_t>, 3> spans(const uint8_t* prefix, const uint8_t* payload, size_t size) {
  return {absl::Span<const uint8_t>(prefix + 4, 44), absl::Span<const uint8_t>(prefix + 52, 0),
          absl::Span<const uint8_t>(payload, size)};
}

uint32_t chain(CrcFn fn, const std::array<absl::Span<const uint8_t>, 3>& d) {
  uint32_t crc = 0xFFFFFFFFu;
  for (const auto& s : d) crc = fn(crc, s.data(), s.size());
  return ~crc;
}

struct Stats {
  double p50, p99, mean;
};

Stats stats(std::vector<double>& ns) {
  std::sort(ns.begin(), ns.end());
  double sum = 0;
  for (double x : ns) sum += x;
  return {ns[ns.size() / 2], ns[(size_t)(ns.size() * 0.99)], sum / (double)ns.size()};
}

}  // namespace

int main(int argc, char** argv) {
  const size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 20000;
  const int fd = memfd_create("subspace_config_a", 0);
  if (fd < 0 || ftruncate(fd, kSlots * kStride) != 0) {
    std::perror("memfd");
    return 1;
  }
  auto* chan = static_cast<uint8_t*>(mmap(nullptr, kSlots * kStride, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0));
  if (chan == MAP_FAILED) {
    std::perror("mmap");
    return 1;
  }
  std::string ora = argc > 2 ? argv[2] : "oracle/liboracle_crc.so";
  void* h = dlopen(ora.c_str(), RTLD_NOW | RTLD_LOCAL);
  CrcFn ref = h ? reinterpret_cast<CrcFn>(dlsym(h, "oracle_crc32")) : nullptr;

  uint64_t rng = 0x5EED000Aull;
  auto next = [&]() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
  };
  std::vector<double> t_drop(n), t_ref(n);
  size_t failures = 0;
  for (size_t i = 0; i < n; i++) {
    uint8_t* prefix = chan + (i % kSlots) * kStride;
    uint8_t* payload = prefix + kPrefix;
    for (size_t k = 0; k < kPayload; k += 8) {
      const uint64_t v = next();
      std::memcpy(payload + k, &v, 8);
    }
    // publisher.cc:645-653: message_size, ordinal, timestamp, vchan, sizes, flags, slot_id
    const int32_t slot_id = (int32_t)(i % kSlots);
    const uint64_t size = kPayload, ordinal = i + 1, ts = 1000000ull * i;
    const int64_t flags = 4;  // SetHasChecksum (kMessageHasChecksum)
    const int32_t vchan = -1;
    const uint16_t cs = 4, ms = 0;
    std::memcpy(prefix + 4, &slot_id, 4);
    std::memcpy(prefix + 8, &size, 8);
    std::memcpy(prefix + 16, &ordinal, 8);
    std::memcpy(prefix + 24, &ts, 8);
    std::memcpy(prefix + 32, &flags, 8);
    std::memcpy(prefix + 40, &vchan, 4);
    std::memcpy(prefix + 44, &cs, 2);
    std::memcpy(prefix + 46, &ms, 2);

    const auto d = spans(prefix, payload, kPayload);
    auto t0 = std::chrono::steady_clock::now();
    subspace::CalculateCRC32Checksum<3>(d, absl::Span<std::byte>(reinterpret_cast<std::byte*>(prefix + 48), 4));
    const bool ok = subspace::VerifyCRC32Checksum<3>(
        d, absl::Span<const std::byte>(reinterpret_cast<const std::byte*>(prefix + 48), 4));
    auto t1 = std::chrono::steady_clock::now();
    t_drop[i] = std::chrono::duration<double, std::nano>(t1 - t0).count();
    failures += !ok;
    if (ref) {
      uint32_t stored;
      t0 = std::chrono::steady_clock::now();
      const uint32_t c = chain(ref, d);  // publish: compute + store
      std::memcpy(prefix + 48, &c, 4);
      std::memcpy(&stored, prefix + 48, 4);
      const bool ok2 = stored == chain(ref, d);  // subscribe: verify
      t1 = std::chrono::steady_clock::now();
      t_ref[i] = std::chrono::duration<double, std::nano>(t1 - t0).count();
      failures += !ok2;
    }
  }
  const Stats a = stats(t_drop);
  std::printf("{\"config\": \"A: 1 pub x 1 sub, 4 KiB messages, checksum on, calc+verify per message\", "
              "\"messages\": %zu, \"failures\": %zu, \"dropin\": {\"p50_ns\": %.0f, \"p99_ns\": %.0f, \"mean_ns\": %.0f}",
              n, failures, a.p50, a.p99, a.mean);
  if (ref) {
    const Stats b = stats(t_ref);
    std::printf(", \"reference\": {\"p50_ns\": %.0f, \"p99_ns\": %.0f, \"mean_ns\": %.0f}", b.p50, b.p99, b.mean);
  }
  std::printf("}\n");
  munmap(chan, kSlots * kStride);
  close(fd);
  return failures ? 2 : 0;
}
