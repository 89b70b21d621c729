// The ValidateChecksum / publisher gates of include/subspace/checksum_batch.h
// (client/subscriber.h:264-275, client/publisher.cc:664-675), on three channels in one memfd:
//   A: CRC32 checksum, checksum_size 4, metadata 16 B  (the device path)
//   B: checksum_size 20 with the Checksum20Byte callback (client/client_test.cc:5210-5272:
//      5 CRC32s from seeds 0xFFFFFFFF ^ k*0x11111111), prefix 128 B (computed on the host)
//   C: checksums off (the publisher stores nothing; the subscriber reads nothing)
// Each channel is published through BatchChecksum::Calculate(slots, size, options), checked
// against the drop-in templates and the callback, corrupted, then drained in one mixed
// VerifyDrain call in a shuffled order; every result must equal what the reference's
// per-message ValidateChecksum would return.
//
//   batch_gates host  -- no device needed: channels B and C only, and a drain holding an A
//                        slot must fail cleanly (no context) on a CPU-only machine
//   batch_gates full  -- all three channels (needs the GPU for A)
// Exit 0 = pass, 1 = failure, 77 = `full` without a device. Prints one JSON line.
#include <sys/mman.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "subspace/checksum.h"
#include "subspace/checksum_batch.h"

namespace {

constexpr int kSlots = 40;
constexpr size_t kSlotSize = 1024;

struct Channel {
  subspace::ChecksumOptions opts;
  size_t prefix_size, stride;
  uint8_t* base;
  std::vector<uint64_t> size;
};

void checksum20(const std::array<absl::Span<const uint8_t>, 3>& data, absl::Span<std::byte> checksum) {
  auto* out = reinterpret_cast<uint32_t*>(checksum.data());
  for (int k = 0; k < 5; k++) {
    uint32_t crc = 0xFFFFFFFFu ^ static_cast<uint32_t>(k * 0x11111111);
    for (const auto& span : data) crc = subspace::SubspaceCRC32(crc, span.data(), span.size());
    out[k] = ~crc;
  }
}

// What the reference's subscriber returns for one slot (client/client.cc:1346-1356 with
// ValidateChecksum): unchecked without the flag, else the gate of the subscriber's options.
subspace::SlotCheck expected(const Channel& ch, const uint8_t* prefix, const uint8_t* payload, uint64_t size) {
  if (!ch.opts.checksum) return subspace::SlotCheck::kSkipped;
  if (!subspace::PrefixHasChecksum(prefix)) return subspace::SlotCheck::kUnchecked;
  auto data = subspace::MessageChecksumData(prefix, payload, size, ch.opts.checksum_size, ch.opts.metadata_size);
  bool ok;
  if (ch.opts.callback) {
    std::vector<std::byte> tmp(static_cast<size_t>(ch.opts.checksum_size));
    ch.opts.callback(data, absl::Span<std::byte>(tmp.data(), tmp.size()));
    ok = std::memcmp(tmp.data(), prefix + 48, tmp.size()) == 0;
  } else {
    ok = subspace::VerifyCRC32Checksum<3>(data, absl::Span<const std::byte>(
                                                    reinterpret_cast<const std::byte*>(prefix + 48), 4));
  }
  return ok ? subspace::SlotCheck::kOk : subspace::SlotCheck::kMismatch;
}

}  // namespace

int main(int argc, char** argv) {
  const bool full = argc > 1 && std::string(argv[1]) == "full";
  subspace::BatchChecksum batch(0);
  if (full && !batch.ok()) {
    std::printf("{\"device\": false, \"error\": \"%s\"}\n", batch.error().c_str());
    return 77;
  }
  Channel ch[3];
  ch[0].opts.checksum_size = 4;
  ch[0].opts.metadata_size = 16;
  ch[1].opts.checksum_size = 20;
  ch[1].opts.callback = checksum20;
  ch[2].opts.checksum = false;
  size_t total = 0;
  for (auto& c : ch) {
    c.prefix_size = (48 + c.opts.checksum_size + c.opts.metadata_size + 63) & ~size_t(63);  // ComputePrefixSize
    c.stride = c.prefix_size + kSlotSize;
    total += c.stride * kSlots;
  }
  const int fd = memfd_create("subspace_batch_gates", 0);
  if (fd < 0 || ftruncate(fd, (off_t)total) != 0) return 1;
  auto* mem = static_cast<uint8_t*>(mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0));
  if (mem == MAP_FAILED) return 1;
  if (full && batch.RegisterBuffer(mem, total) != SUBSPACE_CRC_OK) {
    std::printf("{\"register_error\": \"%s\"}\n", batch.error().c_str());
    return 1;
  }
  uint64_t rng = 0x6A7E5ull;
  auto next = [&]() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
  };
  int failures = 0;
  size_t off = 0;
  for (int c = 0; c < 3; c++) {
    Channel& h = ch[c];
    h.base = mem + off;
    off += h.stride * kSlots;
    if (c == 0 && !full) continue;  // the CRC32 channel needs the device
    std::vector<subspace::ChecksumSlot> pub;
    for (int i = 0; i < kSlots; i++) {
      uint8_t* prefix = h.base + i * h.stride;
      uint8_t* payload = prefix + h.prefix_size;
      h.size.push_back(i == 3 ? 0 : 1 + next() % kSlotSize);
      for (size_t k = 0; k < h.prefix_size + kSlotSize; k++) prefix[k] = (uint8_t)next();
      const int64_t flags = 0;
      std::memcpy(prefix + 32, &flags, 8);  // no kMessageHasChecksum before the publish
      pub.push_back({prefix, payload, h.size.back()});
    }
    if (batch.Calculate(pub, kSlotSize, h.opts) != SUBSPACE_CRC_OK) {
      std::printf("{\"calculate_error\": \"%s\", \"channel\": %d}\n", batch.error().c_str(), c);
      return 1;
    }
    for (int i = 0; i < kSlots; i++) {  // the publisher's gate: flag and checksum, or neither
      const uint8_t* prefix = h.base + i * h.stride;
      const bool flagged = subspace::PrefixHasChecksum(prefix);
      if (flagged != h.opts.checksum) failures++;
      if (h.opts.checksum && expected(h, prefix, prefix + h.prefix_size, h.size[i]) != subspace::SlotCheck::kOk)
        failures++;
    }
  }
  // corruptions: payload, span 0 and a checksum byte past the first 4 (only a full-width
  // compare sees it: the callback channel), a flag cleared
  auto corrupt = [&](int c, int i, size_t at) { ch[c].base[i * ch[c].stride + at] ^= 0x20; };
  for (int c = full ? 0 : 1; c < 3; c++) {
    corrupt(c, 7, ch[c].prefix_size);       // payload byte 0
    corrupt(c, 11, 20);                    // span 0 (prefix[4, 48))
    corrupt(c, 13, 48 + 17 % ch[c].opts.checksum_size);  // checksum byte 17 (c = B), byte 1 (A)
    int64_t f;
    std::memcpy(&f, ch[c].base + 21 * ch[c].stride + 32, 8);
    f &= ~subspace::kMessageHasChecksumFlag;
    std::memcpy(ch[c].base + 21 * ch[c].stride + 32, &f, 8);
  }
  // the mixed drain, interleaved over the channels
  std::vector<subspace::ChecksumSlot> drain;
  std::vector<uint32_t> chan_of;
  std::vector<subspace::SlotCheck> want;
  for (int k = 0; k < kSlots; k++) {
    for (int c = full ? 0 : 1; c < 3; c++) {
      const int i = (k * 7 + c) % kSlots;
      const uint8_t* prefix = ch[c].base + i * ch[c].stride;
      drain.push_back({prefix, prefix + ch[c].prefix_size, ch[c].size[i]});
      chan_of.push_back((uint32_t)c);
      want.push_back(expected(ch[c], prefix, prefix + ch[c].prefix_size, ch[c].size[i]));
    }
  }
  std::vector<subspace::ChecksumOptions> opts = {ch[0].opts, ch[1].opts, ch[2].opts};
  std::vector<subspace::SlotCheck> got;
  uint32_t mism = 0, want_mism = 0, skipped = 0, cb_mism = 0;
  const int rc = batch.VerifyDrain(drain, chan_of, opts, kSlotSize, &got, &mism);
  if (rc != SUBSPACE_CRC_OK) {
    std::printf("{\"verify_error\": \"%s\"}\n", batch.error().c_str());
    return 1;
  }
  for (size_t k = 0; k < drain.size(); k++) {
    failures += got[k] != want[k];
    want_mism += want[k] == subspace::SlotCheck::kMismatch;
    skipped += want[k] == subspace::SlotCheck::kSkipped;
    cb_mism += chan_of[k] == 1 && want[k] == subspace::SlotCheck::kMismatch;
  }
  failures += mism != want_mism;
  failures += cb_mism != 3;  // slots 7, 11 and 13 of channel B (byte 17 of its 20-B checksum)
  int no_device_rc = 0;
  if (!full && !batch.ok()) {
    // a CRC32 slot in the drain needs the device: a clean error, not a crash
    std::vector<subspace::ChecksumSlot> one = {drain[0]};
    std::vector<uint32_t> c0 = {0};
    no_device_rc = batch.VerifyDrain(one, c0, opts, kSlotSize, &got);
    failures += no_device_rc == SUBSPACE_CRC_OK;
  }
  // bad span sizes on the callback forms fail like the device path's (EINVAL), never throw
  // (a negative checksum_size once became a huge scratch vector: ADVICE r03)
  int bad_args = 0;
  {
    subspace::ChecksumOptions neg = ch[1].opts, small = ch[1].opts, negmeta = ch[1].opts;
    neg.checksum_size = -1;
    small.checksum_size = 3;
    negmeta.metadata_size = -5;
    std::vector<subspace::ChecksumSlot> one = {drain[0]};
    std::vector<uint32_t> c0 = {0};
    for (const subspace::ChecksumOptions& o : {neg, small, negmeta}) {
      bad_args += batch.Verify(one, kSlotSize, o, &got) == SUBSPACE_CRC_EINVAL;
      bad_args += batch.Calculate(one, kSlotSize, o) == SUBSPACE_CRC_EINVAL;
      std::vector<subspace::ChecksumOptions> o1 = {o};
      bad_args += batch.VerifyDrain(one, c0, o1, kSlotSize, &got) == SUBSPACE_CRC_EINVAL;
    }
    failures += bad_args != 9;
  }
  std::printf("{\"mode\": \"%s\", \"drained\": %zu, \"mismatches\": %u, \"expected_mismatches\": %u, "
              "\"callback_mismatches\": %u, \"skipped\": %u, \"no_device_rc\": %d, \"bad_args_einval\": %d, "
              "\"failures\": %d}\n",
              full ? "full" : "host", drain.size(), mism, want_mism, cb_mism, skipped, no_device_rc, bad_args, failures);
  if (full) batch.UnregisterBuffer(mem);
  munmap(mem, total);
  close(fd);
  return failures ? 1 : 0;
}
