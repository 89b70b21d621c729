// Header-only C++ helper over the batched slot calls of include/subspace_crc.h: what a
// dallison/subspace client would use at its bulk boundaries instead of one host CRC per
// message.
//
//   - Verify: the subscriber drain (GetAllMessages / ProcessAllMessages,
//     client/client.cc:344-397; per-message verify at :1346-1356). One call checks every
//     drained slot; a mismatch is reported per message, in the two forms the reference
//     uses (client/client.cc:1447-1452): the Message::checksum_error flag
//     (client/message.h:85, :209) when the subscriber passes checksum errors through, else
//     absl::InternalError("Checksum verification failed").
//   - Calculate: a batch of published slots (client/publisher.cc:664-675): sets
//     kMessageHasChecksum and stores ~crc in every prefix.
//
// Slots live in host shared memory (the channel mapping, client/client_channel.h:122-172,
// or split buffers, common/split_buffer.h:43-55). Register each mapping once
// (RegisterBuffer); the GPU then reads prefixes and payloads in place over PCIe
// (subspace_crc32_host_slot_list). Calls are synchronous. One BatchChecksum per thread
// (like the C context it owns).
//
// Error handling follows the C ABI: methods return SUBSPACE_CRC_OK or a negative code and
// never throw; error() holds the library's message for the last failure.
//
// Gates (client/subscriber.h:264-275 ValidateChecksum, client/publisher.cc:664-675): a channel
// endpoint's ChecksumOptions decide what a slot gets, exactly as the reference decides per
// message:
//   - checksum off: the publisher sets no flag and stores nothing; the subscriber's
//     ValidateChecksum returns true without reading the slot (SlotCheck::kSkipped, no device
//     or host read);
//   - a ChecksumCallback (e.g. the 20-byte Checksum20Byte seed chain, client/client_test.cc:
//     5210-5272, or an AES-CMAC): computed by the callback on the host, over the same three
//     spans, and compared on the full checksum_size bytes with memcmp -- the device path only
//     computes the CRC32 checksum, so callback channels never reach it;
//   - otherwise the CRC32 checksum on the device (VerifyCRC32Checksum / CalculateCRC32Checksum).
// VerifyDrain takes a mixed drain (slots of several channels with different options) and
// routes each slot accordingly: one device call per (checksum_size, metadata_size) group of
// CRC32 slots, the callback slots on the host, checksum-off slots not at all.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "subspace/checksum.h"
#include "subspace_crc.h"

#if __has_include("absl/status/status.h")
#include "absl/status/status.h"
#define SUBSPACE_CRC_HAVE_ABSL_STATUS 1
#endif

namespace subspace {

// One drained or published message: its MessagePrefix, its payload and the payload size
// (the delivered size at read, slot->message_size at publish).
struct ChecksumSlot {
  const void* prefix;
  const void* payload;
  uint64_t message_size;
};
static_assert(sizeof(ChecksumSlot) == sizeof(subspace_crc_slot), "ChecksumSlot mirrors subspace_crc_slot");

// Per-message result of Verify (SUBSPACE_CRC_SLOT_* values, and kSkipped).
enum class SlotCheck : uint32_t {
  kOk = SUBSPACE_CRC_SLOT_OK,                // checksum matched
  kMismatch = SUBSPACE_CRC_SLOT_MISMATCH,    // "Checksum verification failed"
  kUnchecked = SUBSPACE_CRC_SLOT_UNCHECKED,  // the publisher stored no checksum
  kSkipped = 3u,                             // the subscriber has checksums off: valid, not read
};
static_assert(SUBSPACE_CRC_SLOT_OVERSIZE != 3u, "kSkipped is not a library status");

inline constexpr const char* kChecksumVerificationFailed = "Checksum verification failed";

// The checksum configuration of one channel endpoint as the reference keeps it:
// options_.Checksum(), ChecksumSize(), MetadataSize() (client/options.h) and the callback set
// with SetChecksumCallback (publisher and subscriber).
struct ChecksumOptions {
  bool checksum = true;
  int32_t checksum_size = 4;
  int32_t metadata_size = 0;
  ChecksumCallback callback;  // empty: the CRC32 checksum (the batched device path)
};

// MessagePrefix fields the gates read (common/channel.h:88-112): flags at offset 32 (int64),
// kMessageHasChecksum = 4; the checksum area at 48.
inline constexpr int64_t kMessageHasChecksumFlag = 4;
inline bool PrefixHasChecksum(const void* prefix) {
  int64_t flags;
  std::memcpy(&flags, static_cast<const uint8_t*>(prefix) + 32, sizeof(flags));
  return (flags & kMessageHasChecksumFlag) != 0;
}
inline void PrefixSetHasChecksum(void* prefix) {
  int64_t flags;
  std::memcpy(&flags, static_cast<uint8_t*>(prefix) + 32, sizeof(flags));
  flags |= kMessageHasChecksumFlag;
  std::memcpy(static_cast<uint8_t*>(prefix) + 32, &flags, sizeof(flags));
}

// GetMessageChecksumData (common/channel.h:527-542): span 0 = prefix[4, 48), span 1 = the
// metadata after the checksum area, span 2 = the payload.
inline std::array<absl::Span<const uint8_t>, 3> MessageChecksumData(const void* prefix, const void* payload,
                                                                    uint64_t size, int32_t checksum_size,
                                                                    int32_t metadata_size) {
  const auto* p = static_cast<const uint8_t*>(prefix);
  return {absl::Span<const uint8_t>(p + 4, 44),
          absl::Span<const uint8_t>(p + 48 + checksum_size, static_cast<size_t>(metadata_size)),
          absl::Span<const uint8_t>(static_cast<const uint8_t*>(payload), static_cast<size_t>(size))};
}

class BatchChecksum {
 public:
  // A context on HIP device `device` for one reflected polynomial (IEEE: the reference's
  // default builds; SUBSPACE_CRC_POLY_CASTAGNOLI: its -msse4.2 builds).
  explicit BatchChecksum(int device = 0, uint32_t reflected_poly = SUBSPACE_CRC_POLY_IEEE) {
    rc_ = subspace_crc_ctx_create_poly(device, reflected_poly, &ctx_);
    if (rc_ != SUBSPACE_CRC_OK) {
      ctx_ = nullptr;
      error_ = subspace_crc_last_error();
    }
  }
  ~BatchChecksum() {
    for (void* p : registered_) subspace_crc_host_unregister(p);
    if (ctx_) subspace_crc_ctx_destroy(ctx_);
  }
  BatchChecksum(const BatchChecksum&) = delete;
  BatchChecksum& operator=(const BatchChecksum&) = delete;
  BatchChecksum(BatchChecksum&& o) noexcept
      : ctx_(std::exchange(o.ctx_, nullptr)), rc_(o.rc_), error_(std::move(o.error_)),
        registered_(std::move(o.registered_)) {
    o.registered_.clear();
  }

  // True when the device context exists (else every call that needs the device returns its
  // creation error; checksum-off and callback slots need none).
  bool ok() const { return ctx_ != nullptr; }
  const std::string& error() const { return error_; }

  // Pin and device-map a channel (or split-buffer) mapping once; it is unregistered by
  // UnregisterBuffer or the destructor (call before munmap).
  int RegisterBuffer(void* addr, size_t bytes) {
    if (!ok()) return rc_;
    const int rc = subspace_crc_host_register(addr, bytes);
    if (rc != SUBSPACE_CRC_OK) return fail(rc);
    registered_.push_back(addr);
    return SUBSPACE_CRC_OK;
  }
  int UnregisterBuffer(void* addr) {
    for (size_t i = 0; i < registered_.size(); i++) {
      if (registered_[i] == addr) {
        registered_.erase(registered_.begin() + (long)i);
        const int rc = subspace_crc_host_unregister(addr);
        return rc == SUBSPACE_CRC_OK ? rc : fail(rc);
      }
    }
    error_ = "buffer was not registered by this BatchChecksum";
    return SUBSPACE_CRC_EINVAL;
  }

  // Subscriber drain: checks every slot (VerifyCRC32Checksum<3> over the spans of
  // GetMessageChecksumData, common/channel.h:527-542). results (resized to slots.size())
  // gets one SlotCheck per slot; *mismatches (optional) the number of kMismatch.
  // max_message_size is the channel's slot size (a larger message is still handled).
  int Verify(const std::vector<ChecksumSlot>& slots, uint64_t max_message_size, int32_t checksum_size,
             int32_t metadata_size, std::vector<SlotCheck>* results, uint32_t* mismatches = nullptr) {
    if (!ok()) return rc_;
    std::vector<uint32_t> status(slots.size());
    uint32_t errors = 0;
    const int rc = subspace_crc32_host_slot_list(ctx_, recs(slots), slots.size(), max_message_size, checksum_size,
                                                 metadata_size, SUBSPACE_CRC_SLOT_VERIFY, status.data(), &errors);
    if (rc != SUBSPACE_CRC_OK) return fail(rc);
    if (results) {
      results->resize(slots.size());
      for (size_t i = 0; i < slots.size(); i++) (*results)[i] = static_cast<SlotCheck>(status[i]);
    }
    if (mismatches) *mismatches = errors;
    return SUBSPACE_CRC_OK;
  }

  // The Message::checksum_error flags of a drain (pass_checksum_errors subscribers,
  // client/client.cc:1449-1451): flags[i] is true for a mismatching slot.
  int VerifyFlags(const std::vector<ChecksumSlot>& slots, uint64_t max_message_size, int32_t checksum_size,
                  int32_t metadata_size, std::vector<bool>* flags) {
    std::vector<SlotCheck> r;
    const int rc = Verify(slots, max_message_size, checksum_size, metadata_size, &r);
    if (rc != SUBSPACE_CRC_OK) return rc;
    flags->assign(slots.size(), false);
    for (size_t i = 0; i < r.size(); i++) (*flags)[i] = r[i] == SlotCheck::kMismatch;
    return SUBSPACE_CRC_OK;
  }

  // Publisher batch: sets kMessageHasChecksum in every prefix and stores its checksum
  // (CalculateCRC32Checksum<3>'s result) at prefix + 48.
  int Calculate(const std::vector<ChecksumSlot>& slots, uint64_t max_message_size, int32_t checksum_size,
                int32_t metadata_size) {
    if (!ok()) return rc_;
    const int rc = subspace_crc32_host_slot_list(ctx_, recs(slots), slots.size(), max_message_size, checksum_size,
                                                 metadata_size, SUBSPACE_CRC_SLOT_CALCULATE, nullptr, nullptr);
    return rc == SUBSPACE_CRC_OK ? rc : fail(rc);
  }

  // --- gated forms: one channel endpoint's ChecksumOptions (see the top of this file) ---

  // Subscriber drain of one channel: ValidateChecksum per slot, for every slot whose prefix
  // has kMessageHasChecksum (client/client.cc:1346-1356); slots without it are kUnchecked.
  int Verify(const std::vector<ChecksumSlot>& slots, uint64_t max_message_size, const ChecksumOptions& opts,
             std::vector<SlotCheck>* results, uint32_t* mismatches = nullptr) {
    if (const int rc = check_options(opts)) return rc;
    if (!opts.checksum) {  // ValidateChecksum: options_.Checksum() false -> true, nothing read
      if (results) results->assign(slots.size(), SlotCheck::kSkipped);
      if (mismatches) *mismatches = 0;
      return SUBSPACE_CRC_OK;
    }
    if (!opts.callback) return Verify(slots, max_message_size, opts.checksum_size, opts.metadata_size, results, mismatches);
    if (results) results->resize(slots.size());
    uint32_t bad = 0;
    std::vector<std::byte> tmp(static_cast<size_t>(opts.checksum_size));
    for (size_t i = 0; i < slots.size(); i++) {
      const ChecksumSlot& s = slots[i];
      SlotCheck r = SlotCheck::kUnchecked;
      if (PrefixHasChecksum(s.prefix)) {
        // the callback writes into a scratch span of checksum.size() bytes, then memcmp over
        // all of them (client/subscriber.h:269-273)
        opts.callback(MessageChecksumData(s.prefix, s.payload, s.message_size, opts.checksum_size, opts.metadata_size),
                      absl::Span<std::byte>(tmp.data(), tmp.size()));
        const bool same = std::memcmp(tmp.data(), static_cast<const uint8_t*>(s.prefix) + 48, tmp.size()) == 0;
        r = same ? SlotCheck::kOk : SlotCheck::kMismatch;
      }
      bad += r == SlotCheck::kMismatch;
      if (results) (*results)[i] = r;
    }
    if (mismatches) *mismatches = bad;
    return SUBSPACE_CRC_OK;
  }

  // Publisher batch of one channel (client/publisher.cc:664-675): nothing with checksums off;
  // else SetHasChecksum() and the callback's or the CRC32 checksum into the checksum area.
  int Calculate(const std::vector<ChecksumSlot>& slots, uint64_t max_message_size, const ChecksumOptions& opts) {
    if (const int rc = check_options(opts)) return rc;
    if (!opts.checksum) return SUBSPACE_CRC_OK;
    if (!opts.callback) return Calculate(slots, max_message_size, opts.checksum_size, opts.metadata_size);
    for (const ChecksumSlot& s : slots) {
      void* prefix = const_cast<void*>(s.prefix);
      PrefixSetHasChecksum(prefix);
      opts.callback(MessageChecksumData(prefix, s.payload, s.message_size, opts.checksum_size, opts.metadata_size),
                    absl::Span<std::byte>(reinterpret_cast<std::byte*>(static_cast<uint8_t*>(prefix) + 48),
                                          static_cast<size_t>(opts.checksum_size)));
    }
    return SUBSPACE_CRC_OK;
  }

  // A mixed drain: slot i belongs to channel endpoint channel_of[i] (an index into
  // `channels`). Checksum-off slots are kSkipped, callback slots are checked on the host,
  // and the CRC32 slots go to the device in one call per (checksum_size, metadata_size).
  // results (resized to slots.size()) and *mismatches (optional) cover the whole drain.
  int VerifyDrain(const std::vector<ChecksumSlot>& slots, const std::vector<uint32_t>& channel_of,
                  const std::vector<ChecksumOptions>& channels, uint64_t max_message_size,
                  std::vector<SlotCheck>* results, uint32_t* mismatches = nullptr) {
    if (channel_of.size() != slots.size()) {
      error_ = "channel_of must name one channel per slot";
      return SUBSPACE_CRC_EINVAL;
    }
    for (uint32_t c : channel_of)
      if (c >= channels.size()) {
        error_ = "channel index out of range";
        return SUBSPACE_CRC_EINVAL;
      }
    for (const ChecksumOptions& o : channels)
      if (const int rc = check_options(o)) return rc;
    std::vector<SlotCheck> out(slots.size(), SlotCheck::kSkipped);
    uint32_t bad = 0;
    // group the slots: by channel for callbacks (each has its own callback), by span shape
    // for the device
    std::map<std::pair<int32_t, int32_t>, std::vector<size_t>> crc_groups;
    std::map<uint32_t, std::vector<size_t>> cb_groups;
    for (size_t i = 0; i < slots.size(); i++) {
      const ChecksumOptions& o = channels[channel_of[i]];
      if (!o.checksum) continue;
      if (o.callback) cb_groups[channel_of[i]].push_back(i);
      else crc_groups[{o.checksum_size, o.metadata_size}].push_back(i);
    }
    auto run = [&](const std::vector<size_t>& idx, const ChecksumOptions& o) {
      std::vector<ChecksumSlot> sub;
      sub.reserve(idx.size());
      for (size_t i : idx) sub.push_back(slots[i]);
      std::vector<SlotCheck> r;
      uint32_t nb = 0;
      const int rc = Verify(sub, max_message_size, o, &r, &nb);
      if (rc != SUBSPACE_CRC_OK) return rc;
      for (size_t k = 0; k < idx.size(); k++) out[idx[k]] = r[k];
      bad += nb;
      return SUBSPACE_CRC_OK;
    };
    for (const auto& g : cb_groups) {
      const int rc = run(g.second, channels[g.first]);
      if (rc != SUBSPACE_CRC_OK) return rc;
    }
    for (const auto& g : crc_groups) {
      ChecksumOptions o;
      o.checksum_size = g.first.first;
      o.metadata_size = g.first.second;
      const int rc = run(g.second, o);
      if (rc != SUBSPACE_CRC_OK) return rc;
    }
    if (results) *results = std::move(out);
    if (mismatches) *mismatches = bad;
    return SUBSPACE_CRC_OK;
  }

#ifdef SUBSPACE_CRC_HAVE_ABSL_STATUS
  // Strict subscribers (no pass_checksum_errors): the first mismatch becomes the error the
  // reference returns from ReadMessage (client/client.cc:1447-1448).
  absl::Status VerifyStatus(const std::vector<ChecksumSlot>& slots, uint64_t max_message_size,
                            int32_t checksum_size, int32_t metadata_size) {
    uint32_t bad = 0;
    const int rc = Verify(slots, max_message_size, checksum_size, metadata_size, nullptr, &bad);
    if (rc != SUBSPACE_CRC_OK) return absl::InternalError(error_);
    return bad ? absl::InternalError(kChecksumVerificationFailed) : absl::OkStatus();
  }
  absl::Status VerifyStatus(const std::vector<ChecksumSlot>& slots, uint64_t max_message_size,
                            const ChecksumOptions& opts) {
    uint32_t bad = 0;
    const int rc = Verify(slots, max_message_size, opts, nullptr, &bad);
    if (rc != SUBSPACE_CRC_OK) return absl::InternalError(error_);
    return bad ? absl::InternalError(kChecksumVerificationFailed) : absl::OkStatus();
  }
#endif

  subspace_crc_ctx* context() const { return ctx_; }

 private:
  static const subspace_crc_slot* recs(const std::vector<ChecksumSlot>& s) {
    return reinterpret_cast<const subspace_crc_slot*>(s.data());
  }
  // The device path's argument rules (capi.hip check_slot_args) for every gated form, so a
  // callback channel with a bad size fails the same way instead of throwing (a negative size
  // as a vector length) or passing silently.
  int check_options(const ChecksumOptions& o) {
    if (o.checksum_size < 4) {
      error_ = "checksum_size < 4";
      return SUBSPACE_CRC_EINVAL;
    }
    if (o.metadata_size < 0) {
      error_ = "metadata_size < 0";
      return SUBSPACE_CRC_EINVAL;
    }
    return SUBSPACE_CRC_OK;
  }

  int fail(int rc) {
    error_ = subspace_crc_last_error();
    return rc;
  }

  subspace_crc_ctx* ctx_ = nullptr;
  int rc_ = SUBSPACE_CRC_OK;
  std::string error_;
  std::vector<void*> registered_;
};

}  // namespace subspace
