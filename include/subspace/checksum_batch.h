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
#pragma once

#include <cstddef>
#include <cstdint>
#include <string>
#include <utility>
#include <vector>

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

// Per-message result of Verify (SUBSPACE_CRC_SLOT_* values).
enum class SlotCheck : uint32_t {
  kOk = SUBSPACE_CRC_SLOT_OK,                // checksum matched
  kMismatch = SUBSPACE_CRC_SLOT_MISMATCH,    // "Checksum verification failed"
  kUnchecked = SUBSPACE_CRC_SLOT_UNCHECKED,  // the publisher stored no checksum
};

inline constexpr const char* kChecksumVerificationFailed = "Checksum verification failed";

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

  // True when the device context exists (else every call returns its creation error).
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
#endif

  subspace_crc_ctx* context() const { return ctx_; }

 private:
  static const subspace_crc_slot* recs(const std::vector<ChecksumSlot>& s) {
    return reinterpret_cast<const subspace_crc_slot*>(s.data());
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
