/*
 * subspace_crc.h -- C ABI of libsubspace_crc.so: the MI355X batched CRC32 path.
 *
 * Boundary (reference paths relative to dallison/subspace):
 *   SubspaceCRC32            replaces client/checksum.cc:125-130 (and declares the
 *                            same symbol as client/checksum.h:18-20). Host code,
 *                            per-message, bit-exact IEEE (0xEDB88320, raw state).
 *   subspace_crc32_batch*    NEW batch entry points. Each computes, for every message
 *                            i of a device-resident batch, exactly
 *                              out[i] = SubspaceCRC32(init, msg_i, len_i)
 *                            (or its complement with SUBSPACE_CRC_FINALIZE, i.e. the
 *                            value CalculateCRC32Checksum stores, client/checksum.h:36).
 *                            They are what a batched publish (client/publisher.cc:664-675)
 *                            or a bulk subscriber drain (client/client.cc:344-397,
 *                            verify at :1346-1356) would call instead of one host CRC
 *                            per message. Stream-ordered, asynchronous, int status.
 *
 * Conventions: plain pointers and sizes only; device pointers are HIP device memory
 * on the context's device; `stream` is a hipStream_t (NULL = default stream). Calls
 * return SUBSPACE_CRC_OK or a negative code, never throw, and set a thread-local
 * message readable with subspace_crc_last_error(). A context serialises its own calls
 * (a mutex on the host; a call on another stream than the previous call's first waits
 * for that stream's work, so the context's device workspaces are never shared by two
 * calls in flight); distinct contexts are independent.
 */
#ifndef SUBSPACE_CRC_H_
#define SUBSPACE_CRC_H_

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SUBSPACE_CRC_OK 0
#define SUBSPACE_CRC_EINVAL (-1)  /* bad argument (null pointer, misaligned stride, ...) */
#define SUBSPACE_CRC_EHIP (-2)    /* a HIP runtime call failed */
#define SUBSPACE_CRC_ENOMEM (-3)  /* device workspace allocation failed */
#define SUBSPACE_CRC_ENODEV (-4)  /* no usable gfx950 device */
#define SUBSPACE_CRC_EFAULT (-5)  /* a kernel of an earlier call on the context gave up a bounded wait
                                     (stale device state or calls racing on one context): its
                                     results are not valid (subspace_crc_ctx_check) */

/* flags */
#define SUBSPACE_CRC_FINALIZE 0x1u /* store ~crc (the stored checksum) instead of the raw state */

typedef struct subspace_crc_ctx subspace_crc_ctx;

/* Reference-compatible host CRC (client/checksum.h:18-20). */
uint32_t SubspaceCRC32(uint32_t crc, const uint8_t* data, size_t length);

/* Same, CRC-32C (Castagnoli): what a -msse4.2 / -march=native x86 build of the reference
 * computes in SubspaceCRC32 (client/checksum.cc:56-76). Raw state in and out. */
uint32_t SubspaceCRC32C(uint32_t crc, const uint8_t* data, size_t length);

/* Reflected polynomials for subspace_crc_ctx_create_poly. */
#define SUBSPACE_CRC_POLY_IEEE 0xEDB88320u       /* the reference's default builds */
#define SUBSPACE_CRC_POLY_CASTAGNOLI 0x82F63B78u /* CRC-32C, -msse4.2 reference builds */

/* Library version (major*10000 + minor*100 + patch). */
int subspace_crc_version(void);

/* Last error message of the calling thread ("" if none). */
const char* subspace_crc_last_error(void);

/* Create a context on HIP device `device` (uploads the CRC tables once). Every batch and
 * slot call on the context computes the IEEE CRC-32 of SubspaceCRC32. */
int subspace_crc_ctx_create(int device, subspace_crc_ctx** out);

/* The same for another reflected polynomial (bit 31 set, the x^0 term), e.g.
 * SUBSPACE_CRC_POLY_CASTAGNOLI: every call on the context then computes SubspaceCRC32C's
 * function. The kernels are table-driven; only the tables and operators differ. */
int subspace_crc_ctx_create_poly(int device, uint32_t reflected_poly, subspace_crc_ctx** out);
void subspace_crc_ctx_destroy(subspace_crc_ctx* ctx);

/* Synchronise `stream` and report whether any kernel launched on the context since the last
 * check gave up a bounded wait (a look-back scan predecessor or a slot ring entry that never
 * arrived): SUBSPACE_CRC_EFAULT with the reason in subspace_crc_last_error(), and the fault
 * is cleared (the context's scan state is reset before its next call); else SUBSPACE_CRC_OK.
 * The synchronous calls (subspace_crc32_host_slots, subspace_crc32_host_slot_list) check
 * it themselves. Device-side state is per context: calls on one context are serialised
 * across streams (a call on a new stream waits for the previous stream's work), and a
 * context is thread-safe (one call at a time). */
int subspace_crc_ctx_check(subspace_crc_ctx* ctx, void* stream);

/* Pre-size the ragged-batch workspace for up to `max_messages` messages and
 * `max_tiles` 8 KiB tiles so later subspace_crc32_batch calls never allocate
 * (required before capturing them into a hipGraph). */
int subspace_crc_ctx_reserve(subspace_crc_ctx* ctx, uint64_t max_messages, uint64_t max_tiles);

/* Fixed-size batch: message i is the `length` bytes at dev_base + i*stride.
 * stride >= length. Any length (0 allowed); any stride. The kernels read only inside
 * [dev_base, dev_base + (count-1)*stride + length), the end rounded up to 16 bytes (gaps
 * between messages included: they are read and ignored). */
int subspace_crc32_batch_uniform(subspace_crc_ctx* ctx, const void* dev_base, uint64_t stride, uint64_t length,
                                 uint64_t count, uint32_t init, uint32_t flags, uint32_t* dev_out, void* stream);

/* Ragged batch: message i is the dev_lengths[i] bytes at dev_base + dev_offsets[i].
 * arena_bytes = bytes readable from dev_base (every message must lie inside it). It sizes the
 * tile workspace and, up to 2^37 bytes, selects the one-kernel tile-count scan + 8-byte tile
 * descriptors; a message found outside it still gets its correct CRC (the kernel then locates
 * every tile by search, slower). dev_offsets / dev_lengths are device arrays of `count` uint64. */
int subspace_crc32_batch(subspace_crc_ctx* ctx, const void* dev_base, uint64_t arena_bytes,
                         const uint64_t* dev_offsets, const uint64_t* dev_lengths, uint64_t count, uint32_t init,
                         uint32_t flags, uint32_t* dev_out, void* stream);

/* ---------------------------------------------------------------------------------
 * Message slots: the reference's full 3-span checksum (common/channel.h:527-542),
 * computed and stored (publisher) or verified (subscriber) for a batch of slots.
 *
 * A slot's 64-B MessagePrefix (common/channel.h:88-112) and its checksum extension live
 * at `prefix`; its payload is the `message_size` bytes at `payload`. For each slot:
 *   span 0 = prefix[4, 48)                      (slot_id .. metadata_size, 44 B)
 *   span 1 = prefix[48 + checksum_size, +metadata_size)   (user metadata)
 *   span 2 = payload[0, message_size)
 *   crc    = ~SubspaceCRC32 chained over the spans from 0xFFFFFFFF (client/checksum.h:29-37)
 * SUBSPACE_CRC_SLOT_CALCULATE (client/publisher.cc:664-675): sets kMessageHasChecksum (4)
 *   in prefix->flags (before the CRC, as SetHasChecksum() does), then stores crc as a
 *   native-endian uint32 at prefix+48 (the first 4 B of the checksum area).
 * SUBSPACE_CRC_SLOT_VERIFY (client/client.cc:1346-1356, client/checksum.h:39-47): a slot
 *   whose prefix has kMessageHasChecksum is compared on the first 4 B of its checksum
 *   area; a slot without the flag is not checked.
 * Prefixes must be 8-B aligned (MessagePrefix holds int64 fields); payloads may have any
 * alignment. Prefix and payload bytes outside the spans (the padding word at offset 0,
 * checksum bytes 4.., padding after the metadata) are neither covered nor modified.
 * --------------------------------------------------------------------------------- */
#define SUBSPACE_CRC_SLOT_CALCULATE 0u
#define SUBSPACE_CRC_SLOT_VERIFY 1u

/* per-slot status written to dev_status (when not NULL) */
#define SUBSPACE_CRC_SLOT_OK 0u        /* checksum stored (CALCULATE) or matched (VERIFY) */
#define SUBSPACE_CRC_SLOT_MISMATCH 1u  /* VERIFY: "Checksum verification failed" (client/client.cc:1447) */
#define SUBSPACE_CRC_SLOT_UNCHECKED 2u /* VERIFY: prefix has no kMessageHasChecksum flag */
#define SUBSPACE_CRC_SLOT_OVERSIZE 4u  /* strided layouts: the slot's size exceeds its payload area
                                          (slot_stride - prefix size); neither checksummed nor
                                          modified, not counted as a mismatch */

/* One slot: device addresses of its MessagePrefix and payload, and the payload size
 * (slot->message_size at publish, the delivered size at read). 24 B, device array. */
typedef struct subspace_crc_slot {
  uint64_t prefix;
  uint64_t payload;
  uint64_t message_size;
} subspace_crc_slot;

/* Slot list (any placement, e.g. split buffers). max_message_size bounds every
 * message_size (pass the channel's slot size): with max_message_size <= 4096 the call is
 * one kernel launch (up to 64 messages per 8 KiB tile -- as many 128-B lines per message as
 * the bound needs -- the slot checksums finished in the same kernel); larger bounds take the
 * ragged pipeline. Either way a message larger than the
 * bound is still handled correctly, only more slowly. The lines per message are sized for
 * payloads on 16-B boundaries (every channel layout's payloads are 64-B aligned): with a bound
 * of at most 2,048 B, a payload starting s & 15 bytes into its 16-B block whose size plus s & 15
 * exceeds the lines' capacity (the least 128 * 2^k >= max_message_size) is computed on its
 * own by its wave after the tile loop -- correct, but one such message costs about a tile.
 * Lists of unaligned payloads close to the bound should pass max_message_size + 15.
 * dev_status: optional uint32[count]. dev_error_count: optional uint32, set to the number
 * of SUBSPACE_CRC_SLOT_MISMATCH slots of this call. */
int subspace_crc32_slots(subspace_crc_ctx* ctx, const subspace_crc_slot* dev_slots, uint64_t count,
                         uint64_t max_message_size, int32_t checksum_size, int32_t metadata_size, uint32_t mode,
                         uint32_t* dev_status, uint32_t* dev_error_count, void* stream);

/* Contiguous channel layout (client/client_channel.h:122-172): slot i's prefix is at
 * dev_buffer + i*slot_stride (slot_stride = PrefixSize + Aligned<64>(SlotSize)), its
 * payload at prefix + ComputePrefixSize(checksum_size, metadata_size)
 * (= Aligned<64>(48 + checksum_size + metadata_size), common/channel.h:914-919).
 * Payload sizes: dev_message_sizes[i] (uint64) when not NULL, else `message_size` for
 * every slot. A per-slot size larger than the slot's payload area (slot_stride - prefix size:
 * the reference never publishes more than the slot holds) gets SUBSPACE_CRC_SLOT_OVERSIZE: its
 * bytes would run into the next slot, whose prefix a publish rewrites in the same call. */
int subspace_crc32_slots_strided(subspace_crc_ctx* ctx, void* dev_buffer, uint64_t slot_stride, uint64_t count,
                                 uint64_t message_size, const uint64_t* dev_message_sizes, int32_t checksum_size,
                                 int32_t metadata_size, uint32_t mode, uint32_t* dev_status,
                                 uint32_t* dev_error_count, void* stream);

/* ---------------------------------------------------------------------------------
 * Host-memory slots: the end-to-end path. A channel's buffer lives in host shared memory
 * (the reference maps it with shm_open/memfd, client/client_channel.h:122-172); this call
 * takes that contiguous layout (slot i's prefix at host_buffer + i*slot_stride, payload
 * after ComputePrefixSize bytes; host_buffer spans count * slot_stride bytes), streams it to
 * the device in ~32 MiB chunks (one chunk's H2D copy overlaps the previous chunk's kernels)
 * and brings back 4 B per slot:
 *   CALCULATE: on return every prefix has kMessageHasChecksum set and its checksum stored
 *              (what client/publisher.cc:664-675 leaves in the slot);
 *   VERIFY:    host_status[i] (optional) and *host_error_count (optional) as for
 *              subspace_crc32_slots_strided; the host buffer is not modified.
 * host_message_sizes (optional, host uint64[count]) overrides message_size per slot.
 * Synchronous: returns when every prefix / status has been written. Pin the buffer once
 * with subspace_crc_host_register for full PCIe bandwidth (pageable memory works, slower).
 * --------------------------------------------------------------------------------- */
int subspace_crc32_host_slots(subspace_crc_ctx* ctx, void* host_buffer, uint64_t slot_stride, uint64_t count,
                              uint64_t message_size, const uint64_t* host_message_sizes, int32_t checksum_size,
                              int32_t metadata_size, uint32_t mode, uint32_t* host_status,
                              uint32_t* host_error_count);

/* Zero-copy slot list in host memory -- the subscriber drain hook: the slots a
 * GetAllMessages / ProcessAllMessages drain (client/client.cc:344-397) would read, in any
 * order and from any channels, as subspace_crc_slot records holding HOST addresses (the
 * records themselves are a host array). Every prefix and payload must lie in a region
 * registered with subspace_crc_host_register; the kernels read them in place over PCIe
 * through the region's device mapping (no staging copy of the payloads). CALCULATE writes
 * flag + checksum into the host prefixes; VERIFY fills host_status / *host_error_count
 * (SUBSPACE_CRC_SLOT_MISMATCH = "Checksum verification failed", client/client.cc:1447).
 * Synchronous. */
int subspace_crc32_host_slot_list(subspace_crc_ctx* ctx, const subspace_crc_slot* host_slots, uint64_t count,
                                  uint64_t max_message_size, int32_t checksum_size, int32_t metadata_size,
                                  uint32_t mode, uint32_t* host_status, uint32_t* host_error_count);

/* Page-lock (pin) host memory for DMA and map it for device access (hipHostRegister,
 * mapped + portable); release with subspace_crc_host_unregister (same pointer). */
int subspace_crc_host_register(void* host_ptr, uint64_t bytes);
int subspace_crc_host_unregister(void* host_ptr);

/* ---------------------------------------------------------------------------------
 * Split-buffer allocator: pinned + device-mapped shared memory for a channel's split
 * buffers (common/split_buffer.h:43-55: the per-slot payload buffers and the prefix buffer
 * of a channel whose publisher set PublisherOptions::SetSplitBufferCallbacks,
 * client/options.h:242-249; subscribers: SubscriberOptions, :404-411). The four functions
 * have exactly the C signatures of the reference C client's SubspaceSplitAllocateCallback,
 * SubspaceSplitMapCallback and SubspaceSplitReleaseCallback (c_client/subspace.h:140-158);
 * the two structs below are layout-identical restatements of SubspaceSplitBufferInfo
 * (c_client/subspace.h:109-119) and SubspaceSplitBufferMapping (:120-127), so a C client
 * passes them in a SubspaceSplitBufferCallbacks unchanged, and
 * the C++ client gets them through the reference's own ToCppSplitCallbacks
 * (c_client/subspace.cc:201-255).
 *
 * allocate: a memfd of allocation_size (full_size if 0) bytes, mapped shared read/write,
 *           then pinned and mapped for device access (subspace_crc_host_register), so the
 *           zero-copy slot-list path (subspace_crc32_host_slot_list) reads and writes it
 *           in place. mapping->fd = mapping->handle = the memfd (the reference shares it
 *           with subscribers through the server), mapping->size, mapping->address.
 * map:      a subscriber's view of a buffer another process allocated: mmap of the
 *           descriptor info->registration_fd (else mapping->handle, as the C++ adapter
 *           presets it) at info->map_offset, then pinned and device-mapped the same way.
 * unmap:    unpin, munmap. free: unpin, munmap, close the memfd.
 * user_data: NULL, or a subspace_crc_split_allocator selecting the options below.
 * Each returns true on success; on failure false, with subspace_crc_last_error() set.
 * --------------------------------------------------------------------------------- */
typedef struct subspace_crc_split_info {
  const char* channel_name;
  uint64_t session_id;
  uint32_t buffer_index;
  uint32_t slot_id;
  bool is_prefix;
  uint64_t full_size;
  uint64_t allocation_size;
  uintptr_t handle;
  int registration_fd;
  int64_t map_offset;
} subspace_crc_split_info;

typedef struct subspace_crc_split_mapping {
  uintptr_t handle;
  void* address;
  size_t size;
  void* private_data;
  int fd;
  int64_t map_offset;
} subspace_crc_split_mapping;

/* subspace_crc_split_allocator.flags */
#define SUBSPACE_CRC_SPLIT_REQUIRE_PIN 0x1u /* fail when pinning fails (default: keep the plain mapping) */

typedef struct subspace_crc_split_allocator {
  uint32_t flags;
} subspace_crc_split_allocator;

bool subspace_crc_split_allocate(const subspace_crc_split_info* info, subspace_crc_split_mapping* mapping,
                                 void* user_data);
bool subspace_crc_split_map(const subspace_crc_split_info* info, subspace_crc_split_mapping* mapping,
                            void* user_data);
bool subspace_crc_split_unmap(const subspace_crc_split_info* info, const subspace_crc_split_mapping* mapping,
                              void* user_data);
bool subspace_crc_split_free(const subspace_crc_split_info* info, const subspace_crc_split_mapping* mapping,
                             void* user_data);
/* 1 if the mapping of `address` is pinned and device-mapped, 0 if not, -1 if unknown. */
int subspace_crc_split_is_pinned(const void* address);

#ifdef __cplusplus
}
#endif
#endif /* SUBSPACE_CRC_H_ */
