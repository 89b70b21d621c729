/* oracle/crc32_oracle.h -- TEST INFRASTRUCTURE ONLY (see crc32_oracle.c header). */
#ifndef SUBSPACE_CRC32_ORACLE_H_
#define SUBSPACE_CRC32_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const uint32_t* oracle_table(void);
uint32_t oracle_crc32(uint32_t crc, const uint8_t* data, size_t length);
uint32_t oracle_crc32c(uint32_t crc, const uint8_t* data, size_t length);
void oracle_calculate_checksum(const uint8_t* const* spans, const size_t* lengths, size_t nspans,
                               uint8_t* checksum_out4);
int oracle_verify_checksum(const uint8_t* const* spans, const size_t* lengths, size_t nspans,
                           const uint8_t* checksum4);
void oracle_message_spans(const uint8_t* prefix, const uint8_t* payload, size_t message_size,
                          int32_t checksum_size, int32_t metadata_size, const uint8_t** spans_out,
                          size_t* lengths_out);
void oracle_publish_slot(uint8_t* prefix, const uint8_t* payload, size_t message_size, int32_t checksum_size,
                         int32_t metadata_size);
int oracle_verify_slot(const uint8_t* prefix, const uint8_t* payload, size_t message_size, int32_t checksum_size,
                       int32_t metadata_size);
void oracle_publish_slots(uint8_t* base, const uint64_t* prefix_off, const uint64_t* payload_off,
                          const uint64_t* sizes, size_t n, int32_t checksum_size, int32_t metadata_size);
void oracle_verify_slots(const uint8_t* base, const uint64_t* prefix_off, const uint64_t* payload_off,
                         const uint64_t* sizes, size_t n, int32_t checksum_size, int32_t metadata_size,
                         uint32_t* status);
void oracle_crc32_batch(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, size_t n,
                        uint32_t init, uint32_t* out, int nthreads);
/* The same with one pinned worker thread per CPU of the caller's affinity set (the
 * CPU-baseline plan), and the first-touch copy of a sample by the same workers. */
int oracle_crc32_batch_pinned(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, size_t n,
                              uint32_t init, uint32_t* out, int nthreads);
int oracle_first_touch_copy(uint8_t* dst, const uint8_t* src, const uint64_t* offsets, const uint64_t* lengths,
                            size_t n, int nthreads);

uint64_t oracle_splitmix64(uint64_t x);
void oracle_synth_fill(uint64_t seed, uint64_t msg, uint64_t start, uint8_t* dst, size_t n);
uint32_t oracle_synth_crc(uint64_t seed, uint64_t msg, uint64_t length, uint32_t init);
void oracle_synth_crc_batch(uint64_t seed, const uint64_t* msg_ids, const uint64_t* lengths, size_t n,
                            uint32_t init, uint32_t* out, int nthreads);
uint64_t oracle_ragged_length(uint64_t seed, uint64_t i);

/* crc32c_sse42.c: the reference's -msse4.2 path (client/checksum.cc:56-76), informational */
int oracle_has_sse42(void);
uint32_t oracle_crc32c_sse42(uint32_t crc, const uint8_t* data, size_t length);
void oracle_crc32c_sse42_batch(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, size_t n,
                               uint32_t init, uint32_t* out, int nthreads);

/* castagnoli != 0: the same with CRC-32C (client/checksum.cc:56-76) */
void oracle_synth_crc_batch_poly(uint64_t seed, const uint64_t* msg_ids, const uint64_t* lengths, size_t n,
                                 uint32_t init, uint32_t* out, int nthreads, int castagnoli);
void oracle_publish_slots_poly(uint8_t* base, const uint64_t* prefix_off, const uint64_t* payload_off,
                               const uint64_t* sizes, size_t n, int32_t checksum_size, int32_t metadata_size,
                               int castagnoli);
void oracle_verify_slots_poly(const uint8_t* base, const uint64_t* prefix_off, const uint64_t* payload_off,
                              const uint64_t* sizes, size_t n, int32_t checksum_size, int32_t metadata_size,
                              uint32_t* status, int castagnoli);

#ifdef __cplusplus
}
#endif
#endif
