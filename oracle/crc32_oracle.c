/*
 * oracle/crc32_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of dallison/subspace's default-build CRC32 path, used
 * by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * CHECKER (and as the timed CPU baseline). Nothing in subspace_amd/ links,
 * loads or calls this file; the product path fails loudly without its own
 * HIP library.
 *
 * What it restates (reference paths relative to /root/reference):
 *   - client/checksum.cc:14-17   x86-64 without __SSE4_2__ undefines
 *                                SUBSPACE_HARDWARE_CRC, selecting the table path;
 *   - client/checksum.cc:78-122  the 256-entry table for the reflected IEEE 802.3
 *                                polynomial 0xEDB88320 (rebuilt here from the
 *                                polynomial, not copied; tests/test_oracle.py
 *                                compares the two when the reference is present);
 *   - client/checksum.cc:125-130 the byte loop crc = (crc >> 8) ^ T[(crc ^ b) & 0xFF],
 *                                raw state in and out (no init / final XOR inside);
 *   - client/checksum.h:29-37    CalculateCRC32Checksum<N>: crc = 0xFFFFFFFF, chain the
 *                                spans, store ~crc as a native-endian uint32;
 *   - client/checksum.h:39-47    VerifyCRC32Checksum<N>: same chain, compare first 4 B;
 *   - common/channel.h:88-112, :527-542  MessagePrefix layout and the three checksum
 *                                spans (prefix+4 for 44 B, metadata, payload).
 *
 * Parity is pinned by (see DESIGN.md "Oracle"): the reference's own known-answer
 * tests (rust_client/tests/client_test.rs:169-218, "hello" -> 0x3610A686), the
 * reference table constants (checked in-container against client/checksum.cc),
 * and zlib's crc32 (an independent implementation of the same published
 * algorithm) on the golden fixtures in tests/golden/.
 *
 * The synthetic-input generator lives here too so the CPU
 * checker regenerates exactly the bytes the GPU bench generates on device.
 *
 * CRC-32C (the *_c functions): client/checksum.cc:56-76, the path a -msse4.2 /
 * -march=native x86 build takes -- _mm_crc32_u64 / _u32 / _u8 fold 8, 4, 1 bytes into a
 * raw CRC-32C state (reflected Castagnoli polynomial 0x82F63B78, no init / final XOR
 * inside), which equals the same byte loop over the Castagnoli table. Pinned by the
 * published CRC-32C check value ("123456789" -> 0xE3069283), the RFC 3720 B.4 vectors
 * and the reference's own -msse4.2 outputs recorded in SURVEY.md 8c ("hello" ->
 * 0x9A71BB4C), tests/golden/crc32c_kat.json.
 */
#define _GNU_SOURCE /* pthread_setaffinity_np, CPU_* (the pinned CPU-baseline workers) */
#include "crc32_oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>

static uint32_t g_table[256], g_table_c[256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* Table entry b = CRC of the single byte b from state 0, reflected poly 0xEDB88320
 * (client/checksum.cc:78: "IEEE 802.3 polynomial: 0xEDB88320"); g_table_c the same for
 * the reflected Castagnoli polynomial 0x82F63B78 (CRC-32C, client/checksum.cc:56-76). */
static void build_table(void) {
  for (uint32_t b = 0; b < 256; b++) {
    uint32_t c = b, d = b;
    for (int k = 0; k < 8; k++) {
      c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
      d = (d & 1u) ? (d >> 1) ^ 0x82F63B78u : (d >> 1);
    }
    g_table[b] = c;
    g_table_c[b] = d;
  }
}

const uint32_t* oracle_table(void) {
  pthread_once(&g_once, build_table);
  return g_table;
}

static const uint32_t* oracle_table_c(void) {
  pthread_once(&g_once, build_table);
  return g_table_c;
}

static uint32_t crc_table(const uint32_t* t, uint32_t crc, const uint8_t* data, size_t length) {
  for (size_t i = 0; i < length; i++) crc = (crc >> 8) ^ t[(crc ^ data[i]) & 0xFFu];
  return crc;
}

/* client/checksum.cc:125-130 */
uint32_t oracle_crc32(uint32_t crc, const uint8_t* data, size_t length) {
  return crc_table(oracle_table(), crc, data, length);
}

/* client/checksum.cc:56-76 (CRC-32C) */
uint32_t oracle_crc32c(uint32_t crc, const uint8_t* data, size_t length) {
  return crc_table(oracle_table_c(), crc, data, length);
}

/* client/checksum.h:29-37 */
static void calculate_checksum_t(const uint32_t* t, const uint8_t* const* spans, const size_t* lengths,
                                 size_t nspans, uint8_t* checksum_out4) {
  uint32_t crc = 0xFFFFFFFFu;
  for (size_t i = 0; i < nspans; i++) crc = crc_table(t, crc, spans[i], lengths[i]);
  crc = ~crc;
  memcpy(checksum_out4, &crc, 4);
}

void oracle_calculate_checksum(const uint8_t* const* spans, const size_t* lengths, size_t nspans,
                               uint8_t* checksum_out4) {
  calculate_checksum_t(oracle_table(), spans, lengths, nspans, checksum_out4);
}

/* client/checksum.h:39-47 */
static int verify_checksum_t(const uint32_t* t, const uint8_t* const* spans, const size_t* lengths, size_t nspans,
                             const uint8_t* checksum4) {
  uint32_t crc = 0xFFFFFFFFu;
  for (size_t i = 0; i < nspans; i++) crc = crc_table(t, crc, spans[i], lengths[i]);
  crc = ~crc;
  uint32_t stored;
  memcpy(&stored, checksum4, 4);
  return stored == crc;
}

int oracle_verify_checksum(const uint8_t* const* spans, const size_t* lengths, size_t nspans,
                           const uint8_t* checksum4) {
  return verify_checksum_t(oracle_table(), spans, lengths, nspans, checksum4);
}

/* common/channel.h:527-542: span [0] = prefix+4 for offsetof(checksum)-offsetof(slot_id)
 * = 48-4 = 44 bytes; [1] = prefix + 48 + checksum_size for metadata_size bytes;
 * [2] = payload for message_size bytes. */
void oracle_message_spans(const uint8_t* prefix, const uint8_t* payload, size_t message_size,
                          int32_t checksum_size, int32_t metadata_size, const uint8_t** spans_out,
                          size_t* lengths_out) {
  spans_out[0] = prefix + 4;
  lengths_out[0] = 44;
  spans_out[1] = prefix + 48 + checksum_size;
  lengths_out[1] = (size_t)metadata_size;
  spans_out[2] = payload;
  lengths_out[2] = message_size;
}

/* Publisher side of one slot (client/publisher.cc:664-675): SetHasChecksum() on the
 * prefix flags (int64 at offset 32, kMessageHasChecksum = 4, common/channel.h:65), then
 * CalculateCRC32Checksum over GetMessageChecksumData's spans into the checksum area. */
static void publish_slot_t(const uint32_t* t, uint8_t* prefix, const uint8_t* payload, size_t message_size,
                           int32_t checksum_size, int32_t metadata_size) {
  int64_t flags;
  memcpy(&flags, prefix + 32, 8);
  flags |= 4;
  memcpy(prefix + 32, &flags, 8);
  const uint8_t* spans[3];
  size_t lens[3];
  oracle_message_spans(prefix, payload, message_size, checksum_size, metadata_size, spans, lens);
  calculate_checksum_t(t, spans, lens, 3, prefix + 48);
}

void oracle_publish_slot(uint8_t* prefix, const uint8_t* payload, size_t message_size, int32_t checksum_size,
                         int32_t metadata_size) {
  publish_slot_t(oracle_table(), prefix, payload, message_size, checksum_size, metadata_size);
}

/* Subscriber side (client/client.cc:1346-1356): 2 = no kMessageHasChecksum flag (not
 * checked), else 0 = VerifyCRC32Checksum passed, 1 = "Checksum verification failed". */
static int verify_slot_t(const uint32_t* t, const uint8_t* prefix, const uint8_t* payload, size_t message_size,
                         int32_t checksum_size, int32_t metadata_size) {
  int64_t flags;
  memcpy(&flags, prefix + 32, 8);
  if (!(flags & 4)) return 2;
  const uint8_t* spans[3];
  size_t lens[3];
  oracle_message_spans(prefix, payload, message_size, checksum_size, metadata_size, spans, lens);
  return verify_checksum_t(t, spans, lens, 3, prefix + 48) ? 0 : 1;
}

int oracle_verify_slot(const uint8_t* prefix, const uint8_t* payload, size_t message_size, int32_t checksum_size,
                       int32_t metadata_size) {
  return verify_slot_t(oracle_table(), prefix, payload, message_size, checksum_size, metadata_size);
}

/* Slot batches over one host buffer: slot i's prefix at base + prefix_off[i], payload at
 * base + payload_off[i], sizes[i] payload bytes. */
void oracle_publish_slots_poly(uint8_t* base, const uint64_t* prefix_off, const uint64_t* payload_off,
                               const uint64_t* sizes, size_t n, int32_t checksum_size, int32_t metadata_size,
                               int castagnoli) {
  const uint32_t* t = castagnoli ? oracle_table_c() : oracle_table();
  for (size_t i = 0; i < n; i++)
    publish_slot_t(t, base + prefix_off[i], base + payload_off[i], (size_t)sizes[i], checksum_size, metadata_size);
}

void oracle_verify_slots_poly(const uint8_t* base, const uint64_t* prefix_off, const uint64_t* payload_off,
                              const uint64_t* sizes, size_t n, int32_t checksum_size, int32_t metadata_size,
                              uint32_t* status, int castagnoli) {
  const uint32_t* t = castagnoli ? oracle_table_c() : oracle_table();
  for (size_t i = 0; i < n; i++)
    status[i] = (uint32_t)verify_slot_t(t, base + prefix_off[i], base + payload_off[i], (size_t)sizes[i],
                                        checksum_size, metadata_size);
}

void oracle_publish_slots(uint8_t* base, const uint64_t* prefix_off, const uint64_t* payload_off,
                          const uint64_t* sizes, size_t n, int32_t checksum_size, int32_t metadata_size) {
  oracle_publish_slots_poly(base, prefix_off, payload_off, sizes, n, checksum_size, metadata_size, 0);
}

void oracle_verify_slots(const uint8_t* base, const uint64_t* prefix_off, const uint64_t* payload_off,
                         const uint64_t* sizes, size_t n, int32_t checksum_size, int32_t metadata_size,
                         uint32_t* status) {
  oracle_verify_slots_poly(base, prefix_off, payload_off, sizes, n, checksum_size, metadata_size, status, 0);
}

/* ------------------------------------------------------------------ batch */
typedef struct {
  const uint8_t* base;
  const uint64_t* offsets;
  const uint64_t* lengths;
  size_t n;
  uint32_t init;
  uint32_t* out;
  int tid, nthreads;
} batch_job;

static void* batch_worker(void* arg) {
  batch_job* j = (batch_job*)arg;
  for (size_t i = (size_t)j->tid; i < j->n; i += (size_t)j->nthreads)
    j->out[i] = oracle_crc32(j->init, j->base + j->offsets[i], (size_t)j->lengths[i]);
  return NULL;
}

/* Round-robin message partition over nthreads pthreads (BASELINE.md CPU-baseline plan). */
void oracle_crc32_batch(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, size_t n,
                        uint32_t init, uint32_t* out, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  batch_job* jobs = (batch_job*)calloc((size_t)nthreads, sizeof(batch_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    batch_job b = {base, offsets, lengths, n, init, out, t, nthreads};
    jobs[t] = b;
    if (t > 0) pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
  }
  batch_worker(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  free(jobs);
  free(th);
}

/* The CPU-baseline plan's threading (BASELINE.md "CPU-baseline plan" 2): one worker thread
 * per core, worker t pinned to the t-th CPU of the calling process's affinity set (the
 * calling thread itself is left alone and only joins), messages partitioned round-robin.
 * oracle_first_touch_copy copies a sample into `dst` with the same workers and partition,
 * so each message's pages are first touched (and, on a NUMA host, placed) by the worker
 * that later checksums it. Both return the number of workers that could be pinned. */
typedef struct {
  uint8_t* dst;
  const uint8_t* src;
  batch_job job;
  int cpu;
  int pinned;
} pinned_job;

static void pin_self(pinned_job* p) {
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(p->cpu, &set);
  p->pinned = pthread_setaffinity_np(pthread_self(), sizeof(set), &set) == 0;
}

static void* pinned_crc_worker(void* arg) {
  pinned_job* p = (pinned_job*)arg;
  pin_self(p);
  batch_worker(&p->job);
  return NULL;
}

static void* pinned_copy_worker(void* arg) {
  pinned_job* p = (pinned_job*)arg;
  pin_self(p);
  const batch_job* j = &p->job;
  for (size_t i = (size_t)j->tid; i < j->n; i += (size_t)j->nthreads)
    memcpy(p->dst + j->offsets[i], p->src + j->offsets[i], (size_t)j->lengths[i]);
  return NULL;
}

static int run_pinned(void* (*fn)(void*), uint8_t* dst, const uint8_t* src, const uint64_t* offsets,
                      const uint64_t* lengths, size_t n, uint32_t init, uint32_t* out, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  cpu_set_t mine;
  int cpus[CPU_SETSIZE], ncpu = 0;
  if (sched_getaffinity(0, sizeof(mine), &mine) == 0)
    for (int c = 0; c < CPU_SETSIZE; c++)
      if (CPU_ISSET(c, &mine)) cpus[ncpu++] = c;
  if (ncpu == 0) cpus[ncpu++] = 0;
  pinned_job* jobs = (pinned_job*)calloc((size_t)nthreads, sizeof(pinned_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    batch_job b = {src, offsets, lengths, n, init, out, t, nthreads};
    jobs[t].dst = dst;
    jobs[t].src = src;
    jobs[t].job = b;
    jobs[t].cpu = cpus[t % ncpu];
    pthread_create(&th[t], NULL, fn, &jobs[t]);
  }
  int pinned = 0;
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    pinned += jobs[t].pinned;
  }
  free(jobs);
  free(th);
  return pinned;
}

int oracle_crc32_batch_pinned(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, size_t n,
                              uint32_t init, uint32_t* out, int nthreads) {
  return run_pinned(pinned_crc_worker, NULL, base, offsets, lengths, n, init, out, nthreads);
}

int oracle_first_touch_copy(uint8_t* dst, const uint8_t* src, const uint64_t* offsets, const uint64_t* lengths,
                            size_t n, int nthreads) {
  return run_pinned(pinned_copy_worker, dst, src, offsets, lengths, n, 0, NULL, nthreads);
}

/* ------------------------------------------------------------------ synthetic inputs */
uint64_t oracle_splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* byte j of message i = byte (j mod 8) (little-endian) of splitmix64(seed ^ (i << 32) ^ (j >> 3)) */
void oracle_synth_fill(uint64_t seed, uint64_t msg, uint64_t start, uint8_t* dst, size_t n) {
  const uint64_t key = seed ^ (msg << 32);
  size_t k = 0;
  uint64_t j = start;
  while (k < n) {
    const uint64_t w = oracle_splitmix64(key ^ (j >> 3));
    const unsigned b0 = (unsigned)(j & 7);
    for (unsigned b = b0; b < 8 && k < n; b++, k++, j++) dst[k] = (uint8_t)(w >> (8 * b));
  }
}

static uint32_t synth_crc_t(const uint32_t* t, uint64_t seed, uint64_t msg, uint64_t length, uint32_t init) {
  uint8_t buf[4096];
  uint32_t crc = init;
  for (uint64_t pos = 0; pos < length; pos += sizeof(buf)) {
    const size_t n = (size_t)((length - pos) < sizeof(buf) ? (length - pos) : sizeof(buf));
    oracle_synth_fill(seed, msg, pos, buf, n);
    crc = crc_table(t, crc, buf, n);
  }
  return crc;
}

uint32_t oracle_synth_crc(uint64_t seed, uint64_t msg, uint64_t length, uint32_t init) {
  return synth_crc_t(oracle_table(), seed, msg, length, init);
}

typedef struct {
  const uint32_t* table;
  uint64_t seed;
  const uint64_t* msg_ids;
  const uint64_t* lengths;
  size_t n;
  uint32_t init;
  uint32_t* out;
  int tid, nthreads;
} synth_job;

static void* synth_worker(void* arg) {
  synth_job* j = (synth_job*)arg;
  for (size_t i = (size_t)j->tid; i < j->n; i += (size_t)j->nthreads)
    j->out[i] = synth_crc_t(j->table, j->seed, j->msg_ids ? j->msg_ids[i] : i, j->lengths[i], j->init);
  return NULL;
}

void oracle_synth_crc_batch_poly(uint64_t seed, const uint64_t* msg_ids, const uint64_t* lengths, size_t n,
                                 uint32_t init, uint32_t* out, int nthreads, int castagnoli) {
  const uint32_t* table = castagnoli ? oracle_table_c() : oracle_table();
  if (nthreads < 1) nthreads = 1;
  synth_job* jobs = (synth_job*)calloc((size_t)nthreads, sizeof(synth_job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    synth_job s = {table, seed, msg_ids, lengths, n, init, out, t, nthreads};
    jobs[t] = s;
    if (t > 0) pthread_create(&th[t], NULL, synth_worker, &jobs[t]);
  }
  synth_worker(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  free(jobs);
  free(th);
}

void oracle_synth_crc_batch(uint64_t seed, const uint64_t* msg_ids, const uint64_t* lengths, size_t n,
                            uint32_t init, uint32_t* out, int nthreads) {
  oracle_synth_crc_batch_poly(seed, msg_ids, lengths, n, init, out, nthreads, 0);
}

/* Config C lengths (integer form so every implementation agrees bit for bit):
 * t = splitmix64(seed ^ 0x4C454E0000000000 ^ i); octave = t % 14; frac = (t >> 16) & 0xFFFF;
 * L = (64 << octave) + (((64 << octave) * frac) >> 16)  -> 64 <= L < 2^20, uniform octave. */
uint64_t oracle_ragged_length(uint64_t seed, uint64_t i) {
  const uint64_t t = oracle_splitmix64(seed ^ 0x4C454E0000000000ull ^ i);
  const uint64_t base = 64ull << (t % 14);
  return base + ((base * ((t >> 16) & 0xFFFFull)) >> 16);
}
