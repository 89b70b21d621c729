/*
 * oracle/crc32c_sse42.c -- TEST INFRASTRUCTURE ONLY (bench.py's informational CPU leg).
 *
 * Restates client/checksum.cc:56-76, the SubspaceCRC32 a -msse4.2 / -march=native x86
 * build of the reference compiles: _mm_crc32_u64 over 8-byte words, one _mm_crc32_u32,
 * then _mm_crc32_u8 for the tail, raw state in and out. It computes CRC-32C, NOT the
 * IEEE CRC of the default build (the parity definition), so bench.py reports its rate
 * only as an informational "sse42_crc32c" figure. This file alone is compiled with
 * -msse4.2; callers check oracle_has_sse42() first.
 */
#include <nmmintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int oracle_has_sse42(void) { return __builtin_cpu_supports("sse4.2"); }

uint32_t oracle_crc32c_sse42(uint32_t crc, const uint8_t* data, size_t length) {
  size_t i = 0;
  for (; i + 8 <= length; i += 8) {
    uint64_t w;
    memcpy(&w, data + i, 8);
    crc = (uint32_t)_mm_crc32_u64(crc, w);
  }
  if (i + 4 <= length) {
    uint32_t w;
    memcpy(&w, data + i, 4);
    crc = _mm_crc32_u32(crc, w);
    i += 4;
  }
  for (; i < length; i++) crc = _mm_crc32_u8(crc, data[i]);
  return crc;
}

typedef struct {
  const uint8_t* base;
  const uint64_t* offsets;
  const uint64_t* lengths;
  size_t n;
  uint32_t init;
  uint32_t* out;
  int tid, nthreads;
} job;

static void* worker(void* arg) {
  job* j = (job*)arg;
  for (size_t i = (size_t)j->tid; i < j->n; i += (size_t)j->nthreads)
    j->out[i] = oracle_crc32c_sse42(j->init, j->base + j->offsets[i], (size_t)j->lengths[i]);
  return NULL;
}

void oracle_crc32c_sse42_batch(const uint8_t* base, const uint64_t* offsets, const uint64_t* lengths, size_t n,
                               uint32_t init, uint32_t* out, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  job* jobs = (job*)calloc((size_t)nthreads, sizeof(job));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; t++) {
    job b = {base, offsets, lengths, n, init, out, t, nthreads};
    jobs[t] = b;
    if (t > 0) pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  worker(&jobs[0]);
  for (int t = 1; t < nthreads; t++) pthread_join(th[t], NULL);
  free(jobs);
  free(th);
}
