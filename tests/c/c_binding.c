/*
 * The C-client binding of INTEGRATION.md section 3, compiled against libsubspace_crc.so.
 *
 * The reference C client (c_client/subspace.h:129-136) takes a checksum callback
 *   typedef void (*SubspaceChecksumCallback)(const SubspaceChecksumSpan* spans, size_t span_count,
 *                                            uint8_t* checksum, size_t checksum_size, void* user_data);
 * registered with subspace_register_publisher_checksum_callback (c_client/subspace.cc:1412-1459);
 * and split-buffer callbacks (c_client/subspace.h:140-158). The typedefs below restate those
 * interfaces (same layout and signatures, local names) so this file compiles without the
 * reference headers; assigning the library's functions to them checks the signatures at
 * compile time (-Werror=incompatible-pointer-types in tests/test_c_binding.py).
 *
 * stdin: one message per line, its spans as hex strings separated by spaces ("-" = empty span).
 * stdout: the checksum the callback stores (a native-endian uint32), one line per message.
 */
#define _POSIX_C_SOURCE 200809L /* getline */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "subspace_crc.h"

typedef struct {
  const uint8_t* data;
  size_t size;
} ChecksumSpan; /* == SubspaceChecksumSpan */

typedef void (*ChecksumCallback)(const ChecksumSpan* spans, size_t span_count, uint8_t* checksum,
                                 size_t checksum_size, void* user_data); /* == SubspaceChecksumCallback */

typedef bool (*SplitAllocate)(const subspace_crc_split_info*, subspace_crc_split_mapping*, void*);
typedef bool (*SplitRelease)(const subspace_crc_split_info*, const subspace_crc_split_mapping*, void*);
typedef struct {
  SplitAllocate allocate;
  SplitAllocate map;
  SplitRelease unmap;
  SplitRelease free;
  void* user_data;
} SplitCallbacks; /* == SubspaceSplitBufferCallbacks */

/* The stub of INTEGRATION.md section 3. */
static void crc_cb(const ChecksumSpan* spans, size_t n, uint8_t* out, size_t out_size, void* ud) {
  (void)ud;
  uint32_t crc = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) crc = SubspaceCRC32(crc, spans[i].data, spans[i].size);
  crc = ~crc;
  if (out_size >= 4) memcpy(out, &crc, 4);
}

static int hexval(int c) { return c <= '9' ? c - '0' : (c | 32) - 'a' + 10; }

int main(void) {
  const ChecksumCallback cb = crc_cb;
  const SplitCallbacks split = {subspace_crc_split_allocate, subspace_crc_split_map, subspace_crc_split_unmap,
                                subspace_crc_split_free, NULL};
  /* one split buffer through the callback table: allocate, write, free */
  subspace_crc_split_info info = {"/c_binding", 1, 0, 0, false, 8192, 8192, 0, -1, 0};
  subspace_crc_split_mapping m;
  memset(&m, 0, sizeof(m));
  if (!split.allocate(&info, &m, split.user_data) || m.size != 8192) {
    fprintf(stderr, "allocate failed: %s\n", subspace_crc_last_error());
    return 2;
  }
  memset(m.address, 0x5A, m.size);
  if (!split.free(&info, &m, split.user_data)) {
    fprintf(stderr, "free failed: %s\n", subspace_crc_last_error());
    return 2;
  }

  char* line = NULL;
  size_t cap = 0;
  ssize_t got;
  while ((got = getline(&line, &cap, stdin)) > 0) {
    ChecksumSpan spans[8];
    uint8_t* bufs[8];
    size_t n = 0;
    for (char* tok = strtok(line, " \n"); tok && n < 8; tok = strtok(NULL, " \n")) {
      size_t len = strcmp(tok, "-") == 0 ? 0 : strlen(tok) / 2;
      bufs[n] = malloc(len ? len : 1); /* exactly len bytes: ASan sees any over-read */
      for (size_t i = 0; i < len; i++) bufs[n][i] = (uint8_t)(hexval(tok[2 * i]) << 4 | hexval(tok[2 * i + 1]));
      spans[n].data = bufs[n];
      spans[n].size = len;
      n++;
    }
    uint8_t out[8] = {0};
    cb(spans, n, out, sizeof(out), NULL);
    uint32_t v;
    memcpy(&v, out, 4);
    printf("%u\n", v);
    for (size_t i = 0; i < n; i++) free(bufs[i]);
  }
  free(line);
  return 0;
}
