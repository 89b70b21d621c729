// Thread-safety stress of the library's host code, built with -fsanitize=thread by
// `make tsan-test` (the reference runs its tests under tsan in CI).
// The reference's SubspaceCRC32 is called concurrently from any client thread
// (client/checksum.h:18-20: pure, reentrant), so every host entry point must be too:
//  * SubspaceCRC32 / SubspaceCRC32C from 8 threads at once, first use included (the run-time
//    CPU dispatch and the lazily built tables), checked against a bitwise CRC here;
//  * the split-buffer allocator callbacks (shared region registry) allocating, writing,
//    querying and freeing concurrently;
//  * the thread-local error string: each thread provokes its own error and must read back
//    its own message;
//  * subspace_crc_host_register / _unregister of private buffers (the registry the
//    zero-copy slot-list path reads), which fail cleanly without a GPU.
// Exit status 0 when every check passes; ThreadSanitizer findings abort (halt_on_error).
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "subspace/checksum.h"
#include "subspace_crc.h"

namespace {

uint32_t bitwise_crc(uint32_t crc, const uint8_t* p, size_t n, uint32_t poly) {
  for (size_t i = 0; i < n; i++) {
    crc ^= p[i];
    for (int k = 0; k < 8; k++) crc = (crc >> 1) ^ ((crc & 1u) ? poly : 0u);
  }
  return crc;
}

std::atomic<int> g_failures{0};

void fail(const char* what, int t) {
  std::fprintf(stderr, "thread %d: %s\n", t, what);
  g_failures++;
}

void worker(int t, int iters) {
  std::mt19937_64 rng(0x75A11 + t);
  std::vector<uint8_t> buf(70000);
  for (auto& b : buf) b = (uint8_t)rng();
  for (int it = 0; it < iters; it++) {
    // host CRCs, random lengths and seeds (the body/tail split of the PCLMULQDQ path)
    const size_t n = rng() % buf.size();
    const size_t off = rng() % 64;
    const size_t len = n > off ? n - off : 0;
    const uint32_t seed = (uint32_t)rng();
    if (SubspaceCRC32(seed, buf.data() + off, len) != bitwise_crc(seed, buf.data() + off, len, 0xEDB88320u))
      fail("SubspaceCRC32 mismatch", t);
    if (SubspaceCRC32C(seed, buf.data() + off, len) != bitwise_crc(seed, buf.data() + off, len, 0x82F63B78u))
      fail("SubspaceCRC32C mismatch", t);

    // split buffers: allocate, write, query, free (no GPU: the mappings stay unpinned)
    subspace_crc_split_info info{};
    const std::string name = "/tsan_" + std::to_string(t);
    info.channel_name = name.c_str();
    info.slot_id = (uint32_t)it;
    info.allocation_size = 4096 * (1 + rng() % 4);
    info.full_size = info.allocation_size;
    info.registration_fd = -1;
    subspace_crc_split_mapping m{};
    if (!subspace_crc_split_allocate(&info, &m, nullptr)) {
      fail(subspace_crc_last_error(), t);
      continue;
    }
    std::memset(m.address, t, m.size);
    if (subspace_crc_split_is_pinned(m.address) < 0) fail("split buffer not registered", t);
    if (!subspace_crc_split_free(&info, &m, nullptr)) fail(subspace_crc_last_error(), t);

    // the thread-local error string: provoke an error, read back this thread's message
    if (subspace_crc_split_unmap(&info, nullptr, nullptr)) fail("unmap(NULL) succeeded", t);
    if (!std::strstr(subspace_crc_last_error(), "split buffer")) fail("error string not this thread's", t);

    // host registration of a private buffer (fails cleanly without a GPU)
    std::vector<uint8_t> pin(8192);
    if (subspace_crc_host_register(pin.data(), pin.size()) == SUBSPACE_CRC_OK)
      (void)subspace_crc_host_unregister(pin.data());
  }
}

}  // namespace

int main(int argc, char** argv) {
  const int threads = argc > 1 ? std::atoi(argv[1]) : 8;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 200;
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; t++) ts.emplace_back(worker, t, iters);
  for (auto& th : ts) th.join();
  std::printf("tsan_stress: %d threads x %d iterations, %d failures\n", threads, iters, g_failures.load());
  return g_failures.load() == 0 ? 0 : 1;
}
