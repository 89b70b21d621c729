// Split-buffer allocator (include/subspace_crc.h "Split-buffer allocator"): pinned +
// device-mapped shared memory for the split buffers of a Subspace channel
// (common/split_buffer.h:43-55), behind the reference C client's callback signatures
// (c_client/subspace.h:140-158). Host code only: the pinning goes through the library's own
// subspace_crc_host_register, which records the region's device alias for the zero-copy
// slot-list path (capi.hip).
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <mutex>
#include <unordered_map>

#include "../../include/subspace_crc.h"

namespace subspace_amd {
int set_error(int code, const char* fmt, ...);  // capi.hip: the thread-local error string
}

namespace {

struct Region {
  size_t size;
  int fd;        // the memfd (allocate) or -1 (map: the descriptor stays the caller's)
  bool pinned;
};

std::mutex g_mu;
std::unordered_map<uintptr_t, Region> g_regions;  // by mapped address

bool fail(const char* fmt, const char* what, int err) {
  subspace_amd::set_error(SUBSPACE_CRC_EINVAL, fmt, what, std::strerror(err));
  return false;
}

uint32_t flags_of(void* user_data) {
  return user_data ? static_cast<const subspace_crc_split_allocator*>(user_data)->flags : 0u;
}

// Pin + device-map a fresh mapping; record it. On a pinning failure the mapping is kept
// (unpinned: the slot-list path then rejects it) unless the caller requires the pin.
bool adopt(void* addr, size_t size, int fd, uint32_t flags) {
  const bool pinned = subspace_crc_host_register(addr, size) == SUBSPACE_CRC_OK;
  if (!pinned && (flags & SUBSPACE_CRC_SPLIT_REQUIRE_PIN)) {
    // keep the registration error (subspace_crc_last_error) for the caller
    munmap(addr, size);
    return false;
  }
  std::lock_guard<std::mutex> lock(g_mu);
  g_regions[reinterpret_cast<uintptr_t>(addr)] = Region{size, fd, pinned};
  return true;
}

bool release(const subspace_crc_split_mapping* mapping, bool close_fd) {
  if (!mapping || !mapping->address) {
    subspace_amd::set_error(SUBSPACE_CRC_EINVAL, "split buffer: empty mapping");
    return false;
  }
  Region r{};
  {
    std::lock_guard<std::mutex> lock(g_mu);
    auto it = g_regions.find(reinterpret_cast<uintptr_t>(mapping->address));
    if (it == g_regions.end()) {
      subspace_amd::set_error(SUBSPACE_CRC_EINVAL, "split buffer %p was not mapped by this allocator",
                              mapping->address);
      return false;
    }
    r = it->second;
    g_regions.erase(it);
  }
  bool ok = true;
  if (r.pinned && subspace_crc_host_unregister(mapping->address) != SUBSPACE_CRC_OK) ok = false;
  if (munmap(mapping->address, r.size) != 0) ok = fail("split buffer %s: munmap: %s", "unmap", errno);
  if (close_fd && r.fd >= 0 && close(r.fd) != 0) ok = fail("split buffer %s: close: %s", "free", errno);
  return ok;
}

}  // namespace

extern "C" {

bool subspace_crc_split_allocate(const subspace_crc_split_info* info, subspace_crc_split_mapping* mapping,
                                 void* user_data) {
  if (!info || !mapping) {
    subspace_amd::set_error(SUBSPACE_CRC_EINVAL, "split buffer allocate: null info or mapping");
    return false;
  }
  const uint64_t size = info->allocation_size ? info->allocation_size : info->full_size;
  if (size == 0) {
    subspace_amd::set_error(SUBSPACE_CRC_EINVAL, "split buffer allocate: zero size");
    return false;
  }
  const char* name = info->channel_name && *info->channel_name ? info->channel_name : "subspace_split";
  const int fd = memfd_create(name, MFD_CLOEXEC);
  if (fd < 0) return fail("split buffer %s: memfd_create: %s", name, errno);
  if (ftruncate(fd, (off_t)size) != 0) {
    const int e = errno;
    close(fd);
    return fail("split buffer %s: ftruncate: %s", name, e);
  }
  void* addr = mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (addr == MAP_FAILED) {
    const int e = errno;
    close(fd);
    return fail("split buffer %s: mmap: %s", name, e);
  }
  if (!adopt(addr, size, fd, flags_of(user_data))) {
    close(fd);
    return false;
  }
  mapping->handle = static_cast<uintptr_t>(fd);
  mapping->address = addr;
  mapping->size = size;
  mapping->private_data = nullptr;
  mapping->fd = fd;
  mapping->map_offset = 0;
  return true;
}

bool subspace_crc_split_map(const subspace_crc_split_info* info, subspace_crc_split_mapping* mapping,
                            void* user_data) {
  if (!info || !mapping) {
    subspace_amd::set_error(SUBSPACE_CRC_EINVAL, "split buffer map: null info or mapping");
    return false;
  }
  const int fd = info->registration_fd >= 0 ? info->registration_fd : static_cast<int>(mapping->handle);
  const uint64_t size = info->allocation_size ? info->allocation_size : info->full_size;
  if (fd < 0 || size == 0) {
    subspace_amd::set_error(SUBSPACE_CRC_EINVAL, "split buffer map: no descriptor (fd %d) or zero size", fd);
    return false;
  }
  void* addr = mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, (off_t)info->map_offset);
  if (addr == MAP_FAILED) return fail("split buffer %s: mmap: %s", "map", errno);
  if (!adopt(addr, size, -1, flags_of(user_data))) return false;
  mapping->handle = static_cast<uintptr_t>(fd);
  mapping->address = addr;
  mapping->size = size;
  mapping->private_data = nullptr;
  mapping->fd = fd;
  mapping->map_offset = info->map_offset;
  return true;
}

bool subspace_crc_split_unmap(const subspace_crc_split_info* /*info*/, const subspace_crc_split_mapping* mapping,
                              void* /*user_data*/) {
  return release(mapping, /*close_fd=*/false);
}

bool subspace_crc_split_free(const subspace_crc_split_info* /*info*/, const subspace_crc_split_mapping* mapping,
                             void* /*user_data*/) {
  return release(mapping, /*close_fd=*/true);
}

int subspace_crc_split_is_pinned(const void* address) {
  std::lock_guard<std::mutex> lock(g_mu);
  auto it = g_regions.find(reinterpret_cast<uintptr_t>(address));
  return it == g_regions.end() ? -1 : (it->second.pinned ? 1 : 0);
}

}  // extern "C"
