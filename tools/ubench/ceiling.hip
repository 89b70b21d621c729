// Read ceilings at config B's launch size (investigation tool): 256 MiB per launch,
// 4 rotated windows (1 GiB), 300 back-to-back launches per variant after a 40 ms warm-up
// of the same variant, variants interleaved twice. Compared with the CRC kernel of every
// library build named in CEILING_LIBS (comma-separated .so paths, dlopen'ed side by side;
// default: the in-tree subspace_amd/libsubspace_crc.so) under the same schedule.
//   hipcc --offload-arch=gfx950 -O3 -o ceiling ceiling.hip -I../../include -ldl
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <functional>
#include <vector>

#include <dlfcn.h>
#include <cstring>
#include <string>

#include "subspace_crc.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)
typedef unsigned int u32;
typedef unsigned long long u64;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

__device__ __forceinline__ u64 front(u32 b, u32 G, u32 wid) { return ((u64)b + (u64)G * (wid >> 1)) * 2 + (wid & 1u); }

// SHAPE 0: lane <-> 128-B line (lane reads 8 consecutive 16-B blocks);
// SHAPE 1: coalesced (instruction i reads 1 KiB: lane l gets block 64*i + l).
// PF: explicit ping-pong prefetch of the next tile (as the CRC kernel does).
// WG: 512 (8 waves per CU) or 256 (4 waves per CU: with PF the same bytes in flight per CU
// as 8 waves without, one wave per SIMD).
template <int SHAPE, bool PF, int WG = 512>
__global__ __launch_bounds__(WG) void readk(const u32x4* __restrict__ p, u64 ntiles, u32* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const u32 wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 w = front(blockIdx.x, gridDim.x, wid), nw = (u64)gridDim.x * (WG / 64);
  const u32 nk = w < ntiles ? (u32)((ntiles - w + nw - 1) / nw) : 0u;
  auto addr = [&](u32 k, int i) -> const u32x4* {
    const u32 kk = k < nk ? k : (nk ? nk - 1 : 0u);
    const u64 t = nk ? w + (u64)kk * nw : 0;
    return SHAPE == 0 ? p + t * 512 + lane * 8 + i : p + t * 512 + i * 64 + lane;
  };
  u32 acc = 0;
  if (!PF) {
    for (u32 k = 0; k < nk; k++) {
      u32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = *addr(k, i);
#pragma unroll
      for (int i = 0; i < 8; i++) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    }
  } else {
    u32x4 a[8], b[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = *addr(0, i);
    u32 k = 0;
    for (; k + 1 < nk; k += 2) {
#pragma unroll
      for (int i = 0; i < 8; i++) b[i] = *addr(k + 1, i);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 8; i++) acc ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
#pragma unroll
      for (int i = 0; i < 8; i++) a[i] = *addr(k + 2, i);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 8; i++) acc ^= b[i].x ^ b[i].y ^ b[i].z ^ b[i].w;
    }
    if (k < nk)
#pragma unroll
      for (int i = 0; i < 8; i++) acc ^= a[i].x ^ a[i].y ^ a[i].z ^ a[i].w;
  }
  out[blockIdx.x * WG + threadIdx.x] = acc;
}

// lines (drain, then issue the next tile) + optional LDS fill prologue + optional dependent
// VALU work per tile (overlapping the next tile's loads, like the CRC kernel's compute).
template <int FILL, int WORK>
__global__ __launch_bounds__(512) void linesx(const u32x4* __restrict__ p, u64 ntiles, u32* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  const int lane = threadIdx.x & 63;
  const u32 wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 w = front(blockIdx.x, gridDim.x, wid), nw = (u64)gridDim.x * 8;
  const u32 nk = w < ntiles ? (u32)((ntiles - w + nw - 1) / nw) : 0u;
  u32x4 a[8];
  const u64 t0 = nk ? w : 0;
#pragma unroll
  for (int i = 0; i < 8; i++) a[i] = p[t0 * 512 + lane * 8 + i];
  if (FILL) {
    for (int i = threadIdx.x; i < 32768; i += 512) smem[i] = (u32)i * 2654435761u;
    __syncthreads();
  }
  u32 acc = 0;
  for (u32 k = 0; k < nk; k++) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    u32x4 b[8];
#pragma unroll
    for (int i = 0; i < 8; i++) b[i] = a[i];
    const u64 tn = w + (u64)(k + 1 < nk ? k + 1 : k) * nw;
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = p[tn * 512 + lane * 8 + i];
    __builtin_amdgcn_sched_barrier(0);
    u32 x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= b[i].x ^ b[i].y ^ b[i].z ^ b[i].w;
    for (int r = 0; r < WORK; r++) x = x * 2654435761u + (x >> 7);
    acc ^= x;
  }
  if (FILL) acc ^= smem[lane];
  out[blockIdx.x * 512 + threadIdx.x] = acc;
}

int main() {
  const u64 win = 256ull << 20, nwin = 4, ntiles = win / 8192;
  u32x4* buf; CK(hipMalloc(&buf, win * nwin));
  u32* out; CK(hipMalloc(&out, 256 * 512 * 4));
  u32* crc; CK(hipMalloc(&crc, 65536 * 4));
  // CEILING_MSG = message length for the library variants (default 4096: config B's
  // 65,536 messages; e.g. 67108864 = config D's 64 MiB messages, 4 per 256 MiB launch)
  const u64 msg = getenv("CEILING_MSG") ? strtoull(getenv("CEILING_MSG"), nullptr, 10) : 4096;
  const u64 nmsg = win / msg;
  CK(hipMemset(buf, 0x5A, win * nwin));
  typedef int (*create_t)(int, subspace_crc_ctx**);
  typedef int (*uni_t)(subspace_crc_ctx*, const void*, uint64_t, uint64_t, uint64_t, uint32_t, uint32_t, uint32_t*,
                       void*);
  struct Lib { std::string path; uni_t uni; subspace_crc_ctx* ctx; };
  std::vector<Lib> libs;
  {
    const char* env = getenv("CEILING_LIBS");
    std::string all = env ? env : "subspace_amd/libsubspace_crc.so";
    size_t pos = 0;
    while (pos <= all.size()) {
      size_t e = all.find(',', pos);
      if (e == std::string::npos) e = all.size();
      std::string path = all.substr(pos, e - pos);
      pos = e + 1;
      if (path.empty()) continue;
      int order = -1;  // "lib.so@N": uniform kernel tile order N (subspace_crc_testutil_tune)
      const size_t at = path.find('@');
      if (at != std::string::npos) {
        order = std::atoi(path.c_str() + at + 1);
        path = path.substr(0, at);
      }
      void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
      if (!h) { fprintf(stderr, "dlopen %s: %s\n", path.c_str(), dlerror()); return 1; }
      auto create = (create_t)dlsym(h, "subspace_crc_ctx_create");
      Lib L{path, (uni_t)dlsym(h, "subspace_crc32_batch_uniform"), nullptr};
      if (!create || !L.uni || create(0, &L.ctx)) { fprintf(stderr, "ctx for %s failed\n", path.c_str()); return 1; }
      if (order >= 0) {
        typedef int (*tune_t)(subspace_crc_ctx*, int, int, int);
        auto tune = (tune_t)dlsym(h, "subspace_crc_testutil_tune");
        if (!tune || tune(L.ctx, 512, 0, order)) { fprintf(stderr, "tune %s failed\n", path.c_str()); return 1; }
        L.path += "@" + std::to_string(order);
      }
      libs.push_back(L);
    }
  }
  CK(hipFuncSetAttribute((const void*)linesx<1, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024));
  CK(hipFuncSetAttribute((const void*)linesx<1, 800>, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024));
  CK(hipDeviceSynchronize());
  struct V { const char* name; std::function<void(const u32x4*)> f; };
  std::vector<V> vs = {
      {"lines", [&](const u32x4* p) { readk<0, false><<<256, 512>>>(p, ntiles, out); }},
      {"lines+pf", [&](const u32x4* p) { readk<0, true><<<256, 512>>>(p, ntiles, out); }},
      {"lines wg256", [&](const u32x4* p) { readk<0, false, 256><<<256, 256>>>(p, ntiles, out); }},
      {"lines+pf wg256", [&](const u32x4* p) { readk<0, true, 256><<<256, 256>>>(p, ntiles, out); }},
      {"coalesced", [&](const u32x4* p) { readk<1, false><<<256, 512>>>(p, ntiles, out); }},
      {"coalesced+pf", [&](const u32x4* p) { readk<1, true><<<256, 512>>>(p, ntiles, out); }},
      {"lines + 152 KiB LDS fill", [&](const u32x4* p) { linesx<1, 0><<<256, 512, 152 * 1024>>>(p, ntiles, out); }},
  };
  hipStream_t s2[2];
  CK(hipStreamCreateWithFlags(&s2[0], hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2[1], hipStreamNonBlocking));
  u32* crc2; CK(hipMalloc(&crc2, 65536 * 4));
  int flip = 0;
  for (auto& L : libs) {
    vs.push_back({strdup(("crc " + L.path).c_str()), [&L, crc, msg, nmsg](const u32x4* p) {
                    L.uni(L.ctx, p, msg, msg, nmsg, 0xFFFFFFFFu, 1, crc, nullptr); }});
    // consecutive launches alternate between two streams (independent batches): the next
    // launch may start on CUs the previous one has released
    vs.push_back({strdup(("crc 2 streams " + L.path).c_str()), [&L, crc, crc2, &s2, &flip, msg, nmsg](const u32x4* p) {
                    flip ^= 1;
                    L.uni(L.ctx, p, msg, msg, nmsg, 0xFFFFFFFFu, 1, flip ? crc : crc2, s2[flip]); }});
  }
  for (int rep = 0; rep < 2; rep++)
    for (auto& v : vs) {
      u64 r = 0;
      auto t0 = std::chrono::steady_clock::now();
      while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 0.04) {
        for (int i = 0; i < 16; i++) v.f(buf + (r++ % nwin) * (win / 16));
        CK(hipDeviceSynchronize());
      }
      CK(hipDeviceSynchronize());
      const int n = 300;
      auto w0 = std::chrono::steady_clock::now();
      for (int i = 0; i < n; i++) v.f(buf + (r++ % nwin) * (win / 16));
      CK(hipDeviceSynchronize());
      const float ms = (float)std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
      printf("%-50s %7.2f us/launch %6.3f TB/s\n", v.name, ms * 1e3 / n, win / (ms * 1e-3 / n) / 1e12);
      fflush(stdout);
    }
  return 0;
}
