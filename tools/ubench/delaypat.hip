// Memory-side model of the CRC kernels (investigation tool): each wave streams 8 KiB
// tiles in sweep order (lane <-> 128-B line), keeps DEPTH tiles of loads in flight, and
// "computes" for SLEEP x 64 cycles per tile (s_sleep) instead of running the CRC.
//   hipcc --offload-arch=gfx950 -O3 -o delaypat delaypat.hip && ./delaypat
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)
typedef unsigned int u32;
typedef unsigned long long u64;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

template <int SLEEP>
__device__ __forceinline__ void fake_compute() {
#pragma unroll
  for (int i = 0; i < SLEEP; i++) __builtin_amdgcn_s_sleep(1);  // ~64 cycles each
}

template <int WG, int DEPTH, int SLEEP>
__global__ __launch_bounds__(WG) void delaypat(const u32x4* __restrict__ p, u64 ntiles, u32* out) {
  const int lane = threadIdx.x & 63;
  const u64 w = (u64)blockIdx.x * (WG / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 nw = (u64)gridDim.x * (WG / 64);
  const u64 nk = w < ntiles ? (ntiles - w + nw - 1) / nw : 0;
  if (nk == 0) return;
  u32 acc = 0;
  u32x4 buf[DEPTH + 1][8];
  auto ld = [&](int slot, u64 k) {
    const u64 kk = k < nk ? k : nk - 1;
    const u32x4* q = p + (kk * nw + w) * 512 + lane * 8;
#pragma unroll
    for (int i = 0; i < 8; i++) buf[slot][i] = q[i];
    __builtin_amdgcn_sched_barrier(0);
  };
#pragma unroll
  for (int d = 0; d < DEPTH; d++) ld(d, d);
  for (u64 k = 0; k < nk; k += DEPTH + 1) {
#pragma unroll
    for (int s = 0; s <= DEPTH; s++) {
      if (k + s >= nk) break;
      ld((s + DEPTH) % (DEPTH + 1), k + s + DEPTH);
#pragma unroll
      for (int i = 0; i < 8; i++) acc ^= buf[s][i].x ^ buf[s][i].y ^ buf[s][i].z ^ buf[s][i].w;
      fake_compute<SLEEP>();
    }
  }
  out[blockIdx.x * WG + threadIdx.x] = acc;
}

template <typename F>
static float time_it(F f, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; i++) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

__global__ void gen(u32x4* p, u64 n16) {
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n16; i += (u64)gridDim.x * blockDim.x)
    p[i] = u32x4{(u32)i, (u32)(i >> 7), (u32)(i * 3), (u32)(i * 5)};
}

int main() {
  const u64 bytes = 4ull << 30, n16 = bytes / 16, ntiles = bytes / 8192;
  u32x4* buf; CK(hipMalloc(&buf, bytes));
  u32* out; CK(hipMalloc(&out, 64ull << 20));
  gen<<<4096, 256>>>(buf, n16);
  CK(hipDeviceSynchronize());
  u64 cur_bytes = bytes, cur_tiles = ntiles;
  auto rep = [&](const char* nm, float ms) { printf("%-28s %5llu MiB %8.1f us %6.2f TB/s\n", nm, cur_bytes >> 20, ms * 1e3, cur_bytes / (ms * 1e-3) / 1e12); fflush(stdout); };
  // each launch reads the next cur_bytes window of the 4 GiB buffer (rotation defeats the 256 MB MALL)
  u64 rot = 0;
  auto win = [&]() { const u64 nwin = bytes / cur_bytes; return buf + ((rot++ % nwin) * (cur_bytes / 16)); };
#define R(WG, D, S) rep("wg" #WG " depth" #D " sleep" #S, time_it([&] { delaypat<WG, D, S><<<256, WG>>>(win(), cur_tiles, out); }, 32))
  // sleep 24 x ~64 cycles ~= 1500 cycles ~ the CRC's per-tile compute latency
  R(512, 1, 0); R(512, 1, 24); R(512, 2, 24); R(512, 3, 24);
  R(768, 1, 24); R(768, 2, 24);
  R(1024, 1, 24); R(1024, 2, 24);
  R(256, 2, 24); R(256, 3, 24);
  R(512, 1, 48); R(512, 2, 48); R(1024, 1, 48); R(1024, 2, 48);
  // the bench's batch size (256 MiB): fixed per-launch cost shows here
  cur_bytes = 256ull << 20; cur_tiles = cur_bytes / 8192;
  R(512, 1, 0); R(512, 1, 24); R(512, 2, 24); R(768, 1, 24); R(1024, 1, 24); R(1024, 2, 24); R(256, 3, 24);
  return 0;
}
