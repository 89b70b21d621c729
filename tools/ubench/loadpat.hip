// Load-pattern sweep (investigation tool). Pure-read kernels that differ only in
// which 16-B pieces each lane reads, to find the access shapes that run near the
// coalesced HBM rate on MI355X.
//   hipcc --offload-arch=gfx950 -O3 -o loadpat loadpat.hip && ./loadpat
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)
typedef unsigned int u32;
typedef unsigned long long u64;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

__global__ void gen(u32x4* p, u64 n16) {
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n16; i += (u64)gridDim.x * blockDim.x)
    p[i] = u32x4{(u32)i, (u32)(i >> 7), (u32)(i * 3), (u32)(i * 5)};
}

// Lane-contiguous chunk of CHUNK bytes, walked line by line (8 x 16 B per line).
template <int CHUNK, int WG>
__global__ __launch_bounds__(WG) void lanechunk(const u32x4* __restrict__ p, u64 n16, u32* out) {
  u32 acc = 0;
  constexpr int C16 = CHUNK / 16;
  const u64 nchunks = n16 / C16;
  const u64 gw = (blockIdx.x * (u64)WG + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * (WG / 64);
  const int lane = threadIdx.x & 63;
  for (u64 c0 = gw * 64; c0 < nchunks; c0 += nw * 64) {
    const u32x4* q = p + (c0 + lane) * C16;
    for (int t = 0; t < C16; t += 8) {
      u32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = q[t + j];
#pragma unroll
      for (int j = 0; j < 8; j++) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
  }
  out[blockIdx.x * WG + threadIdx.x] = acc;
}

// Tile-line: lane i reads line i of NT consecutive 8 KiB tiles. ORDER 0: tile-outer
// (8 loads per tile back to back); ORDER 1: piece-outer (for j: for t: tile t piece j).
template <int NT, int ORDER, int WG>
__global__ __launch_bounds__(WG) void tileline(const u32x4* __restrict__ p, u64 n16, u32* out) {
  u32 acc = 0;
  const u64 ngroups = n16 / (512 * NT);
  const u64 gw = (blockIdx.x * (u64)WG + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * (WG / 64);
  const int lane = threadIdx.x & 63;
  for (u64 g = gw; g < ngroups; g += nw) {
    const u32x4* q = p + g * 512 * NT + lane * 8;
    u32x4 v[NT * 8];
    if (ORDER == 0) {
#pragma unroll
      for (int t = 0; t < NT; t++)
#pragma unroll
        for (int j = 0; j < 8; j++) v[t * 8 + j] = q[t * 512 + j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; j++)
#pragma unroll
        for (int t = 0; t < NT; t++) v[t * 8 + j] = q[t * 512 + j];
    }
#pragma unroll
    for (int j = 0; j < NT * 8; j++) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  }
  out[blockIdx.x * WG + threadIdx.x] = acc;
}

// Strided single line: lane i reads one 128-B line at g*64*S + i*S (S bytes apart); tiles walk the buffer
// so every byte is read once when S divides... only S=128 covers all bytes; others read 128/S of the data,
// and we report bytes actually read.
template <int S, int WG>
__global__ __launch_bounds__(WG) void strideline(const u32x4* __restrict__ p, u64 n16, u32* out) {
  u32 acc = 0;
  constexpr int S16 = S / 16;
  const u64 ngroups = n16 / (64 * S16);
  const u64 gw = (blockIdx.x * (u64)WG + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * (WG / 64);
  const int lane = threadIdx.x & 63;
  for (u64 g = gw; g < ngroups; g += nw) {
    const u32x4* q = p + g * 64 * S16 + lane * S16;
    u32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = q[j];
#pragma unroll
    for (int j = 0; j < 8; j++) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
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

int main() {
  const u64 bytes = 4ull << 30, n16 = bytes / 16;
  u32x4* buf; CK(hipMalloc(&buf, bytes));
  u32* out; CK(hipMalloc(&out, 64ull << 20));
  gen<<<4096, 256>>>(buf, n16);
  CK(hipDeviceSynchronize());
  auto rep = [&](const char* nm, float ms, double frac) {
    printf("%-34s %7.3f ms %6.2f TB/s\n", nm, ms, bytes * frac / (ms * 1e-3) / 1e12); fflush(stdout);
  };
#define LC(C, WG, NB) rep("lanechunk " #C " wg" #WG " nb" #NB, time_it([&] { lanechunk<C, WG><<<NB, WG>>>(buf, n16, out); }, 10), 1.0)
  LC(128, 256, 2048); LC(256, 256, 2048); LC(512, 256, 2048); LC(1024, 256, 2048); LC(2048, 256, 2048);
  LC(4096, 256, 2048); LC(8192, 256, 2048); LC(16384, 256, 2048);
  LC(1024, 256, 512); LC(1024, 256, 1024); LC(1024, 512, 256); LC(1024, 1024, 256); LC(1024, 64, 4096);
  LC(4096, 512, 256); LC(128, 512, 256);
#define TL(NT, O, WG, NB) rep("tileline nt" #NT " o" #O " wg" #WG " nb" #NB, time_it([&] { tileline<NT, O, WG><<<NB, WG>>>(buf, n16, out); }, 10), 1.0)
  TL(1, 0, 256, 2048); TL(2, 0, 256, 2048); TL(4, 0, 256, 2048); TL(2, 1, 256, 2048); TL(4, 1, 256, 2048);
  TL(1, 0, 512, 256); TL(2, 0, 512, 256); TL(4, 1, 512, 256); TL(1, 0, 1024, 256);
#define SL(S) rep("strideline " #S, time_it([&] { strideline<S, 256><<<2048, 256>>>(buf, n16, out); }, 10), 128.0 / S)
  SL(128); SL(256); SL(512); SL(1024); SL(2048); SL(4096); SL(8192);
  return 0;
}
