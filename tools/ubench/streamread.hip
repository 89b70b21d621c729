// HBM read ceilings per launch size (investigation tool): which load shape and grid a
// 256 MiB read-only launch can reach, with every launch reading a fresh window of a 4 GiB
// buffer (defeats the 256 MB MALL).
//   hipcc --offload-arch=gfx950 -O3 -o streamread streamread.hip && ./streamread
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)
typedef unsigned int u32;
typedef unsigned long long u64;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

// Coalesced: each wave instruction reads 1 KiB contiguous; a wave owns 8 KiB chunks in sweep order.
template <int WG>
__global__ __launch_bounds__(WG) void coalesced(const u32x4* __restrict__ p, u64 nchunks, u32* out) {
  const int lane = threadIdx.x & 63;
  const u64 w = (u64)blockIdx.x * (WG / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 nw = (u64)gridDim.x * (WG / 64);
  u32 acc = 0;
  for (u64 c = w; c < nchunks; c += nw) {
    const u32x4* q = p + c * 512 + lane;
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = q[i * 64];
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  }
  out[blockIdx.x * WG + threadIdx.x] = acc;
}

// Lane <-> 128-B line (the CRC kernels' shape): lane reads its 8 x 16 B line.
template <int WG>
__global__ __launch_bounds__(WG) void lines(const u32x4* __restrict__ p, u64 nchunks, u32* out) {
  const int lane = threadIdx.x & 63;
  const u64 w = (u64)blockIdx.x * (WG / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 nw = (u64)gridDim.x * (WG / 64);
  u32 acc = 0;
  for (u64 c = w; c < nchunks; c += nw) {
    const u32x4* q = p + c * 512 + lane * 8;
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = q[i];
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  }
  out[blockIdx.x * WG + threadIdx.x] = acc;
}

// Lines with the tile mapping of SUB-wave sub-blocks: wave (block b, wid) acts as wave
// wid%SUB of virtual block b + gridDim*(wid/SUB) -- the mapping a grid of 4x more, 4x
// smaller workgroups would get, inside one big workgroup.
template <int WG, int SUB>
__global__ __launch_bounds__(WG) void lines_remap(const u32x4* __restrict__ p, u64 nchunks, u32* out) {
  const int lane = threadIdx.x & 63;
  const u64 wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 vb = blockIdx.x + (u64)gridDim.x * (wid / SUB);
  const u64 w = vb * SUB + wid % SUB;
  const u64 nw = (u64)gridDim.x * (WG / 64);
  u32 acc = 0;
  for (u64 c = w; c < nchunks; c += nw) {
    const u32x4* q = p + c * 512 + lane * 8;
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = q[i];
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  }
  out[blockIdx.x * WG + threadIdx.x] = acc;
}

// lines_remap sub2 + the CRC kernels' result stores: every 4 tiles a wave stores the 8
// results of its last 4 tiles (2 adjacent words per tile) from 8 lanes (ST=1), as 4 u64
// pairs (ST=2), or not at all (ST=0: one store per wave at the end).
template <int WG, int ST>
__global__ __launch_bounds__(WG) void lines_store(const u32x4* __restrict__ p, u64 nchunks, u32* out, u32* res) {
  const int lane = threadIdx.x & 63;
  const u64 wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 w = ((u64)blockIdx.x + (u64)gridDim.x * (wid / 2)) * 2 + wid % 2;
  const u64 nw = (u64)gridDim.x * (WG / 64);
  u32 acc = 0;
  u64 k = 0;
  for (u64 c = w; c < nchunks; c += nw, k++) {
    const u32x4* q = p + c * 512 + lane * 8;
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = q[i];
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    if (ST && (k & 3) == 3) {
      const int M = lane >> 3;
      const u64 tile = c - (3 - (u64)(M >> 1)) * nw;  // tile of result slot M
      if (ST == 1) {
        if ((lane & 7) == 0) res[2 * tile + (M & 1)] = acc;
      } else {
        if ((lane & 15) == 0) *reinterpret_cast<unsigned long long*>(res + 2 * tile) = acc * 3ull;
      }
    }
  }
  out[blockIdx.x * WG + threadIdx.x] = acc;
}

// lines_remap sub2 shape with the CRC kernel's workgroup footprint: LDS (dynamic, 152 KiB
// at launch) and optionally FILL (128 KiB of LDS writes + barrier before the loop) and a
// CHAIN of dependent LDS round trips every 4 tiles (the combine tree's latency).
template <int WG, bool FILL, int CHAIN>
__global__ __launch_bounds__(WG) void lines_lds(const u32x4* __restrict__ p, u64 nchunks, u32* out) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  const int lane = threadIdx.x & 63;
  const u64 wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 w = ((u64)blockIdx.x + (u64)gridDim.x * (wid / 2)) * 2 + wid % 2;
  const u64 nw = (u64)gridDim.x * (WG / 64);
  if (FILL) {
    for (int i = threadIdx.x; i < 32768; i += WG) smem[i] = (u32)i * 2654435761u;
    __syncthreads();
  }
  u32 acc = 0;
  u64 k = 0;
  for (u64 c = w; c < nchunks; c += nw, k++) {
    const u32x4* q = p + c * 512 + lane * 8;
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = q[i];
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
    if (CHAIN && (k & 3) == 3) {
#pragma unroll
      for (int j = 0; j < CHAIN; j++) acc ^= smem[(acc ^ lane) & 32767];
    }
  }
  out[blockIdx.x * WG + threadIdx.x] = acc;
}

// Lines, but the 8 loads of a lane go out as 16-B pieces interleaved across lanes within
// 2 KiB: instruction i reads piece (i) of lines lane/... -- kept simple: lane reads its line
// as 2 x 64 B halves placed 4 KiB apart (two half-tiles), i.e. 32-B granularity per lane.
template <int WG>
__global__ __launch_bounds__(WG) void halflines(const u32x4* __restrict__ p, u64 nchunks, u32* out) {
  const int lane = threadIdx.x & 63;
  const u64 w = (u64)blockIdx.x * (WG / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const u64 nw = (u64)gridDim.x * (WG / 64);
  u32 acc = 0;
  for (u64 c = w; c < nchunks; c += nw) {
    // instruction i: lane l reads 16 B at ((i>>1)*64 + l)*32 + (i&1)*16 -> each instruction
    // covers 2 KiB in 32-B steps (half the lanes' bytes of a 64-B segment)
    const u32x4* q = p + c * 512;
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = q[((i >> 1) * 64 + lane) * 2 + (i & 1)];
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
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
  const u64 bytes = 4ull << 30, n16 = bytes / 16;
  u32x4* buf; CK(hipMalloc(&buf, bytes));
  u32* out; CK(hipMalloc(&out, 64ull << 20));
  u32* res; CK(hipMalloc(&res, (bytes / 4096) * 4 + 64));
  CK(hipFuncSetAttribute((const void*)lines_lds<512, false, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024));
  CK(hipFuncSetAttribute((const void*)lines_lds<512, true, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024));
  CK(hipFuncSetAttribute((const void*)lines_lds<512, true, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024));
  CK(hipFuncSetAttribute((const void*)lines_lds<512, true, 32>, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024));
  CK(hipFuncSetAttribute((const void*)lines_lds<512, true, 128>, hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024));
  gen<<<4096, 256>>>(buf, n16);
  CK(hipDeviceSynchronize());
  for (u64 win : {256ull << 20, 1ull << 30, 4ull << 30}) {
    const u64 chunks = win / 8192, nwin = bytes / win;
    u64 rot = 0;
    auto W = [&]() { return buf + (rot++ % nwin) * (win / 16); };
    auto rep = [&](const char* nm, float ms) {
      printf("%-28s %5llu MiB %8.1f us %6.2f TB/s\n", nm, win >> 20, ms * 1e3, win / (ms * 1e-3) / 1e12);
      fflush(stdout);
    };
#define RUN(K, WG, G) rep(#K " wg" #WG " grid" #G, time_it([&] { K<WG><<<G, WG>>>(W(), chunks, out); }, 32))
#define RUN2(WG, SUB, G) rep("lines_remap wg" #WG " sub" #SUB, time_it([&] { lines_remap<WG, SUB><<<G, WG>>>(W(), chunks, out); }, 32))
#define RUN3(ST) rep("lines_store st" #ST, time_it([&] { lines_store<512, ST><<<256, 512>>>(W(), chunks, out, res); }, 32))
#define RUN4(F, C) rep("lines_lds fill" #F " chain" #C, time_it([&] { lines_lds<512, F, C><<<256, 512, 152 * 1024>>>(W(), chunks, out); }, 32))
    RUN4(false, 0);
    RUN4(true, 0);
    RUN4(true, 8);
    RUN4(true, 32);
    RUN4(true, 128);
    RUN3(0);
    RUN3(1);
    RUN3(2);
    RUN(lines, 512, 256);
    RUN(lines, 256, 1024);
    RUN2(512, 2, 256);
  }
  return 0;
}
