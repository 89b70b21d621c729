// Design-space microbenchmark (investigation tool, not product code).
// Measures, on one MI355X, the HBM read rate of the load patterns a batched
// CRC32 kernel can use, and a first slice-by-4 CRC kernel built on the
// lane-contiguous-chunk pattern with 32-way replicated LDS tables.
//
//   hipcc --offload-arch=gfx950 -O3 -o ubench ubench.hip && ./ubench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <chrono>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

typedef unsigned int u32;
typedef unsigned long long u64;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

// ---------------------------------------------------------------- host CRC math
static u32 T[4][256];
static void host_tables() {
  for (u32 b = 0; b < 256; b++) {
    u32 c = b;
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    T[0][b] = c;
  }
  for (int k = 1; k < 4; k++)
    for (u32 b = 0; b < 256; b++) T[k][b] = (T[k - 1][b] >> 8) ^ T[0][T[k - 1][b] & 0xFF];
}
static u32 host_crc(u32 c, const uint8_t* p, size_t n) {
  for (size_t i = 0; i < n; i++) c = (c >> 8) ^ T[0][(c ^ p[i]) & 0xFF];
  return c;
}
// Z_n(c): advance raw state c over n zero bytes, as a 32x32 GF(2) matrix (columns).
struct Mat { u32 col[32]; };
static u32 apply(const Mat& m, u32 v) { u32 r = 0; for (int i = 0; i < 32; i++) if (v >> i & 1) r ^= m.col[i]; return r; }
static Mat zpow2(int bit) {  // matrix advancing over 2^bit zero bytes
  Mat m; for (int i = 0; i < 32; i++) { u32 c = 1u << i; c = (c >> 8) ^ T[0][c & 0xFF]; m.col[i] = c; }
  for (int s = 0; s < bit; s++) { Mat r; for (int i = 0; i < 32; i++) r.col[i] = apply(m, m.col[i]); m = r; }
  return m;
}

// ---------------------------------------------------------------- data gen
__global__ void gen(u32x4* p, u64 n16, u64 seed) {
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n16; i += (u64)gridDim.x * blockDim.x) {
    u64 z = seed + i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; z ^= z >> 31;
    u64 y = z * 0xD6E8FEB86659FD93ull; y ^= y >> 32;
    p[i] = u32x4{(u32)z, (u32)(z >> 32), (u32)y, (u32)(y >> 32)};
  }
}

// ---------------------------------------------------------------- load patterns
// P0: fully coalesced: each wave instruction reads 1 KiB contiguous.
__global__ __launch_bounds__(256) void p_coalesced(const u32x4* __restrict__ p, u64 n16, u32* out) {
  u32 acc = 0;
  const u64 stride = (u64)gridDim.x * 256 * 8;
  for (u64 base = blockIdx.x * 256ull * 8 + (threadIdx.x & ~63u) * 8 + (threadIdx.x & 63); base < n16; base += stride) {
    u32x4 v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = __builtin_nontemporal_load(p + base + j * 64);
#pragma unroll
    for (int j = 0; j < 8; j++) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// P1: lane-contiguous chunk of CHUNK bytes; burst of BURST x 16 B per lane.
template <int CHUNK, int BURST>
__global__ __launch_bounds__(256) void p_lanechunk(const u32x4* __restrict__ p, u64 n16, u32* out) {
  u32 acc = 0;
  constexpr int C16 = CHUNK / 16;
  const u64 nchunks = n16 / C16;
  const u64 gw = (blockIdx.x * 256ull + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * 4;
  const int lane = threadIdx.x & 63;
  for (u64 c0 = gw * 64; c0 < nchunks; c0 += nw * 64) {
    const u32x4* q = p + (c0 + lane) * C16;
    for (int t = 0; t < C16; t += BURST) {
      u32x4 v[BURST];
#pragma unroll
      for (int j = 0; j < BURST; j++) v[j] = q[t + j];
#pragma unroll
      for (int j = 0; j < BURST; j++) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// ---------------------------------------------------------------- CRC prototype
// LDS: 4 slice tables x 256 entries x 32 copies (one per bank) = 128 KiB.
// Entry e of table k, copy b at byte ((k>>1)<<16) | (e<<8) | ((k&1)<<7) | (b<<2).
// Table order: k=0 -> used for byte0 (T[3]), k=1 byte1 (T[2]), k=2 byte2 (T[1]), k=3 byte3 (T[0]).
__device__ __forceinline__ u32 lds_ld(u32 addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) u32*>(addr);
}

template <int CHUNK, bool PERM>
__global__ __launch_bounds__(1024) void crc_lanechunk(const u32x4* __restrict__ p, u64 nmsg, const u32* __restrict__ gtab,
                                                      const u32* __restrict__ ztab, u32 init, u32* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  // table fill: thread t -> (table k = t & 3, entry e = t >> 2)
  {
    const int t = threadIdx.x;
    const int k = t & 3, e = t >> 2;
    const u32 v = gtab[(3 - k) * 256 + e];
    u32x4 vv = {v, v, v, v};
    u32x4* dst = reinterpret_cast<u32x4*>(reinterpret_cast<char*>(smem) + (((k >> 1) << 16) | (e << 8) | ((k & 1) << 7)));
#pragma unroll
    for (int i = 0; i < 8; i++) dst[i] = vv;
  }
  __syncthreads();
  const u32 sbase = (u32)(uintptr_t)smem;
  const int lane = threadIdx.x & 63;
  const u32 lc0 = sbase + ((lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  constexpr int C16 = CHUNK / 16;
  constexpr int QPM = 4096 / CHUNK;  // lanes per 4 KiB message
  const u64 nchunks = nmsg * QPM;
  const u64 gw = (blockIdx.x * 1024ull + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * 16;
  const int j = lane % QPM;
  for (u64 c0 = gw * 64; c0 < nchunks; c0 += nw * 64) {
    const u32x4* q = p + (c0 + lane) * C16;
    u32 crc = (j == 0) ? init : 0u;
    for (int t = 0; t < C16; t += 8) {
      u32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = q[t + i];
#pragma unroll
      for (int i = 0; i < 8; i++) {
#pragma unroll
        for (int w = 0; w < 4; w++) {
          const u32 x = crc ^ v[i][w];
          u32 a0, a1, a2, a3;
          if (PERM) {
            // v_perm_b32: byte i of result = sel.byte[i] in 0..3 -> S1.byte, 4..7 -> S0.byte, 0x0c -> 0
            a0 = __builtin_amdgcn_perm(x, lc0, 0x0c020400u);
            a1 = __builtin_amdgcn_perm(x, lc0, 0x0c020500u);
            a2 = __builtin_amdgcn_perm(x, lc1, 0x0c020600u);
            a3 = __builtin_amdgcn_perm(x, lc1, 0x0c020700u);
          } else {
            a0 = ((x & 0xFFu) << 8) | lc0;
            a1 = (x & 0xFF00u) | lc0;
            a2 = ((x >> 8) & 0xFF00u) | lc1;
            a3 = ((x >> 16) & 0xFF00u) | lc1;
          }
          crc = lds_ld(a0) ^ lds_ld(a1 + 128) ^ lds_ld(a2) ^ lds_ld(a3 + 128);
        }
      }
    }
    // combine: multiply by x^(8*CHUNK*(QPM-1-j)) using Z_{2^b} tables (global)
    u32 d = (u32)(CHUNK * (QPM - 1 - j));
    while (d) {
      const int b = __builtin_ctz(d);
      d &= d - 1;
      const u32* z = ztab + b * 1024;
      crc = z[crc & 0xFF] ^ z[256 + ((crc >> 8) & 0xFF)] ^ z[512 + ((crc >> 16) & 0xFF)] ^ z[768 + (crc >> 24)];
    }
#pragma unroll
    for (int o = 1; o < QPM; o <<= 1) crc ^= __shfl_xor(crc, o);
    if (j == 0) out[(c0 + lane) / QPM] = crc;
  }
}


// P2: lane-contiguous chunk, but lane i walks its chunk's 128-B lines starting at line (i mod LPC)
template <int CHUNK>
__global__ __launch_bounds__(256) void p_lanechunk_rot(const u32x4* __restrict__ p, u64 n16, u32* out) {
  u32 acc = 0;
  constexpr int C16 = CHUNK / 16, LPC = CHUNK / 128;
  const u64 nchunks = n16 / C16;
  const u64 gw = (blockIdx.x * 256ull + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * 4;
  const int lane = threadIdx.x & 63;
  const int r = lane % LPC;
  for (u64 c0 = gw * 64; c0 < nchunks; c0 += nw * 64) {
    const u32x4* q = p + (c0 + lane) * C16;
    for (int t = 0; t < LPC; t++) {
      const int line = (r + t) % LPC;
      u32x4 v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = q[line * 8 + j];
#pragma unroll
      for (int j = 0; j < 8; j++) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__device__ __forceinline__ u32 zmul(const u32* z, u32 c) {
  return z[c & 0xFF] ^ z[256 + ((c >> 8) & 0xFF)] ^ z[512 + ((c >> 16) & 0xFF)] ^ z[768 + (c >> 24)];
}

// CRC over lane-contiguous chunks with rotated line order; ztab: Z_{2^b} (32 ops), zline: Z_{128*k} k=0..LPC
template <int CHUNK, int WG>
__global__ __launch_bounds__(WG) void crc_rot(const u32x4* __restrict__ p, u64 nmsg, const u32* __restrict__ gtab,
                                              const u32* __restrict__ ztab, const u32* __restrict__ zline, u32 init,
                                              u32* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  for (int t = threadIdx.x; t < 1024; t += WG) {
    const int k = t & 3, e = t >> 2;
    const u32 v = gtab[(3 - k) * 256 + e];
    u32x4 vv = {v, v, v, v};
    u32x4* dst = reinterpret_cast<u32x4*>(reinterpret_cast<char*>(smem) + (((k >> 1) << 16) | (e << 8) | ((k & 1) << 7)));
#pragma unroll
    for (int i = 0; i < 8; i++) dst[i] = vv;
  }
  __syncthreads();
  const u32 sbase = (u32)(uintptr_t)smem;
  const int lane = threadIdx.x & 63;
  const u32 lc0 = sbase + ((lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  constexpr int C16 = CHUNK / 16, LPC = CHUNK / 128;
  constexpr int QPM = 4096 / CHUNK;
  const u64 nchunks = nmsg * QPM;
  const u64 gw = (blockIdx.x * (u64)WG + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * (WG / 64);
  const int j = lane % QPM;
  const int r = lane % LPC;
  for (u64 c0 = gw * 64; c0 < nchunks; c0 += nw * 64) {
    const u32x4* q = p + (c0 + lane) * C16;
    const u32 s0 = (j == 0) ? init : 0u;
    u32 crc = (r == 0) ? s0 : 0u;
    u32 sA = 0;
    for (int t = 0; t < LPC; t++) {
      const int line = (r + t) % LPC;
      if (line == 0 && t != 0) { sA = crc; crc = s0; }
      u32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = q[line * 8 + i];
#pragma unroll
      for (int i = 0; i < 8; i++) {
#pragma unroll
        for (int w = 0; w < 4; w++) {
          const u32 x = crc ^ v[i][w];
          const u32 a0 = __builtin_amdgcn_perm(x, lc0, 0x0c020400u);
          const u32 a1 = __builtin_amdgcn_perm(x, lc0, 0x0c020500u);
          const u32 a2 = __builtin_amdgcn_perm(x, lc1, 0x0c020600u);
          const u32 a3 = __builtin_amdgcn_perm(x, lc1, 0x0c020700u);
          crc = lds_ld(a0) ^ lds_ld(a1 + 128) ^ lds_ld(a2) ^ lds_ld(a3 + 128);
        }
      }
    }
    if (r != 0) crc = zmul(zline + (LPC - r) * 1024, crc) ^ sA;
    u32 d = (u32)(CHUNK * (QPM - 1 - j));
    while (d) {
      const int b = __builtin_ctz(d);
      d &= d - 1;
      crc = zmul(ztab + b * 1024, crc);
    }
#pragma unroll
    for (int o = 1; o < QPM; o <<= 1) crc ^= __shfl_xor(crc, o);
    if (j == 0) out[(c0 + lane) / QPM] = crc;
  }
}


__device__ __forceinline__ void fill_tables(u32* smem, const u32* gtab, int tid, int nthr) {
  for (int t = tid; t < 1024; t += nthr) {
    const int k = t & 3, e = t >> 2;
    const u32 v = gtab[(3 - k) * 256 + e];
    u32x4 vv = {v, v, v, v};
    u32x4* dst = reinterpret_cast<u32x4*>(reinterpret_cast<char*>(smem) + (((k >> 1) << 16) | (e << 8) | ((k & 1) << 7)));
#pragma unroll
    for (int i = 0; i < 8; i++) dst[i] = vv;
  }
}
__device__ __forceinline__ u32 step4(u32 x, u32 lc0, u32 lc1) {
  const u32 a0 = __builtin_amdgcn_perm(x, lc0, 0x0c020400u);
  const u32 a1 = __builtin_amdgcn_perm(x, lc0, 0x0c020500u);
  const u32 a2 = __builtin_amdgcn_perm(x, lc1, 0x0c020600u);
  const u32 a3 = __builtin_amdgcn_perm(x, lc1, 0x0c020700u);
  return lds_ld(a0) ^ lds_ld(a1 + 128) ^ lds_ld(a2) ^ lds_ld(a3 + 128);
}

// V_A: config-B shape. lane <-> 128-B line of an 8 KiB tile (2 messages per tile).
// zA: Z_{128a} a=0..7 ; zB: Z_{1024b} b=0..7 (identity at 0), global memory.
template <int WG>
__global__ __launch_bounds__(WG) void crc_tileline(const u32x4* __restrict__ p, u64 nmsg, const u32* __restrict__ gtab,
                                                   const u32* __restrict__ zA, const u32* __restrict__ zB, u32 init,
                                                   u32* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  fill_tables(smem, gtab, threadIdx.x, WG);
  __syncthreads();
  const u32 sbase = (u32)(uintptr_t)smem;
  const int lane = threadIdx.x & 63;
  const u32 lc0 = sbase + ((lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  const int li = lane & 31;
  const u64 ntiles = nmsg / 2;
  const u64 gw = (blockIdx.x * (u64)WG + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * (WG / 64);
  const u32* za = zA + ((31 - li) & 7) * 1024;
  const u32* zb = zB + ((31 - li) >> 3) * 1024;
  for (u64 t = gw; t < ntiles; t += nw) {
    const u32x4* q = p + t * 512 + lane * 8;
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = q[i];
    u32 crc = (li == 0) ? init : 0u;
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int w = 0; w < 4; w++) crc = step4(crc ^ v[i][w], lc0, lc1);
    crc = zmul(za, crc);
    crc = zmul(zb, crc);
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) crc ^= __shfl_xor(crc, o);
    if (li == 0) out[t * 2 + (lane >> 5)] = crc;
  }
}

// V_D: large-message shape. wave run = RT tiles of 8 KiB; lane <-> line i of each tile;
// the last word of each line (except the run's last) uses jump tables J4 = Z_8064 o T4 (LDS, not replicated).
// Output: raw CRC (init 0) of each run.
template <int WG, int RT>
__global__ __launch_bounds__(WG) void crc_tilejump(const u32x4* __restrict__ p, u64 nruns, const u32* __restrict__ gtab,
                                                   const u32* __restrict__ jtab, const u32* __restrict__ zA,
                                                   const u32* __restrict__ zB, u32* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  fill_tables(smem, gtab, threadIdx.x, WG);
  for (int t = threadIdx.x; t < 1024; t += WG) smem[32768 + t] = jtab[t];
  __syncthreads();
  const u32 sbase = (u32)(uintptr_t)smem;
  const int lane = threadIdx.x & 63;
  const u32 lc0 = sbase + ((lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  const u32 jb = sbase + 131072;
  const u64 gw = (blockIdx.x * (u64)WG + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * (WG / 64);
  const u32* za = zA + ((63 - lane) & 7) * 1024;
  const u32* zb = zB + ((63 - lane) >> 3) * 1024;
  for (u64 r = gw; r < nruns; r += nw) {
    const u32x4* q = p + r * (512 * RT) + lane * 8;
    u32 crc = 0;
    for (int t = 0; t < RT; t++) {
      u32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = q[t * 512 + i];
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int w = 0; w < 4; w++) {
          if (i == 7 && w == 3) {
            const u32 x = crc ^ v[i][w];
            if (t + 1 < RT) {
              crc = lds_ld(jb + ((x & 0xFF) << 2)) ^ lds_ld(jb + 1024 + ((x >> 6) & 0x3FC)) ^
                    lds_ld(jb + 2048 + ((x >> 14) & 0x3FC)) ^ lds_ld(jb + 3072 + ((x >> 22) & 0x3FC));
            } else {
              crc = step4(x, lc0, lc1);
            }
          } else {
            crc = step4(crc ^ v[i][w], lc0, lc1);
          }
        }
    }
    crc = zmul(za, crc);
    crc = zmul(zb, crc);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) crc ^= __shfl_xor(crc, o);
    if (lane == 0) out[r] = crc;
  }
}

// ---------------------------------------------------------------- driver
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

int main(int argc, char** argv) {
  host_tables();
  const u64 bytes = (argc > 1 ? strtoull(argv[1], 0, 0) : 4ull) << 30;
  const u64 n16 = bytes / 16;
  u32x4* buf; CK(hipMalloc(&buf, bytes));
  u32* out; CK(hipMalloc(&out, 64ull << 20));
  gen<<<4096, 256>>>(buf, n16, 0x5EED000Bull);
  CK(hipDeviceSynchronize());
  const int iters = 10;
  auto report = [&](const char* name, float ms) {
    double gibs = bytes / (ms * 1e-3) / (1024.0 * 1024 * 1024);
    printf("%-28s %8.3f ms  %8.1f GiB/s  %6.2f TB/s  %5.1f%% of 8TB/s\n", name, ms, gibs, bytes / (ms * 1e-3) / 1e12,
           100.0 * bytes / (ms * 1e-3) / 8e12);
    fflush(stdout);
  };
  int nblk[] = {1024, 2048, 4096};
  for (int nb : nblk) {
    char nm[64];
    snprintf(nm, 64, "coalesced nb=%d", nb);
    report(nm, time_it([&] { p_coalesced<<<nb, 256>>>(buf, n16, out); }, iters));
  }
  report("lanechunk 1K burst8", time_it([&] { p_lanechunk<1024, 8><<<2048, 256>>>(buf, n16, out); }, iters));
  report("lanechunk 1K burst4", time_it([&] { p_lanechunk<1024, 4><<<2048, 256>>>(buf, n16, out); }, iters));
  report("lanechunk 4K burst8", time_it([&] { p_lanechunk<4096, 8><<<2048, 256>>>(buf, n16, out); }, iters));
  report("lanechunk 256 burst8", time_it([&] { p_lanechunk<256, 8><<<2048, 256>>>(buf, n16, out); }, iters));
  report("lanechunk rot 1K", time_it([&] { p_lanechunk_rot<1024><<<2048, 256>>>(buf, n16, out); }, iters));
  report("lanechunk rot 2K", time_it([&] { p_lanechunk_rot<2048><<<2048, 256>>>(buf, n16, out); }, iters));
  report("lanechunk rot 4K", time_it([&] { p_lanechunk_rot<4096><<<2048, 256>>>(buf, n16, out); }, iters));
  report("lanechunk 128 burst8", time_it([&] { p_lanechunk<128, 8><<<2048, 256>>>(buf, n16, out); }, iters));

  // CRC prototype
  std::vector<u32> gt(1024);
  for (int k = 0; k < 4; k++) for (int b = 0; b < 256; b++) gt[k * 256 + b] = T[k][b];
  std::vector<u32> zt(32 * 1024);
  for (int bit = 0; bit < 32; bit++) {
    Mat m = zpow2(bit);
    for (int k = 0; k < 4; k++)
      for (u32 b = 0; b < 256; b++) zt[bit * 1024 + k * 256 + b] = apply(m, b << (8 * k));
  }
  u32 *dgt, *dzt; CK(hipMalloc(&dgt, 4096)); CK(hipMalloc(&dzt, zt.size() * 4));
  CK(hipMemcpy(dgt, gt.data(), 4096, hipMemcpyHostToDevice));
  CK(hipMemcpy(dzt, zt.data(), zt.size() * 4, hipMemcpyHostToDevice));
  const u64 nmsg = bytes / 4096;
  std::vector<u32> zl(33 * 1024);
  {
    Mat m1 = zpow2(7);  // 128 bytes
    Mat acc; for (int i = 0; i < 32; i++) acc.col[i] = 1u << i;  // identity
    for (int k = 0; k <= 32; k++) {
      for (int kk = 0; kk < 4; kk++) for (u32 b = 0; b < 256; b++) zl[k * 1024 + kk * 256 + b] = apply(acc, b << (8 * kk));
      Mat r; for (int i = 0; i < 32; i++) r.col[i] = apply(m1, acc.col[i]); acc = r;
    }
  }
  u32* dzl; CK(hipMalloc(&dzl, zl.size() * 4));
  CK(hipMemcpy(dzl, zl.data(), zl.size() * 4, hipMemcpyHostToDevice));
  // zA: Z_{128a}, zB: Z_{1024b}; jtab: Z_8064 o T4 with layout [k][byte] for byte k of x (k=0 lowest)
  std::vector<u32> zA(8 * 1024), zB(8 * 1024), jt(1024);
  for (int a = 0; a < 8; a++) for (int i = 0; i < 1024; i++) zA[a * 1024 + i] = zl[a * 1024 + i];
  for (int b = 0; b < 8; b++) for (int i = 0; i < 1024; i++) zB[b * 1024 + i] = zl[8 * b * 1024 + i];
  {
    // J4(x) = Z_8064(T4(x)); T4 of byte k value v: T[3-k][v]
    Mat mj; { Mat m1 = zpow2(7); Mat acc; for (int i = 0; i < 32; i++) acc.col[i] = 1u << i;
      for (int k = 0; k < 63; k++) { Mat r; for (int i = 0; i < 32; i++) r.col[i] = apply(m1, acc.col[i]); acc = r; } mj = acc; }
    for (int k = 0; k < 4; k++) for (u32 b = 0; b < 256; b++) jt[k * 256 + b] = apply(mj, T[3 - k][b]);
  }
  u32 *dzA, *dzB, *djt;
  CK(hipMalloc(&dzA, zA.size() * 4)); CK(hipMalloc(&dzB, zB.size() * 4)); CK(hipMalloc(&djt, 4096));
  CK(hipMemcpy(dzA, zA.data(), zA.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dzB, zB.data(), zB.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(djt, jt.data(), 4096, hipMemcpyHostToDevice));
  std::vector<uint8_t> msg(4096);
  int total_bad = 0;
  auto verify = [&](const char* name) {
    CK(hipDeviceSynchronize());
    std::vector<u32> got(nmsg);
    CK(hipMemcpy(got.data(), out, got.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0, checked = 0;
    for (u64 m = 0; m < got.size(); m += 9973) {
      CK(hipMemcpy(msg.data(), (char*)buf + m * 4096, 4096, hipMemcpyDeviceToHost));
      u32 want = host_crc(0xFFFFFFFFu, msg.data(), 4096);
      if (want != got[m]) { if (bad < 3) printf("  %s mismatch msg %llu got %08x want %08x\n", name, m, got[m], want); bad++; }
      checked++;
    }
    printf("  %s verify: %d/%d mismatches\n", name, bad, checked);
    total_bad += bad;
  };
#define RUN_CRC(C, P, NB, NAME) do { \
    CK(hipFuncSetAttribute((const void*)crc_lanechunk<C, P>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072)); \
    CK(hipMemset(out, 0, nmsg * 4)); \
    report(NAME, time_it([&] { crc_lanechunk<C, P><<<NB, 1024, 131072>>>(buf, nmsg, dgt, dzt, 0xFFFFFFFFu, out); }, iters)); \
    verify(NAME); } while (0)
#define RUN_ROT(C, WG, NB, NAME) do { \
    CK(hipFuncSetAttribute((const void*)crc_rot<C, WG>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072)); \
    CK(hipMemset(out, 0, nmsg * 4)); \
    report(NAME, time_it([&] { crc_rot<C, WG><<<NB, WG, 131072>>>(buf, nmsg, dgt, dzt, dzl, 0xFFFFFFFFu, out); }, iters)); \
    verify(NAME); } while (0)
#define RUN_TL(WG, NAME) do { \
    CK(hipFuncSetAttribute((const void*)crc_tileline<WG>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072)); \
    CK(hipMemset(out, 0, nmsg * 4)); \
    report(NAME, time_it([&] { crc_tileline<WG><<<256, WG, 131072>>>(buf, nmsg, dgt, dzA, dzB, 0xFFFFFFFFu, out); }, iters)); \
    verify(NAME); } while (0)
  RUN_TL(256, "crc tileline wg256");
  RUN_TL(512, "crc tileline wg512");
  RUN_TL(1024, "crc tileline wg1024");
  {
    const int RT = 8;
    const u64 nruns = bytes / (8192 * RT);
    CK(hipFuncSetAttribute((const void*)crc_tilejump<512, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072 + 4096));
    CK(hipFuncSetAttribute((const void*)crc_tilejump<1024, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072 + 4096));
    for (int wg : {512, 1024}) {
      CK(hipMemset(out, 0, nruns * 4));
      char nm[64]; snprintf(nm, 64, "crc tilejump RT8 wg%d", wg);
      if (wg == 512) report(nm, time_it([&] { crc_tilejump<512, 8><<<256, 512, 131072 + 4096>>>(buf, nruns, dgt, djt, dzA, dzB, out); }, iters));
      else report(nm, time_it([&] { crc_tilejump<1024, 8><<<256, 1024, 131072 + 4096>>>(buf, nruns, dgt, djt, dzA, dzB, out); }, iters));
      CK(hipDeviceSynchronize());
      std::vector<u32> got(nruns);
      CK(hipMemcpy(got.data(), out, nruns * 4, hipMemcpyDeviceToHost));
      std::vector<uint8_t> run(8192 * RT);
      int bad = 0, checked = 0;
      for (u64 m = 0; m < nruns; m += 4099) {
        CK(hipMemcpy(run.data(), (char*)buf + m * run.size(), run.size(), hipMemcpyDeviceToHost));
        u32 want = host_crc(0u, run.data(), run.size());
        if (want != got[m]) { if (bad < 3) printf("  mismatch run %llu got %08x want %08x\n", m, got[m], want); bad++; }
        checked++;
      }
      printf("  %s verify: %d/%d mismatches\n", nm, bad, checked);
      total_bad += bad;
    }
  }
  RUN_ROT(1024, 1024, 256, "crc rot 1K wg1024");
  RUN_ROT(2048, 1024, 256, "crc rot 2K wg1024");
  RUN_ROT(4096, 1024, 256, "crc rot 4K wg1024");
  RUN_ROT(1024, 512, 256, "crc rot 1K wg512");
  RUN_ROT(1024, 768, 256, "crc rot 1K wg768");
  RUN_CRC(1024, false, 256, "crc 1K nb256");
    RUN_CRC(1024, true, 256, "crc 1K perm nb256");
  RUN_CRC(512, true, 256, "crc 512 perm");
  RUN_CRC(2048, true, 256, "crc 2K perm");
  return total_bad ? 1 : 0;
}
