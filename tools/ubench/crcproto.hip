// CRC kernel prototypes (investigation tool). Lane <-> 128-B line of an 8 KiB tile
// (the access shape that runs near the coalesced rate), slice-by-4 steps from
// 32-way replicated byte tables, and GF(2) combine operators as conflict-free
// nibble tables (8 x 16 entries = 512 B per operator).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)
typedef unsigned int u32;
typedef unsigned long long u64;
using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;

// ---------------------------------------------------------------- host math
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
struct Mat { u32 col[32]; };
static u32 apply(const Mat& m, u32 v) { u32 r = 0; for (int i = 0; i < 32; i++) if (v >> i & 1) r ^= m.col[i]; return r; }
static Mat mul(const Mat& a, const Mat& b) { Mat r; for (int i = 0; i < 32; i++) r.col[i] = apply(a, b.col[i]); return r; }
static Mat ident() { Mat m; for (int i = 0; i < 32; i++) m.col[i] = 1u << i; return m; }
static Mat zbytes(u64 n) {  // advance over n zero bytes
  Mat one; for (int i = 0; i < 32; i++) { u32 c = 1u << i; one.col[i] = (c >> 8) ^ T[0][c & 0xFF]; }
  Mat r = ident(), p = one;
  while (n) { if (n & 1) r = mul(p, r); p = mul(p, p); n >>= 1; }
  return r;
}
static Mat t4mat() { Mat m; for (int i = 0; i < 32; i++) { u32 c = 1u << i; m.col[i] = T[3][c & 0xFF] ^ T[2][(c >> 8) & 0xFF] ^ T[1][(c >> 16) & 0xFF] ^ T[0][c >> 24]; } return m; }
static void nib(const Mat& m, u32* out) { for (int k = 0; k < 8; k++) for (u32 n = 0; n < 16; n++) out[k * 16 + n] = apply(m, n << (4 * k)); }

// ---------------------------------------------------------------- device helpers
typedef __attribute__((address_space(3))) u32 lds_u32;
__device__ __forceinline__ u32 lds_ld(u32 addr) { return *reinterpret_cast<const lds_u32*>(addr); }
__device__ __forceinline__ void lds_st(u32 addr, u32 v) { *reinterpret_cast<lds_u32*>(addr) = v; }
__device__ __forceinline__ u32x4 lds_ld4(u32 addr) {
  return *reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(addr);
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
// GF(2) operator from nibble tables at LDS byte address `op` (8 tables x 16 dwords).
__device__ __forceinline__ u32 nmul(u32 op, u32 v) {
  u32 r = lds_ld(op + ((v << 2) & 0x3C));
#pragma unroll
  for (int k = 1; k < 8; k++) r ^= lds_ld(op + 64 * k + ((v >> (4 * k - 2)) & 0x3C));
  return r;
}
__device__ __forceinline__ u32 shfl_down(u32 v, int d) { return __shfl_down(v, d); }

#define OPS_OFF 131072
// operator slots (512 B each): 0 Z128, 1 Z256, 2 Z512, 3 Z1024, 4 Z2048, 5 Z4096, 6 J (Z8064 o T4)
#define OP(i) (sbase + OPS_OFF + 512 * (i))
#define XPOSE_OFF (OPS_OFF + 8192)

// K1: uniform 4 KiB messages. Wave group = 8 messages (4 tiles of 8 KiB).
// Lane i <-> line (i&31) of message 2t + (i>>5). Partials transposed through LDS,
// then a tree: within lane (4 lines), across 8 lanes.
template <int WG, bool PREFETCH, int MODE = 0>
__global__ __launch_bounds__(WG) void crc_uniform4k(const u32x4* __restrict__ p, u64 nmsg, const u32* __restrict__ gtab,
                                                    const u32* __restrict__ gops, u32 init, u32* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  fill_tables(smem, gtab, threadIdx.x, WG);
  for (int t = threadIdx.x; t < 2048; t += WG) smem[OPS_OFF / 4 + t] = gops[t];
  __syncthreads();
  const u32 sbase = (u32)(uintptr_t)smem;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const u32 lc0 = sbase + ((lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  const u32 xb = sbase + XPOSE_OFF + wid * 1024;
  const int l = lane & 31, h = lane >> 5;
  const u64 ngroups = nmsg / 8;
  const u64 gw = (blockIdx.x * (u64)WG + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * (WG / 64);
  const u32 s_init = (l == 0) ? init : 0u;
  for (u64 g = gw; g < ngroups; g += nw) {
    // MODE 3/4: sweep order -- the 4 tiles of this wave's group are (4k+t)*NW + w, so all waves
    // together read one compact front of memory. q points at tile 0, tile t at q + tstride*t.
    const u64 k4 = (g - gw) / nw;
    const bool sweep = (MODE == 3 || MODE == 4);
    const u32x4* q = sweep ? p + ((4 * k4) * nw + gw) * 512 + lane * 8
                           : p + (MODE == 2 ? (g & 255) : g) * 2048 + lane * 8;
    const u64 tstride = sweep ? nw * 512 : 512;
    u32 part[4];
    u32x4 v[8], nv[8];
    if (PREFETCH) {
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = q[i];
    }
#pragma unroll
    for (int t = 0; t < 4; t++) {
      if (PREFETCH) {
        if (t < 3) {
#pragma unroll
          for (int i = 0; i < 8; i++) nv[i] = q[(t + 1) * tstride + i];
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = q[t * tstride + i];
      }
      u32 crc = s_init;
      if (MODE == 1 || MODE == 4) {
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
          for (int w = 0; w < 4; w++) crc = (crc << 1 | crc >> 31) ^ v[i][w];
      } else {
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
          for (int w = 0; w < 4; w++) crc = step4(crc ^ v[i][w], lc0, lc1);
      }
      part[t] = crc;
      if (PREFETCH && t < 3) {
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = nv[i];
      }
    }
    // transpose: message M = 2t+h, line l -> xb + M*128 + l*4
#pragma unroll
    for (int t = 0; t < 4; t++) lds_st(xb + (2 * t + h) * 128 + l * 4, part[t]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int M = lane >> 3, q8 = lane & 7;
    const u32x4 s = lds_ld4(xb + M * 128 + q8 * 16);
    u32 a = nmul(OP(0), s[0]) ^ s[1];
    u32 b = nmul(OP(0), s[2]) ^ s[3];
    u32 c = nmul(OP(1), a) ^ b;                 // lines 4q8..4q8+3 combined
    c = nmul(OP(2), c) ^ shfl_down(c, 1);       // valid at q8 even
    c = nmul(OP(3), c) ^ shfl_down(c, 2);       // valid at q8 % 4 == 0
    c = nmul(OP(4), c) ^ shfl_down(c, 4);       // valid at q8 == 0
    if (q8 == 0) {
      if (sweep) out[2 * ((4 * k4 + (M >> 1)) * nw + gw) + (M & 1)] = c;
      else out[g * 8 + M] = c;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// K1s: continuous tile stream per wave (sweep order tau = k*NW + w), one tile prefetched ahead
// at all times; every 4 tiles the 8 messages' partials are transposed and tree-combined while
// the next tile's loads are in flight. MODE 0 crc, 1 no crc (rotate-xor), 2 L2-resident source.
template <int WG, int MODE>
__global__ __launch_bounds__(WG) void crc_stream4k(const u32x4* __restrict__ p, u64 nmsg, const u32* __restrict__ gtab,
                                                   const u32* __restrict__ gops, u32 init, u32* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  fill_tables(smem, gtab, threadIdx.x, WG);
  for (int t = threadIdx.x; t < 2048; t += WG) smem[OPS_OFF / 4 + t] = gops[t];
  __syncthreads();
  const u32 sbase = (u32)(uintptr_t)smem;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const u32 lc0 = sbase + ((lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  const u32 xb = sbase + XPOSE_OFF + wid * 1024;
  const int l = lane & 31, h = lane >> 5;
  const u64 ntiles = nmsg / 2;
  const u64 w = (blockIdx.x * (u64)WG + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * (WG / 64);
  if (w >= ntiles) return;
  const u64 nk = (ntiles - w + nw - 1) / nw;  // tiles for this wave: tau = k*nw + w, k < nk
  const u32 s_init = (l == 0) ? init : 0u;
  auto tile_ptr = [&](u64 k) {
    const u64 tau = k * nw + w;
    return p + (MODE == 2 ? (tau & 63) : tau) * 512 + lane * 8;
  };
  u32x4 v[8];
  {
    const u32x4* q = tile_ptr(0);
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = q[i];
  }
  u32 part[4] = {0, 0, 0, 0};
  for (u64 k = 0; k < nk; k++) {
    u32x4 nv[8];
    const bool more = k + 1 < nk;
    if (more) {
      const u32x4* q = tile_ptr(k + 1);
#pragma unroll
      for (int i = 0; i < 8; i++) nv[i] = q[i];
    }
    u32 crc = s_init;
    if (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) crc = (crc << 1 | crc >> 31) ^ v[i][j];
    } else {
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) crc = step4(crc ^ v[i][j], lc0, lc1);
    }
    const int t = (int)(k & 3);
    part[0] = t == 0 ? crc : part[0];
    part[1] = t == 1 ? crc : part[1];
    part[2] = t == 2 ? crc : part[2];
    part[3] = t == 3 ? crc : part[3];
    if (t == 3 || !more) {
      const u64 k0 = k & ~3ull;
#pragma unroll
      for (int tt = 0; tt < 4; tt++) lds_st(xb + (2 * tt + h) * 128 + l * 4, part[tt]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int M = lane >> 3, q8 = lane & 7;
      const u32x4 s = lds_ld4(xb + M * 128 + q8 * 16);
      u32 a = nmul(OP(0), s[0]) ^ s[1];
      u32 b = nmul(OP(0), s[2]) ^ s[3];
      u32 c = nmul(OP(1), a) ^ b;
      c = nmul(OP(2), c) ^ shfl_down(c, 1);
      c = nmul(OP(3), c) ^ shfl_down(c, 2);
      c = nmul(OP(4), c) ^ shfl_down(c, 4);
      const u64 kt = k0 + (M >> 1);
      if (q8 == 0 && kt <= k) out[2 * (kt * nw + w) + (M & 1)] = c;
      __builtin_amdgcn_wave_barrier();
    }
    if (more) {
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = nv[i];
    }
  }
}

// K1c: stream4k + NCH independent chains per line (chain c ends with Z_{shift_c} o T4 as a nibble op,
// slots 8..10: slot 8+c' for shift (c'+1)*128/NCH bytes), optional nontemporal loads.
template <int WG, int NCH, bool NT>
__global__ __launch_bounds__(WG) void crc_stream4k_ch(const u32x4* __restrict__ p, u64 nmsg, const u32* __restrict__ gtab,
                                                      const u32* __restrict__ gops, u32 init, u32* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  fill_tables(smem, gtab, threadIdx.x, WG);
  for (int t = threadIdx.x; t < 2048; t += WG) smem[OPS_OFF / 4 + t] = gops[t];
  __syncthreads();
  const u32 sbase = (u32)(uintptr_t)smem;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const u32 lc0 = sbase + ((lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  const u32 xb = sbase + XPOSE_OFF + wid * 1024;
  const int l = lane & 31, h = lane >> 5;
  const u64 ntiles = nmsg / 2;
  const u64 w = (blockIdx.x * (u64)WG + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * (WG / 64);
  if (w >= ntiles) return;
  const u64 nk = (ntiles - w + nw - 1) / nw;
  const u32 s_init = (l == 0) ? init : 0u;
  auto ld = [&](const u32x4* q) { return NT ? __builtin_nontemporal_load(q) : *q; };
  u32x4 v[8];
  {
    const u32x4* q = p + w * 512 + lane * 8;
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = ld(q + i);
  }
  u32 part[4] = {0, 0, 0, 0};
  constexpr int L = 32 / NCH;
  for (u64 k = 0; k < nk; k++) {
    u32x4 nv[8];
    const bool more = k + 1 < nk;
    if (more) {
      const u32x4* q = p + ((k + 1) * nw + w) * 512 + lane * 8;
#pragma unroll
      for (int i = 0; i < 8; i++) nv[i] = ld(q + i);
    }
    u32 c[NCH];
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) c[ch] = (ch == 0) ? s_init : 0u;
#pragma unroll
    for (int s = 0; s < L; s++) {
#pragma unroll
      for (int ch = 0; ch < NCH; ch++) {
        const int wi = ch * L + s;
        const u32 x = c[ch] ^ v[wi >> 2][wi & 3];
        if (s == L - 1 && ch < NCH - 1) c[ch] = nmul(OP(8 + (NCH - 2 - ch)), x);
        else c[ch] = step4(x, lc0, lc1);
      }
    }
    u32 crc = c[0];
#pragma unroll
    for (int ch = 1; ch < NCH; ch++) crc ^= c[ch];
    const int t = (int)(k & 3);
    part[0] = t == 0 ? crc : part[0];
    part[1] = t == 1 ? crc : part[1];
    part[2] = t == 2 ? crc : part[2];
    part[3] = t == 3 ? crc : part[3];
    if (t == 3 || !more) {
      const u64 k0 = k & ~3ull;
#pragma unroll
      for (int tt = 0; tt < 4; tt++) lds_st(xb + (2 * tt + h) * 128 + l * 4, part[tt]);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int M = lane >> 3, q8 = lane & 7;
      const u32x4 sv = lds_ld4(xb + M * 128 + q8 * 16);
      u32 a = nmul(OP(0), sv[0]) ^ sv[1];
      u32 b = nmul(OP(0), sv[2]) ^ sv[3];
      u32 cc = nmul(OP(1), a) ^ b;
      cc = nmul(OP(2), cc) ^ shfl_down(cc, 1);
      cc = nmul(OP(3), cc) ^ shfl_down(cc, 2);
      cc = nmul(OP(4), cc) ^ shfl_down(cc, 4);
      const u64 kt = k0 + (M >> 1);
      if (q8 == 0 && kt <= k) out[2 * (kt * nw + w) + (M & 1)] = cc;
      __builtin_amdgcn_wave_barrier();
    }
    if (more) {
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = nv[i];
    }
  }
}

// K1b: like K1 (no prefetch), but tiles processed in pairs with two interleaved chains.
template <int WG>
__global__ __launch_bounds__(WG) void crc_uniform4k_ilp2(const u32x4* __restrict__ p, u64 nmsg, const u32* __restrict__ gtab,
                                                         const u32* __restrict__ gops, u32 init, u32* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  fill_tables(smem, gtab, threadIdx.x, WG);
  for (int t = threadIdx.x; t < 2048; t += WG) smem[OPS_OFF / 4 + t] = gops[t];
  __syncthreads();
  const u32 sbase = (u32)(uintptr_t)smem;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const u32 lc0 = sbase + ((lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  const u32 xb = sbase + XPOSE_OFF + wid * 1024;
  const int l = lane & 31, h = lane >> 5;
  const u64 ngroups = nmsg / 8;
  const u64 gw = (blockIdx.x * (u64)WG + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * (WG / 64);
  const u32 s_init = (l == 0) ? init : 0u;
  for (u64 g = gw; g < ngroups; g += nw) {
    const u32x4* q = p + g * 2048 + lane * 8;
    u32 part[4];
#pragma unroll
    for (int t = 0; t < 4; t += 2) {
      u32x4 v[8], w2[8];
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = q[t * 512 + i];
#pragma unroll
      for (int i = 0; i < 8; i++) w2[i] = q[(t + 1) * 512 + i];
      u32 c0 = s_init, c1 = s_init;
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int w = 0; w < 4; w++) { c0 = step4(c0 ^ v[i][w], lc0, lc1); c1 = step4(c1 ^ w2[i][w], lc0, lc1); }
      part[t] = c0; part[t + 1] = c1;
    }
#pragma unroll
    for (int t = 0; t < 4; t++) lds_st(xb + (2 * t + h) * 128 + l * 4, part[t]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int M = lane >> 3, q8 = lane & 7;
    const u32x4 s = lds_ld4(xb + M * 128 + q8 * 16);
    u32 a = nmul(OP(0), s[0]) ^ s[1];
    u32 b = nmul(OP(0), s[2]) ^ s[3];
    u32 c = nmul(OP(1), a) ^ b;
    c = nmul(OP(2), c) ^ shfl_down(c, 1);
    c = nmul(OP(3), c) ^ shfl_down(c, 2);
    c = nmul(OP(4), c) ^ shfl_down(c, 4);
    if (q8 == 0) out[g * 8 + M] = c;
    __builtin_amdgcn_wave_barrier();
  }
}

// K2: large-message runs. wave run = RT tiles (8 KiB) of contiguous data; lane i <-> line i of each tile.
// Last word of each line (but the run's last) uses jump operator J = Z8064 o T4 (nibbles); run end: 6-level tree.
template <int WG, int RT>
__global__ __launch_bounds__(WG) void crc_tilejump(const u32x4* __restrict__ p, u64 nruns, const u32* __restrict__ gtab,
                                                   const u32* __restrict__ gops, u32* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) u32 smem[];
  fill_tables(smem, gtab, threadIdx.x, WG);
  for (int t = threadIdx.x; t < 2048; t += WG) smem[OPS_OFF / 4 + t] = gops[t];
  __syncthreads();
  const u32 sbase = (u32)(uintptr_t)smem;
  const int lane = threadIdx.x & 63;
  const u32 lc0 = sbase + ((lane & 31) << 2);
  const u32 lc1 = lc0 + 0x10000u;
  const u64 gw = (blockIdx.x * (u64)WG + threadIdx.x) >> 6;
  const u64 nw = (u64)gridDim.x * (WG / 64);
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
          const u32 x = crc ^ v[i][w];
          if (i == 7 && w == 3 && t + 1 < RT) crc = nmul(OP(6), x);
          else crc = step4(x, lc0, lc1);
        }
    }
    // tree over 64 lanes: level k operator Z_{128 * 2^k}
#pragma unroll
    for (int k = 0; k < 6; k++) crc = nmul(OP(k), crc) ^ shfl_down(crc, 1 << k);
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
__global__ void gen(u32x4* p, u64 n16, u64 seed) {
  for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n16; i += (u64)gridDim.x * blockDim.x) {
    u64 z = seed + i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; z ^= z >> 31;
    u64 y = z * 0xD6E8FEB86659FD93ull; y ^= y >> 32;
    p[i] = u32x4{(u32)z, (u32)(z >> 32), (u32)y, (u32)(y >> 32)};
  }
}

int main(int argc, char** argv) {
  host_tables();
  const u64 bytes = 4ull << 30, n16 = bytes / 16;
  u32x4* buf; CK(hipMalloc(&buf, bytes));
  u32* out; CK(hipMalloc(&out, 64ull << 20));
  gen<<<4096, 256>>>(buf, n16, 0x5EED000Bull);
  CK(hipDeviceSynchronize());
  std::vector<u32> gt(1024), ops(1024);
  for (int k = 0; k < 4; k++) for (int b = 0; b < 256; b++) gt[k * 256 + b] = T[k][b];
  for (int i = 0; i < 6; i++) nib(zbytes(128ull << i), &ops[i * 128]);
  nib(mul(zbytes(8064), t4mat()), &ops[6 * 128]);
  ops.resize(2048);
  u32 *dgt, *dops; CK(hipMalloc(&dgt, 4096)); CK(hipMalloc(&dops, 8192));
  CK(hipMemcpy(dgt, gt.data(), 4096, hipMemcpyHostToDevice));
  CK(hipMemcpy(dops, ops.data(), 8192, hipMemcpyHostToDevice));
  // chain ops for NCH=2 (slot 8: Z64 o T4) and NCH=4 (slots 8,9,10: Z32, Z64, Z96 o T4)
  std::vector<u32> ops2(ops), ops4(ops);
  nib(mul(zbytes(64), t4mat()), &ops2[8 * 128]);
  for (int j = 0; j < 3; j++) nib(mul(zbytes(32 * (j + 1)), t4mat()), &ops4[(8 + j) * 128]);
  u32 *dops2, *dops4; CK(hipMalloc(&dops2, 8192)); CK(hipMalloc(&dops4, 8192));
  CK(hipMemcpy(dops2, ops2.data(), 8192, hipMemcpyHostToDevice));
  CK(hipMemcpy(dops4, ops4.data(), 8192, hipMemcpyHostToDevice));
  int total_bad = 0;
  auto report = [&](const char* name, float ms) {
    printf("%-34s %8.3f ms %8.1f GiB/s %6.2f TB/s %5.1f%%\n", name, ms, bytes / (ms * 1e-3) / (1 << 30),
           bytes / (ms * 1e-3) / 1e12, 100.0 * bytes / (ms * 1e-3) / 8e12);
    fflush(stdout);
  };
  auto verify = [&](const char* name, u64 unit, u64 nunits, u32 init) {
    CK(hipDeviceSynchronize());
    std::vector<u32> got(nunits);
    CK(hipMemcpy(got.data(), out, nunits * 4, hipMemcpyDeviceToHost));
    std::vector<uint8_t> m(unit);
    int bad = 0, checked = 0;
    for (u64 i = 0; i < nunits; i += nunits / 97 + 1) {
      CK(hipMemcpy(m.data(), (char*)buf + i * unit, unit, hipMemcpyDeviceToHost));
      u32 want = host_crc(init, m.data(), unit);
      if (want != got[i]) { if (bad < 3) printf("  %s mismatch %llu got %08x want %08x\n", name, i, got[i], want); bad++; }
      checked++;
    }
    printf("  %s verify: %d/%d mismatches\n", name, bad, checked);
    total_bad += bad;
  };
  const size_t lds = OPS_OFF + 8192 + 16 * 1024;
  const u64 nmsg = bytes / 4096;
#define U4K(WG, PF) do { \
    CK(hipFuncSetAttribute((const void*)crc_uniform4k<WG, PF>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    CK(hipMemset(out, 0, nmsg * 4)); \
    report("uniform4k wg" #WG " pf" #PF, time_it([&] { crc_uniform4k<WG, PF><<<256, WG, lds>>>(buf, nmsg, dgt, dops, 0xFFFFFFFFu, out); }, 10)); \
    verify("uniform4k", 4096, nmsg, 0xFFFFFFFFu); } while (0)
  const int sel = argc > 1 ? atoi(argv[1]) : 0;
#define U4KM(WG, PF, MODE, NAME) do { \
    CK(hipFuncSetAttribute((const void*)crc_uniform4k<WG, PF, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    report(NAME, time_it([&] { crc_uniform4k<WG, PF, MODE><<<256, WG, lds>>>(buf, nmsg, dgt, dops, 0xFFFFFFFFu, out); }, 10)); } while (0)
  if (sel == 1) { U4K(512, true); return 0; }
  if (sel == 6) {
#define SCH(WG, NCH, NT) do { \
    CK(hipFuncSetAttribute((const void*)crc_stream4k_ch<WG, NCH, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    CK(hipMemset(out, 0, nmsg * 4)); \
    u32* dd = NCH == 4 ? dops4 : (NCH == 2 ? dops2 : dops); \
    report("stream4k_ch wg" #WG " nch" #NCH " nt" #NT, time_it([&] { crc_stream4k_ch<WG, NCH, NT><<<256, WG, lds>>>(buf, nmsg, dgt, dd, 0xFFFFFFFFu, out); }, 20)); \
    verify("ch", 4096, nmsg, 0xFFFFFFFFu); } while (0)
    SCH(768, 1, false); SCH(768, 2, false); SCH(768, 4, false);
    SCH(768, 1, true); SCH(768, 2, true); SCH(768, 4, true);
    SCH(512, 2, false); SCH(512, 4, false); SCH(1024, 2, false); SCH(1024, 4, false);
    SCH(640, 2, false); SCH(896, 2, false); SCH(640, 4, false); SCH(896, 4, false);
    SCH(512, 4, true); SCH(1024, 4, true);
    return 0;
  }
  if (sel == 5) {
#define S4K(WG, MODE, NAME) do { \
    CK(hipFuncSetAttribute((const void*)crc_stream4k<WG, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    CK(hipMemset(out, 0, nmsg * 4)); \
    report(NAME, time_it([&] { crc_stream4k<WG, MODE><<<256, WG, lds>>>(buf, nmsg, dgt, dops, 0xFFFFFFFFu, out); }, 10)); \
    if (MODE == 0) verify(NAME, 4096, nmsg, 0xFFFFFFFFu); } while (0)
    S4K(512, 0, "stream4k wg512"); S4K(1024, 0, "stream4k wg1024"); S4K(768, 0, "stream4k wg768"); S4K(256, 0, "stream4k wg256");
    S4K(512, 1, "stream4k nocrc wg512"); S4K(1024, 1, "stream4k nocrc wg1024");
    S4K(512, 2, "stream4k L2 wg512"); S4K(1024, 2, "stream4k L2 wg1024"); S4K(256, 2, "stream4k L2 wg256");
    return 0;
  }
  if (sel == 4) {
#define U4KS(WG, PF) do { \
    CK(hipFuncSetAttribute((const void*)crc_uniform4k<WG, PF, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    CK(hipMemset(out, 0, nmsg * 4)); \
    report("uniform4k SWEEP wg" #WG " pf" #PF, time_it([&] { crc_uniform4k<WG, PF, 3><<<256, WG, lds>>>(buf, nmsg, dgt, dops, 0xFFFFFFFFu, out); }, 10)); \
    verify("sweep", 4096, nmsg, 0xFFFFFFFFu); } while (0)
    U4KS(512, false); U4KS(512, true); U4KS(1024, false); U4KS(1024, true); U4KS(256, true); U4KS(768, true);
    U4KM(512, true, 4, "uniform4k SWEEP nocrc wg512 pf");
    U4KM(1024, false, 4, "uniform4k SWEEP nocrc wg1024");
    return 0;
  }
  if (sel == 2) { U4KM(512, true, 1, "uniform4k nocrc wg512 pf"); return 0; }
  if (sel == 3) { U4KM(512, true, 2, "uniform4k L2buf wg512 pf"); return 0; }
  U4K(512, false); U4K(512, true); U4K(1024, true);
  U4KM(512, true, 1, "uniform4k nocrc wg512 pf");
  U4KM(1024, true, 1, "uniform4k nocrc wg1024 pf");
  U4KM(512, false, 1, "uniform4k nocrc wg512 nopf");
  U4KM(512, true, 2, "uniform4k L2buf wg512 pf");
  U4KM(1024, true, 2, "uniform4k L2buf wg1024 pf");
  U4KM(256, true, 2, "uniform4k L2buf wg256 pf");
  CK(hipFuncSetAttribute((const void*)crc_uniform4k_ilp2<512>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void*)crc_uniform4k_ilp2<1024>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void*)crc_uniform4k_ilp2<256>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipMemset(out, 0, nmsg * 4));
  report("uniform4k ilp2 wg512", time_it([&] { crc_uniform4k_ilp2<512><<<256, 512, lds>>>(buf, nmsg, dgt, dops, 0xFFFFFFFFu, out); }, 10));
  verify("ilp2", 4096, nmsg, 0xFFFFFFFFu);
  report("uniform4k ilp2 wg1024", time_it([&] { crc_uniform4k_ilp2<1024><<<256, 1024, lds>>>(buf, nmsg, dgt, dops, 0xFFFFFFFFu, out); }, 10));
  report("uniform4k ilp2 wg256", time_it([&] { crc_uniform4k_ilp2<256><<<256, 256, lds>>>(buf, nmsg, dgt, dops, 0xFFFFFFFFu, out); }, 10));
#define TJ(WG, RT) do { \
    const u64 nruns = bytes / (8192 * RT); \
    CK(hipFuncSetAttribute((const void*)crc_tilejump<WG, RT>, hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    CK(hipMemset(out, 0, nruns * 4)); \
    report("tilejump wg" #WG " rt" #RT, time_it([&] { crc_tilejump<WG, RT><<<256, WG, lds>>>(buf, nruns, dgt, dops, out); }, 10)); \
    verify("tilejump", 8192 * RT, nruns, 0u); } while (0)
  TJ(512, 8);
  printf("TOTAL_BAD %d\n", total_bad);
  return total_bad ? 1 : 0;
}
