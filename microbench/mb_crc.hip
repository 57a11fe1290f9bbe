// Design-space microbenchmark for the batch CRC-32 engine on gfx950.
// Not product code: it answers two questions before the real kernels are written.
//   (1) which per-lane load shape streams HBM at full rate (coalesced vs per-lane spans);
//   (2) which LDS table layout sustains one lookup per payload byte at HBM speed.
// Build: hipcc -O3 --offload-arch=gfx950 -o mb_crc mb_crc.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include "annety_crc.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

static uint32_t h_t256[256];
static void make_tables() {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    h_t256[i] = c;
  }
}
static uint32_t cpu_crc(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  while (n--) c = h_t256[(c ^ *p++) & 0xff] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}
// shift a raw register by 4 zero bytes (used for slicing tables)
static uint32_t shift_bytes(uint32_t c, int n) {
  while (n--) c = h_t256[c & 0xff] ^ (c >> 8);
  return c;
}

__global__ void fill_kernel(uint4* p, size_t n16, uint64_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull; x ^= x >> 33;
    uint64_t y = x * 0xD6E8FEB86659FD93ull; y ^= y >> 32;
    p[i] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32));
  }
}

// ---------------- (1) load shapes: xor-reduce, no CRC ----------------
// stream: lane reads 16 B at 16*gid, grid-stride (fully coalesced)
__global__ __launch_bounds__(256) void k_stream(const uint4* __restrict__ d, size_t n16, uint32_t* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t st = (size_t)gridDim.x * blockDim.x;
  uint32_t a = 0;
  for (; i + 3 * st < n16; i += 4 * st) {
    uint4 v0 = d[i], v1 = d[i + st], v2 = d[i + 2 * st], v3 = d[i + 3 * st];
    a ^= v0.x ^ v0.y ^ v0.z ^ v0.w ^ v1.x ^ v1.y ^ v1.z ^ v1.w ^ v2.x ^ v2.y ^ v2.z ^ v2.w ^ v3.x ^ v3.y ^ v3.z ^ v3.w;
  }
  for (; i < n16; i += st) { uint4 v = d[i]; a ^= v.x ^ v.y ^ v.z ^ v.w; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}
// span: lane owns SPAN contiguous bytes (SPAN/16 back-to-back dwordx4), spans grid-strided
template <int SPAN>
__global__ __launch_bounds__(1024) void k_span(const uint4* __restrict__ d, size_t nspan, uint32_t* out) {
  constexpr int Q = SPAN / 16;
  size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t st = (size_t)gridDim.x * blockDim.x;
  uint32_t a = 0;
  for (; s < nspan; s += st) {
    const uint4* p = d + s * Q;
#pragma unroll
    for (int q0 = 0; q0 < Q; q0 += 8) {
      uint4 v[8];
#pragma unroll
      for (int j = 0; j < 8 && q0 + j < Q; j++) v[j] = p[q0 + j];
#pragma unroll
      for (int j = 0; j < 8 && q0 + j < Q; j++) a ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

// ---------------- (2) CRC kernels, one 1 KiB payload per lane ----------------
// table variants:
//  R1  : 1 KiB byte table, not replicated (north-star baseline)
//  R32 : byte table replicated 32x: entry e for lane l at dword e*32 + (l&31) -> bank = l&31, conflict-free
//  S4R : slicing-by-4, 4 tables each replicated 32x (128 KiB)
//  NIB : 8 nibble tables x 16 entries (512 B), slicing-by-8-nibbles; same address -> broadcast, conflict-free
enum { R1 = 0, R32 = 1, S4R = 2, NIB = 3, S4 = 4 };

template <int V>
struct LdsSize { static constexpr int dwords = 256; };
template <> struct LdsSize<R32> { static constexpr int dwords = 256 * 32; };
template <> struct LdsSize<S4R> { static constexpr int dwords = 4 * 256 * 32; };
template <> struct LdsSize<NIB> { static constexpr int dwords = 128; };
template <> struct LdsSize<S4> { static constexpr int dwords = 4 * 256; };

template <int V>
__device__ __forceinline__ uint32_t word_step(uint32_t c, uint32_t w, const uint32_t* __restrict__ t, uint32_t lane) {
  uint32_t x = c ^ w;
  if constexpr (V == R1) {
#pragma unroll
    for (int k = 0; k < 4; k++) x = t[x & 0xff] ^ (x >> 8);
    return x;
  } else if constexpr (V == R32) {
#pragma unroll
    for (int k = 0; k < 4; k++) x = t[((x & 0xff) << 5) | lane] ^ (x >> 8);
    return x;
  } else if constexpr (V == S4R) {
    // tables: T3 at 0, T2 at 8192, T1 at 16384, T0 at 24576 (dwords)
    return t[(((x)&0xff) << 5 | lane) + 0] ^ t[(((x >> 8) & 0xff) << 5 | lane) + 8192] ^
           t[(((x >> 16) & 0xff) << 5 | lane) + 16384] ^ t[(((x >> 24)) << 5 | lane) + 24576];
  } else if constexpr (V == S4) {
    return t[(x)&0xff] ^ t[((x >> 8) & 0xff) + 256] ^ t[((x >> 16) & 0xff) + 512] ^ t[(x >> 24) + 768];
  } else {  // NIB
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= t[k * 16 + ((x >> (4 * k)) & 0xf)];
    return r;
  }
}

template <int V, int BLK>
__global__ __launch_bounds__(BLK) void k_crc_lane(const uint4* __restrict__ d, size_t n, uint32_t* __restrict__ out,
                                                  const uint32_t* __restrict__ gtab) {
  __shared__ uint32_t lds[LdsSize<V>::dwords];
  for (int i = threadIdx.x; i < LdsSize<V>::dwords; i += BLK) lds[i] = gtab[i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 31;
  size_t p = blockIdx.x * (size_t)BLK + threadIdx.x;
  size_t st = (size_t)gridDim.x * BLK;
  for (; p < n; p += st) {
    const uint4* src = d + p * 64;
    uint32_t c = 0xFFFFFFFFu;
    for (int q0 = 0; q0 < 64; q0 += 8) {
      uint4 v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = src[q0 + j];
#pragma unroll
      for (int j = 0; j < 8; j++) {
        c = word_step<V>(c, v[j].x, lds, lane);
        c = word_step<V>(c, v[j].y, lds, lane);
        c = word_step<V>(c, v[j].z, lds, lane);
        c = word_step<V>(c, v[j].w, lds, lane);
      }
    }
    out[p] = ~c;
  }
}

// generic per-lane kernel with explicit double-buffered prefetch.
//   NB  = dwordx4 loads per prefetch group (NB*16 bytes per lane in flight per buffer)
//   ILP = payloads processed concurrently per lane (independent CRC chains)
template <int V, int NB, int ILP>
__device__ __forceinline__ void compute_group(uint32_t (&c)[ILP], const uint4 (&v)[ILP][NB],
                                              const uint32_t* __restrict__ lds, uint32_t lane) {
#pragma unroll
  for (int j = 0; j < NB; j++) {
#pragma unroll
    for (int k = 0; k < ILP; k++) c[k] = word_step<V>(c[k], v[k][j].x, lds, lane);
#pragma unroll
    for (int k = 0; k < ILP; k++) c[k] = word_step<V>(c[k], v[k][j].y, lds, lane);
#pragma unroll
    for (int k = 0; k < ILP; k++) c[k] = word_step<V>(c[k], v[k][j].z, lds, lane);
#pragma unroll
    for (int k = 0; k < ILP; k++) c[k] = word_step<V>(c[k], v[k][j].w, lds, lane);
  }
}

template <int V, int BLK, int NB, int ILP>
__global__ __launch_bounds__(BLK) void k_crc_pf(const uint4* __restrict__ d, size_t n, uint32_t* __restrict__ out,
                                                const uint32_t* __restrict__ gtab) {
  __shared__ uint32_t lds[LdsSize<V>::dwords];
  for (int i = threadIdx.x; i < LdsSize<V>::dwords; i += BLK) lds[i] = gtab[i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 31;
  const size_t st = (size_t)gridDim.x * BLK;
  for (size_t p = blockIdx.x * (size_t)BLK + threadIdx.x; p < n; p += ILP * st) {
    const uint4* src[ILP];
#pragma unroll
    for (int k = 0; k < ILP; k++) src[k] = d + ((p + k * st < n) ? p + k * st : p) * 64;
    uint32_t c[ILP];
#pragma unroll
    for (int k = 0; k < ILP; k++) c[k] = 0xFFFFFFFFu;
    uint4 A[ILP][NB], B[ILP][NB];
#pragma unroll
    for (int k = 0; k < ILP; k++)
#pragma unroll
      for (int j = 0; j < NB; j++) A[k][j] = src[k][j];
    for (int q = 0; q < 64; q += 2 * NB) {
#pragma unroll
      for (int k = 0; k < ILP; k++)
#pragma unroll
        for (int j = 0; j < NB; j++) B[k][j] = src[k][q + NB + j];
      __builtin_amdgcn_sched_barrier(0);
      compute_group<V, NB, ILP>(c, A, lds, lane);
      if (q + 2 * NB < 64) {
#pragma unroll
        for (int k = 0; k < ILP; k++)
#pragma unroll
          for (int j = 0; j < NB; j++) A[k][j] = src[k][q + 2 * NB + j];
      }
      __builtin_amdgcn_sched_barrier(0);
      compute_group<V, NB, ILP>(c, B, lds, lane);
    }
#pragma unroll
    for (int k = 0; k < ILP; k++)
      if (p + k * st < n) out[p + k * st] = ~c[k];
  }
}

// ---------------- v2: flattened prefetch, in-kernel table build, perm+b64 lookups ----------------
__device__ __forceinline__ uint32_t dev_shift_bits(uint32_t c, int nbits) {
  for (int i = 0; i < nbits; i++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
  return c;
}
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
enum { F_S4R = 0, F_P4A = 1, F_P4C = 2 };
// F_S4R: 4 tables x 32 replicas, entry e / replica r at dword (t*8192 + e*32 + r)       [128 KiB]
// F_P4A: 2 paired slots (T3,T2) (T1,T0), slot for (pair P, e, r) at byte P*65536 + e*256 + r*8, read as ds_read_b64
//        via inline asm (both halves loaded, one used) -> conflict-free on the 64-bank b64 rule; address = one v_perm
// F_P4C: same layout, plain C++ loads (compiler narrows to ds_read_b32 -> 2-way conflict)
template <int V, int BLK>
__device__ __forceinline__ void build_tables(uint32_t* lds) {
  if constexpr (V == F_S4R) {
    for (int i = threadIdx.x; i < 1024; i += BLK) {
      int t = i >> 8, e = i & 255;
      uint32_t v = dev_shift_bits((uint32_t)e, 8 * (4 - t));  // t=0 -> T3 (32 bits)
      uint4 q = make_uint4(v, v, v, v);
      uint4* dst = reinterpret_cast<uint4*>(lds + t * 8192 + e * 32);
#pragma unroll
      for (int r = 0; r < 8; r++) dst[r] = q;
    }
  } else {
    for (int i = threadIdx.x; i < 512; i += BLK) {
      int P = i >> 8, e = i & 255;
      uint32_t lo = dev_shift_bits((uint32_t)e, 8 * (4 - 2 * P));  // P0: T3 ; P1: T1
      uint32_t hi = dev_shift_bits((uint32_t)e, 8 * (3 - 2 * P));  // P0: T2 ; P1: T0
      uint4 q = make_uint4(lo, hi, lo, hi);
      uint4* dst = reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds) + P * 65536 + e * 256);
#pragma unroll
      for (int r = 0; r < 16; r++) dst[r] = q;
    }
  }
}

template <int V>
struct WordCtx {
  uint32_t lane, L0, L1;
};

template <int V>
__device__ __forceinline__ uint32_t word4(uint32_t x, uint32_t wnext, const uint32_t* __restrict__ lds, const WordCtx<V>& k) {
  // x = state already xored with this word; returns next x (= crc after word, xored with wnext)
  if constexpr (V == F_S4R) {
    uint32_t l = k.lane;
    uint32_t t3 = lds[(((x)&0xff) << 5 | l) + 0];
    uint32_t t2 = lds[(((x >> 8) & 0xff) << 5 | l) + 8192];
    uint32_t t1 = lds[(((x >> 16) & 0xff) << 5 | l) + 16384];
    uint32_t t0 = lds[(((x >> 24)) << 5 | l) + 24576];
    return xor3(xor3(t3, t2, t1), t0, wnext);
  } else if constexpr (V == F_P4C) {
    const char* b = reinterpret_cast<const char*>(lds);
    uint32_t a0 = __builtin_amdgcn_perm(x, k.L0, 0x0C020400u);
    uint32_t a1 = __builtin_amdgcn_perm(x, k.L0, 0x0C020500u);
    uint32_t a2 = __builtin_amdgcn_perm(x, k.L1, 0x0C020600u);
    uint32_t a3 = __builtin_amdgcn_perm(x, k.L1, 0x0C020700u);
    uint32_t t3 = reinterpret_cast<const uint2*>(b + a0)->x;
    uint32_t t2 = reinterpret_cast<const uint2*>(b + a1)->y;
    uint32_t t1 = reinterpret_cast<const uint2*>(b + a2)->x;
    uint32_t t0 = reinterpret_cast<const uint2*>(b + a3)->y;
    return xor3(xor3(t3, t2, t1), t0, wnext);
  } else {
    uint32_t a0 = __builtin_amdgcn_perm(x, k.L0, 0x0C020400u);
    uint32_t a1 = __builtin_amdgcn_perm(x, k.L0, 0x0C020500u);
    uint32_t a2 = __builtin_amdgcn_perm(x, k.L1, 0x0C020600u);
    uint32_t a3 = __builtin_amdgcn_perm(x, k.L1, 0x0C020700u);
    uint2 v0, v1, v2, v3;
    asm volatile("ds_read_b64 %0, %1" : "=v"(v0) : "v"(a0));
    asm volatile("ds_read_b64 %0, %1" : "=v"(v1) : "v"(a1));
    asm volatile("ds_read_b64 %0, %1" : "=v"(v2) : "v"(a2));
    asm volatile("ds_read_b64 %0, %1" : "=v"(v3) : "v"(a3));
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
    return xor3(xor3(v0.x, v1.y, v2.x), v3.y, wnext);
  }
}

template <int V, int NB>
__device__ __forceinline__ uint32_t group_crc(uint32_t c, const uint4 (&v)[NB], const uint32_t* __restrict__ lds,
                                             const WordCtx<V>& k) {
  // returns raw crc register after the group (x form: not yet xored with any next word)
  uint32_t x = c ^ v[0].x;
#pragma unroll
  for (int j = 0; j < NB; j++) {
    x = word4<V>(x, v[j].y, lds, k);
    x = word4<V>(x, v[j].z, lds, k);
    x = word4<V>(x, v[j].w, lds, k);
    x = word4<V>(x, j + 1 < NB ? v[j + 1].x : 0u, lds, k);
  }
  return x;
}

template <int V, int BLK, int NB, bool CO>
__global__ __launch_bounds__(BLK) void k_crc_flat(const uint4* __restrict__ d, size_t n, uint32_t* __restrict__ out,
                                                  const uint32_t* __restrict__ unused) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[32768];
  build_tables<V, BLK>(lds);
  __syncthreads();
  WordCtx<V> k;
  k.lane = threadIdx.x & 31;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  const size_t st = (size_t)gridDim.x * BLK;
  const size_t p0 = blockIdx.x * (size_t)BLK + threadIdx.x;
  const int np = p0 < n ? (int)((n - 1 - p0) / st + 1) : 0;
  constexpr int GP = 64 / NB;
  const int G = np * GP;
  auto gptr = [&](int g) -> const uint4* {
    size_t p = p0 + (size_t)(g / GP) * st;
    if (CO) p &= 4095;
    return d + p * 64 + (g % GP) * NB;
  };
  uint32_t c = 0xFFFFFFFFu;
  uint4 A[NB], B[NB];
  if (G > 0) {
    const uint4* s = gptr(0);
#pragma unroll
    for (int j = 0; j < NB; j++) A[j] = s[j];
  }
  for (int g = 0; g < G; g += 2) {
    {
      const uint4* s = gptr(g + 1);
#pragma unroll
      for (int j = 0; j < NB; j++) B[j] = s[j];
    }
    __builtin_amdgcn_sched_barrier(0);
    c = group_crc<V, NB>(c, A, lds, k);
    if (g + 2 < G) {
      const uint4* s = gptr(g + 2);
#pragma unroll
      for (int j = 0; j < NB; j++) A[j] = s[j];
    }
    __builtin_amdgcn_sched_barrier(0);
    c = group_crc<V, NB>(c, B, lds, k);
    if ((g + 1) % GP == GP - 1) {
      out[p0 + (size_t)(g / GP) * st] = ~c;
      c = 0xFFFFFFFFu;
    }
  }
}

// ---------------- v3: pure-compute ceiling (data from registers, no memory in the loop) ----------------
template <int V, int BLK, int ILP, int WORDS>
__global__ __launch_bounds__(BLK) void k_compute(const uint4* __restrict__ d, size_t n, uint32_t* __restrict__ out,
                                                 const uint32_t* __restrict__ unused) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[32768];
  build_tables<V, BLK>(lds);
  __syncthreads();
  WordCtx<V> k;
  k.lane = threadIdx.x & 31;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  const size_t gid = blockIdx.x * (size_t)BLK + threadIdx.x;
  uint4 v[4];
#pragma unroll
  for (int j = 0; j < 4; j++) v[j] = d[gid * 4 + j];
  uint32_t x[ILP];
#pragma unroll
  for (int i = 0; i < ILP; i++) x[i] = 0xFFFFFFFFu ^ v[0].x ^ i;
  for (int it = 0; it < WORDS / 16; it++) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
#pragma unroll
      for (int i = 0; i < ILP; i++) x[i] = word4<V>(x[i], v[j].y, lds, k);
#pragma unroll
      for (int i = 0; i < ILP; i++) x[i] = word4<V>(x[i], v[j].z, lds, k);
#pragma unroll
      for (int i = 0; i < ILP; i++) x[i] = word4<V>(x[i], v[j].w, lds, k);
#pragma unroll
      for (int i = 0; i < ILP; i++) x[i] = word4<V>(x[i], v[j].x, lds, k);
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < ILP; i++) r ^= x[i];
  out[gid] = r;
}

// ---------------- v4: G lanes per payload (one 128-B line per lane per round) + GF(2) combine ----------------
// GF(2) 32x32 matrix times vector: r = XOR_{i: bit i of s} col[i]
__device__ __forceinline__ uint32_t gf2_mat_vec(uint32_t s, const uint32_t (&col)[32]) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)s, i, 1);
    r ^= m & col[i];
  }
  return r;
}
__device__ __forceinline__ uint32_t xor_reduce8(uint32_t x) {
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
  return x;
}
// L = 1024, G = 8 lanes per payload, lane j owns bytes [128j, 128j+128)
// cols: [8][32] lane-position matrices M_{(7-j)*128}
template <int BLK>
__global__ __launch_bounds__(BLK) void k_stripe8(const uint4* __restrict__ d, size_t n, uint32_t* __restrict__ out,
                                                 const uint32_t* __restrict__ cols) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[32768];
  build_tables<F_P4A, BLK>(lds);
  const uint32_t j = threadIdx.x & 7;
  uint32_t col[32];
#pragma unroll
  for (int i = 0; i < 32; i += 4) {
    uint4 q = reinterpret_cast<const uint4*>(cols + j * 32)[i / 4];
    col[i] = q.x; col[i + 1] = q.y; col[i + 2] = q.z; col[i + 3] = q.w;
  }
  __syncthreads();
  WordCtx<F_P4A> k;
  k.lane = threadIdx.x & 31;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  const uint32_t sinit = j == 0 ? 0xFFFFFFFFu : 0u;
  // task t = group of 8 payloads handled by this 8-lane group
  const size_t ntask = n;
  const size_t gl = (blockIdx.x * (size_t)BLK + threadIdx.x) >> 3;  // lane-group id
  const size_t ngroups = ((size_t)gridDim.x * BLK) >> 3;
  const int T = gl < ntask ? (int)((ntask - 1 - gl) / ngroups + 1) : 0;
  auto ptr = [&](int t) -> const uint4* { return d + ((gl + (size_t)t * ngroups) * 8 + 0) * 64 + 0; };
  // lane-group gl at task t handles payload q = gl + t*ngroups ... (one payload per 8-lane group)
  auto pptr = [&](int t) -> const uint4* { return d + (gl + (size_t)t * ngroups) * 64 + j * 8; };
  uint4 A[8], B[8];
  if (T > 0) {
    const uint4* s = pptr(0);
#pragma unroll
    for (int q = 0; q < 8; q++) A[q] = s[q];
  }
  (void)ptr;
  for (int t = 0; t < T; t += 2) {
    if (t + 1 < T) {
      const uint4* s = pptr(t + 1);
#pragma unroll
      for (int q = 0; q < 8; q++) B[q] = s[q];
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      uint32_t c = group_crc<F_P4A, 8>(sinit, A, lds, k);
      uint32_t r = xor_reduce8(gf2_mat_vec(c, col));
      if (j == 0) out[gl + (size_t)t * ngroups] = ~r;
    }
    if (t + 2 < T) {
      const uint4* s = pptr(t + 2);
#pragma unroll
      for (int q = 0; q < 8; q++) A[q] = s[q];
    }
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < T) {
      uint32_t c = group_crc<F_P4A, 8>(sinit, B, lds, k);
      uint32_t r = xor_reduce8(gf2_mat_vec(c, col));
      if (j == 0) out[gl + (size_t)(t + 1) * ngroups] = ~r;
    }
  }
}

// ---------------- v4b: stripe8 with tree combine using compile-time uniform matrices ----------------
struct Mat32 { uint32_t c[32]; };
constexpr uint32_t ce_shift_bytes(uint32_t c, int nbytes) {
  for (int b = 0; b < nbytes * 8; b++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
  return c;
}
template <int D>
struct ShiftMat {
  static constexpr Mat32 make() {
    Mat32 m{};
    for (int i = 0; i < 32; i++) m.c[i] = ce_shift_bytes(1u << i, D);
    return m;
  }
  static constexpr Mat32 value = make();
};
template <int D>
__device__ __forceinline__ uint32_t shift_const(uint32_t s) {
  constexpr Mat32 m = ShiftMat<D>::value;
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 32; i++) {
    uint32_t msk = (uint32_t)__builtin_amdgcn_sbfe((int)s, i, 1);
    r ^= msk & m.c[i];
  }
  return r;
}
__device__ __forceinline__ uint32_t combine8_tree(uint32_t s) {
  // lanes j=0..7 hold chunk states; returns full-block state on lane j==0 (others garbage)
  uint32_t u = shift_const<128>(s) ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0xB1, 0xF, 0xF, false);
  uint32_t v = shift_const<256>(u) ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)u, 0x4E, 0xF, 0xF, false);
  uint32_t w = shift_const<512>(v) ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x104, 0xF, 0xF, false);  // row_shl:4
  return w;
}
template <int BLK>
__global__ __launch_bounds__(BLK) void k_stripe8t(const uint4* __restrict__ d, size_t n, uint32_t* __restrict__ out,
                                                  const uint32_t* __restrict__ unused) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[32768];
  build_tables<F_P4A, BLK>(lds);
  const uint32_t j = threadIdx.x & 7;
  __syncthreads();
  WordCtx<F_P4A> k;
  k.lane = threadIdx.x & 31;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  const uint32_t sinit = j == 0 ? 0xFFFFFFFFu : 0u;
  const size_t ntask = n;
  const size_t gl = (blockIdx.x * (size_t)BLK + threadIdx.x) >> 3;
  const size_t ngroups = ((size_t)gridDim.x * BLK) >> 3;
  const int T = gl < ntask ? (int)((ntask - 1 - gl) / ngroups + 1) : 0;
  auto pptr = [&](int t) -> const uint4* { return d + (gl + (size_t)t * ngroups) * 64 + j * 8; };
  uint4 A[8], B[8];
  if (T > 0) {
    const uint4* s = pptr(0);
#pragma unroll
    for (int q = 0; q < 8; q++) A[q] = s[q];
  }
  for (int t = 0; t < T; t += 2) {
    if (t + 1 < T) {
      const uint4* s = pptr(t + 1);
#pragma unroll
      for (int q = 0; q < 8; q++) B[q] = s[q];
    }
    __builtin_amdgcn_sched_barrier(0);
    {
      uint32_t c = group_crc<F_P4A, 8>(sinit, A, lds, k);
      uint32_t r = combine8_tree(c);
      if (j == 0) out[gl + (size_t)t * ngroups] = ~r;
    }
    if (t + 2 < T) {
      const uint4* s = pptr(t + 2);
#pragma unroll
      for (int q = 0; q < 8; q++) A[q] = s[q];
    }
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < T) {
      uint32_t c = group_crc<F_P4A, 8>(sinit, B, lds, k);
      uint32_t r = combine8_tree(c);
      if (j == 0) out[gl + (size_t)(t + 1) * ngroups] = ~r;
    }
  }
}

// ---------------- v5: NBUF-deep register ring of 128-B groups (more bytes in flight per lane) ----------------
template <int V, int BLK, int NB, int NBUF>
__global__ __launch_bounds__(BLK) void k_crc_ring(const uint4* __restrict__ d, size_t n, uint32_t* __restrict__ out,
                                                  const uint32_t* __restrict__ unused) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[32768];
  build_tables<V, BLK>(lds);
  __syncthreads();
  WordCtx<V> k;
  k.lane = threadIdx.x & 31;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  const size_t st = (size_t)gridDim.x * BLK;
  const size_t p0 = blockIdx.x * (size_t)BLK + threadIdx.x;
  const int np = p0 < n ? (int)((n - 1 - p0) / st + 1) : 0;
  constexpr int GP = 64 / NB;
  const int G = np * GP;
  auto gptr = [&](int g) -> const uint4* {
    size_t p = p0 + (size_t)(g / GP) * st;
    return d + p * 64 + (g % GP) * NB;
  };
  uint32_t c = 0xFFFFFFFFu;
  uint4 buf[NBUF][NB];
#pragma unroll
  for (int b = 0; b < NBUF - 1; b++) {
    if (b < G) {
      const uint4* s = gptr(b);
#pragma unroll
      for (int j = 0; j < NB; j++) buf[b][j] = s[j];
    }
  }
  for (int g = 0; g < G; g += NBUF) {
#pragma unroll
    for (int b = 0; b < NBUF; b++) {
      const int gl = g + b + NBUF - 1;
      if (gl < G) {
        const uint4* s = gptr(gl);
#pragma unroll
        for (int j = 0; j < NB; j++) buf[(b + NBUF - 1) % NBUF][j] = s[j];
      }
      __builtin_amdgcn_sched_barrier(0);
      if (g + b < G) {
        c = group_crc<V, NB>(c, buf[b], lds, k);
        if ((g + b) % GP == GP - 1) {
          out[p0 + (size_t)((g + b) / GP) * st] = ~c;
          c = 0xFFFFFFFFu;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

template <int NB>
__device__ __forceinline__ uint32_t group_xor(uint32_t c, const uint4 (&v)[NB]) {
#pragma unroll
  for (int j = 0; j < NB; j++) c ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  return c;
}
// ---- v5-nc: same structure, compute replaced by xor (memory-only ceiling of this structure)
template <int V, int BLK, int NB, int NBUF>
__global__ __launch_bounds__(BLK) void k_ring_nc(const uint4* __restrict__ d, size_t n, uint32_t* __restrict__ out,
                                                  const uint32_t* __restrict__ unused) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[32768];
  build_tables<V, BLK>(lds);
  __syncthreads();
  WordCtx<V> k;
  k.lane = threadIdx.x & 31;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  const size_t st = (size_t)gridDim.x * BLK;
  const size_t p0 = blockIdx.x * (size_t)BLK + threadIdx.x;
  const int np = p0 < n ? (int)((n - 1 - p0) / st + 1) : 0;
  constexpr int GP = 64 / NB;
  const int G = np * GP;
  auto gptr = [&](int g) -> const uint4* {
    size_t p = p0 + (size_t)(g / GP) * st;
    return d + p * 64 + (g % GP) * NB;
  };
  uint32_t c = 0xFFFFFFFFu;
  uint4 buf[NBUF][NB];
#pragma unroll
  for (int b = 0; b < NBUF - 1; b++) {
    if (b < G) {
      const uint4* s = gptr(b);
#pragma unroll
      for (int j = 0; j < NB; j++) buf[b][j] = s[j];
    }
  }
  for (int g = 0; g < G; g += NBUF) {
#pragma unroll
    for (int b = 0; b < NBUF; b++) {
      const int gl = g + b + NBUF - 1;
      if (gl < G) {
        const uint4* s = gptr(gl);
#pragma unroll
        for (int j = 0; j < NB; j++) buf[(b + NBUF - 1) % NBUF][j] = s[j];
      }
      __builtin_amdgcn_sched_barrier(0);
      if (g + b < G) {
        c = group_xor<NB>(c, buf[b]);
        if ((g + b) % GP == GP - 1) {
          out[p0 + (size_t)((g + b) / GP) * st] = ~c;
          c = 0xFFFFFFFFu;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// ---------------- v6: loads spread through the compute (one dwordx4 per 4 words), optional nontemporal ----------------
template <bool NT>
__device__ __forceinline__ uint4 ld16(const uint4* p) {
  if constexpr (NT) {
    uint4 r;
    r.x = __builtin_nontemporal_load(&reinterpret_cast<const uint32_t*>(p)[0]);
    r.y = __builtin_nontemporal_load(&reinterpret_cast<const uint32_t*>(p)[1]);
    r.z = __builtin_nontemporal_load(&reinterpret_cast<const uint32_t*>(p)[2]);
    r.w = __builtin_nontemporal_load(&reinterpret_cast<const uint32_t*>(p)[3]);
    return r;
  } else {
    return *p;
  }
}
template <int V, int BLK, bool NT, int SPREAD>
__global__ __launch_bounds__(BLK) void k_crc_spread(const uint4* __restrict__ d, size_t n, uint32_t* __restrict__ out,
                                                    const uint32_t* __restrict__ unused) {
  constexpr int NB = 8;
  __shared__ __attribute__((aligned(16))) uint32_t lds[32768];
  build_tables<V, BLK>(lds);
  __syncthreads();
  WordCtx<V> k;
  k.lane = threadIdx.x & 31;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  const size_t st = (size_t)gridDim.x * BLK;
  const size_t p0 = blockIdx.x * (size_t)BLK + threadIdx.x;
  const int np = p0 < n ? (int)((n - 1 - p0) / st + 1) : 0;
  constexpr int GP = 64 / NB;
  const int G = np * GP;
  auto gptr = [&](int g) -> const uint4* {
    int gg = g < G ? g : G - 1;  // clamp: re-load last group (never used)
    size_t p = p0 + (size_t)(gg / GP) * st;
    return d + p * 64 + (gg % GP) * NB;
  };
  uint32_t c = 0xFFFFFFFFu;
  uint4 A[NB], B[NB];
  if (G > 0) {
    const uint4* s = gptr(0);
#pragma unroll
    for (int j = 0; j < NB; j++) A[j] = ld16<NT>(s + j);
  }
  auto run = [&](uint4 (&cur)[NB], uint4 (&nxt)[NB], int g) {
    const uint4* s = gptr(g + 1);
    uint32_t x = c ^ cur[0].x;
#pragma unroll
    for (int j = 0; j < NB; j++) {
      if (SPREAD) {
        nxt[j] = ld16<NT>(s + j);
        __builtin_amdgcn_sched_barrier(0);
      } else if (j == 0) {
#pragma unroll
        for (int q = 0; q < NB; q++) nxt[q] = ld16<NT>(s + q);
        __builtin_amdgcn_sched_barrier(0);
      }
      x = word4<V>(x, cur[j].y, lds, k);
      x = word4<V>(x, cur[j].z, lds, k);
      x = word4<V>(x, cur[j].w, lds, k);
      x = word4<V>(x, j + 1 < NB ? cur[j + 1].x : 0u, lds, k);
    }
    c = x;
    if (g % GP == GP - 1) {
      out[p0 + (size_t)(g / GP) * st] = ~c;
      c = 0xFFFFFFFFu;
    }
  };
  for (int g = 0; g < G; g += 2) {
    run(A, B, g);
    run(B, A, g + 1);
  }
}

// ---------------- v7: stripe8 with LDS nibble-table lane-position combine ----------------
// combine tables at LDS byte offset 131072: entry (k, v, slot) at 131072 + k*2048 + v*128 + slot*4,
// slot = lane & 31 (so j = slot & 7), value = N_{j,k}[v] = M^(7-j) applied to (v << 4k)
__device__ __forceinline__ uint32_t dev_shift_bytes_bits(uint32_t c, int nbytes) { return dev_shift_bits(c, nbytes * 8); }
template <int BLK>
__device__ __forceinline__ void build_combine8(uint32_t* lds, const uint32_t* __restrict__ ctab) {
  for (int i = threadIdx.x; i < 8 * 16 * 8; i += BLK) {  // (j, k, v)
    int j = i >> 7, k = (i >> 4) & 7, v = i & 15;
    uint32_t val = ctab[i];
    for (int q = 0; q < 4; q++) lds[32768 + k * 512 + v * 32 + q * 8 + j] = val;
  }
}
__device__ __forceinline__ uint32_t combine8_lds(uint32_t s, const uint32_t* lds, uint32_t laneoff4) {
  const char* b = reinterpret_cast<const char*>(lds) + 131072;
  uint32_t t[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint32_t v = __builtin_amdgcn_ubfe(s, 4 * k, 4);
    t[k] = *reinterpret_cast<const uint32_t*>(b + k * 2048 + ((v << 7) | laneoff4));
  }
  uint32_t r = xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6] ^ t[7]);
  r ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)r, 0xB1, 0xF, 0xF, false);
  r ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)r, 0x4E, 0xF, 0xF, false);
  r ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)r, 0x141, 0xF, 0xF, false);
  return r;
}
// MODE 0 = full, 1 = memory only (xor instead of crc), 2 = compute only (loads hit first 4 MiB)
template <int BLK, int MODE>
__global__ __launch_bounds__(BLK) void k_stripe8n(const uint4* __restrict__ d, size_t n, uint32_t* __restrict__ out,
                                                  const uint32_t* __restrict__ unused) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[32768 + 4096];
  build_tables<F_P4A, BLK>(lds);
  build_combine8<BLK>(lds, unused);
  const uint32_t j = threadIdx.x & 7;
  __syncthreads();
  WordCtx<F_P4A> k;
  k.lane = threadIdx.x & 31;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  const uint32_t laneoff4 = (threadIdx.x & 31) << 2;
  const uint32_t sinit = j == 0 ? 0xFFFFFFFFu : 0u;
  const size_t gl = (blockIdx.x * (size_t)BLK + threadIdx.x) >> 3;
  const size_t ngroups = ((size_t)gridDim.x * BLK) >> 3;
  const int T = gl < n ? (int)((n - 1 - gl) / ngroups + 1) : 0;
  auto pptr = [&](int t) -> const uint4* {
    size_t p = gl + (size_t)t * ngroups;
    if (MODE == 2) p &= 4095;
    return d + p * 64 + j * 8;
  };
  auto proc = [&](const uint4 (&v)[8], int t) {
    uint32_t c;
    if (MODE == 1) c = group_xor<8>(sinit, v);
    else c = group_crc<F_P4A, 8>(sinit, v, lds, k);
    uint32_t r = combine8_lds(c, lds, laneoff4);
    if (j == 0) out[gl + (size_t)t * ngroups] = ~r;
  };
  uint4 A[8], B[8];
  if (T > 0) {
    const uint4* s = pptr(0);
#pragma unroll
    for (int q = 0; q < 8; q++) A[q] = s[q];
  }
  for (int t = 0; t < T; t += 2) {
    if (t + 1 < T) {
      const uint4* s = pptr(t + 1);
#pragma unroll
      for (int q = 0; q < 8; q++) B[q] = s[q];
    }
    __builtin_amdgcn_sched_barrier(0);
    proc(A, t);
    if (t + 2 < T) {
      const uint4* s = pptr(t + 2);
#pragma unroll
      for (int q = 0; q < 8; q++) A[q] = s[q];
    }
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < T) proc(B, t + 1);
  }
}

// ---------------- v8: memory-structure variants (xor only) ----------------
// ASSIGN 0: grid-stride over payloads (stripe8n); 1: per-WG contiguous payload block
// BUF 1: single buffer (load 8, consume); 2: double buffer
template <int BLK, int ASSIGN, int BUF>
__global__ __launch_bounds__(BLK) void k_memvar(const uint4* __restrict__ d, size_t n, uint32_t* __restrict__ out) {
  const uint32_t j = threadIdx.x & 7;
  size_t first, step;
  int T;
  if (ASSIGN == 0) {
    const size_t gl = (blockIdx.x * (size_t)BLK + threadIdx.x) >> 3;
    step = ((size_t)gridDim.x * BLK) >> 3;
    first = gl;
    T = gl < n ? (int)((n - 1 - gl) / step + 1) : 0;
  } else if (ASSIGN == 2) {
    // virtual 256-thread workgroups: sub-block v of block b acts as block b + gridDim.x * v
    const size_t vb = blockIdx.x + (size_t)gridDim.x * (threadIdx.x / 256);
    const size_t gl = (vb * 256 + (threadIdx.x % 256)) >> 3;
    step = ((size_t)gridDim.x * BLK) >> 3;
    first = gl;
    T = gl < n ? (int)((n - 1 - gl) / step + 1) : 0;
  } else {
    size_t per = (n + gridDim.x - 1) / gridDim.x;
    size_t b0 = blockIdx.x * per, b1 = b0 + per < n ? b0 + per : n;
    size_t gl = threadIdx.x >> 3;
    step = BLK >> 3;
    first = b0 + gl;
    T = first < b1 ? (int)((b1 - 1 - first) / step + 1) : 0;
  }
  auto pptr = [&](int t) -> const uint4* { return d + (first + (size_t)t * step) * 64 + j * 8; };
  uint32_t acc = 0;
  if (BUF == 1) {
    for (int t = 0; t < T; t++) {
      uint4 A[8];
      const uint4* s = pptr(t);
#pragma unroll
      for (int q = 0; q < 8; q++) A[q] = s[q];
      acc = group_xor<8>(acc, A);
    }
  } else {
    uint4 A[8], B[8];
    if (T > 0) {
      const uint4* s = pptr(0);
#pragma unroll
      for (int q = 0; q < 8; q++) A[q] = s[q];
    }
    for (int t = 0; t < T; t += 2) {
      if (t + 1 < T) {
        const uint4* s = pptr(t + 1);
#pragma unroll
        for (int q = 0; q < 8; q++) B[q] = s[q];
      }
      __builtin_amdgcn_sched_barrier(0);
      acc = group_xor<8>(acc, A);
      if (t + 2 < T) {
        const uint4* s = pptr(t + 2);
#pragma unroll
        for (int q = 0; q < 8; q++) A[q] = s[q];
      }
      __builtin_amdgcn_sched_barrier(0);
      if (t + 1 < T) acc = group_xor<8>(acc, B);
    }
  }
  out[blockIdx.x * BLK + threadIdx.x] = acc;
}

// ---------------- host ----------------
struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
};

template <typename F>
static double time_ms(F f, int reps = 15) {
  Timer t;
  f();
  CK(hipDeviceSynchronize());
  std::vector<float> ms;
  for (int r = 0; r < reps; r++) {
    CK(hipEventRecord(t.a));
    f();
    CK(hipEventRecord(t.b));
    CK(hipEventSynchronize(t.b));
    float x;
    CK(hipEventElapsedTime(&x, t.a, t.b));
    ms.push_back(x);
  }
  std::sort(ms.begin(), ms.end());
  return ms[ms.size() / 2];
}

static int ab_main();
int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "ab") return ab_main();
  const bool mv_only = argc > 1 && std::string(argv[1]) == "mv";
  make_tables();
  const size_t n = 1u << 20;  // payloads
  const size_t L = 1024;
  const size_t bytes = n * L;
  uint4* d;
  uint32_t *out, *gtab;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&out, n * 4 + (1 << 22)));
  CK(hipMalloc(&gtab, 4 * 256 * 32 * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, d, bytes / 16, 0x1234ull);
  CK(hipDeviceSynchronize());
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs %d clock %d kHz\n", prop.name, prop.multiProcessorCount, prop.clockRate);

  // ---- load shapes
  auto report = [&](const char* name, double ms, size_t b) {
    printf("%-40s %8.4f ms  %8.1f GB/s\n", name, ms, b / ms / 1e6);
    fflush(stdout);
  };
  for (int g : {2048}) {
    char nm[64];
    snprintf(nm, sizeof nm, "stream grid=%d", g);
    report(nm, time_ms([&] { hipLaunchKernelGGL(k_stream, dim3(g), dim3(256), 0, 0, d, bytes / 16, out); }), bytes);
  }
#define SPAN(S)                                                                                              \
  for (int g : {1024, 2048, 4096}) {                                                                         \
    char nm[64];                                                                                             \
    snprintf(nm, sizeof nm, "span%d grid=%d", S, g);                                                         \
    report(nm, time_ms([&] { hipLaunchKernelGGL(k_span<S>, dim3(g), dim3(256), 0, 0, d, bytes / S, out); }), \
           bytes);                                                                                           \
  }
  SPAN(128)

  // ---- CRC variants
  std::vector<uint32_t> tab(4 * 256 * 32);
  // sample reference digests
  const int NS = 4096;
  std::vector<uint8_t> hbuf(NS * L);
  std::vector<uint32_t> ref(NS), got(n);
  // sample = payloads spread through batch
  for (int s = 0; s < NS; s++) {
    size_t p = (size_t)s * (n / NS) + (s % 7);
    CK(hipMemcpy(hbuf.data() + s * L, (char*)d + p * L, L, hipMemcpyDeviceToHost));
    ref[s] = cpu_crc(hbuf.data() + s * L, L);
  }
  auto check = [&](const char* name) {
    CK(hipMemcpy(got.data(), out, n * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int s = 0; s < NS; s++) {
      size_t p = (size_t)s * (n / NS) + (s % 7);
      if (got[p] != ref[s]) bad++;
    }
    printf("   check %s: %s (%d bad of %d)\n", name, bad ? "FAIL" : "ok", bad, NS);
  };
  auto setup = [&](int V) {
    int nd = 0;
    if (V == R1) { for (int i = 0; i < 256; i++) tab[i] = h_t256[i]; nd = 256; }
    if (V == R32) { for (int e = 0; e < 256; e++) for (int r = 0; r < 32; r++) tab[e * 32 + r] = h_t256[e]; nd = 8192; }
    if (V == S4R || V == S4) {
      // T_k[b] = table value shifted by k more zero bytes; slicing: x bytes b0..b3 use T3,T2,T1,T0
      int rep = V == S4R ? 32 : 1;
      for (int t = 0; t < 4; t++)
        for (int e = 0; e < 256; e++) {
          uint32_t v = shift_bytes(h_t256[e], 3 - t);  // t=0 -> T3 (byte 0)
          for (int r = 0; r < rep; r++) tab[t * 256 * rep + e * rep + r] = v;
        }
      nd = 4 * 256 * rep;
    }
    if (V == NIB) {
      for (int k = 0; k < 8; k++)
        for (int m = 0; m < 16; m++) tab[k * 16 + m] = shift_bytes((uint32_t)m << (4 * k), 4);
      nd = 128;
    }
    CK(hipMemcpy(gtab, tab.data(), nd * 4, hipMemcpyHostToDevice));
  };
  const double algo = (double)bytes + n * 4.0;
#define CRC(KER, V, BLK, G, NAME, ...)                                                                              \
  {                                                                                                            \
    setup(V);                                                                                                  \
    CK(hipMemset(out, 0, n * 4));                                                                              \
    double ms = time_ms([&] { hipLaunchKernelGGL((KER<V, BLK, ##__VA_ARGS__>), dim3(G), dim3(BLK), 0, 0, d, n, out, gtab); }); \
    char nm[96];                                                                                               \
    snprintf(nm, sizeof nm, "%s blk=%d grid=%d", NAME, BLK, G);                                                \
    report(nm, ms, (size_t)algo);                                                                              \
    check(nm);                                                                                                 \
  }
#define CRCP(V, BLK, NB, ILP, G, NAME) CRC(k_crc_pf, V, BLK, G, NAME " nb" #NB " ilp" #ILP, NB, ILP)
#define CRCF(V, BLK, NB, CO, G, NAME) CRC(k_crc_flat, V, BLK, G, NAME " nb" #NB " co" #CO, NB, CO)
  {
    // lane-position matrices for G=8, C=128
    std::vector<uint32_t> hc(8 * 32);
    for (int jj = 0; jj < 8; jj++)
      for (int i = 0; i < 32; i++) hc[jj * 32 + i] = shift_bytes(1u << i, (7 - jj) * 128);
    uint32_t* dcols;
    CK(hipMalloc(&dcols, hc.size() * 4));
    CK(hipMemcpy(dcols, hc.data(), hc.size() * 4, hipMemcpyHostToDevice));
    for (int blk : {1024, 512}) {
      for (int G : {256, 512}) {
        CK(hipMemset(out, 0, n * 4));
        double ms;
        if (blk == 1024) ms = time_ms([&] { hipLaunchKernelGGL((k_stripe8<1024>), dim3(G), dim3(1024), 0, 0, d, n, out, dcols); });
        else ms = time_ms([&] { hipLaunchKernelGGL((k_stripe8<512>), dim3(G), dim3(512), 0, 0, d, n, out, dcols); });
        char nm[96];
        snprintf(nm, sizeof nm, "stripe8 blk=%d grid=%d", blk, G);
        report(nm, ms, (size_t)algo);
        check(nm);
      }
    }
  }
  for (int G : {256, 512}) {
    CK(hipMemset(out, 0, n * 4));
    double ms = time_ms([&] { hipLaunchKernelGGL((k_stripe8t<1024>), dim3(G), dim3(1024), 0, 0, d, n, out, gtab); });
    char nm[96];
    snprintf(nm, sizeof nm, "stripe8t blk=1024 grid=%d", G);
    report(nm, ms, (size_t)algo);
    check(nm);
    ms = time_ms([&] { hipLaunchKernelGGL((k_stripe8t<512>), dim3(G), dim3(512), 0, 0, d, n, out, gtab); });
    snprintf(nm, sizeof nm, "stripe8t blk=512 grid=%d", G);
    report(nm, ms, (size_t)algo);
    check(nm);
  }
#define RING(V, BLK, NB, NBUF, G)                                                                             \
  {                                                                                                          \
    CK(hipMemset(out, 0, n * 4));                                                                            \
    double ms = time_ms([&] { hipLaunchKernelGGL((k_crc_ring<V, BLK, NB, NBUF>), dim3(G), dim3(BLK), 0, 0, d, n, out, gtab); }); \
    char nm[96];                                                                                             \
    snprintf(nm, sizeof nm, "ring %s blk=%d nb=%d nbuf=%d grid=%d", #V, BLK, NB, NBUF, G);                    \
    report(nm, ms, (size_t)algo);                                                                            \
    check(nm);                                                                                               \
  }
  RING(F_P4A, 1024, 8, 2, 256)
  RING(F_P4A, 1024, 8, 3, 256)
  RING(F_P4A, 1024, 4, 4, 256)
  RING(F_P4A, 1024, 4, 5, 256)
  RING(F_P4A, 1024, 4, 6, 256)
  RING(F_P4A, 768, 8, 3, 256)
  RING(F_P4A, 768, 8, 4, 256)
  RING(F_P4A, 512, 8, 3, 256)
  RING(F_P4A, 512, 8, 4, 256)
  RING(F_P4A, 512, 8, 5, 256)
#define SPR(V, BLK, NT, SP, G)                                                                               \
  {                                                                                                          \
    CK(hipMemset(out, 0, n * 4));                                                                            \
    double ms = time_ms([&] { hipLaunchKernelGGL((k_crc_spread<V, BLK, NT, SP>), dim3(G), dim3(BLK), 0, 0, d, n, out, gtab); }); \
    char nm[96];                                                                                             \
    snprintf(nm, sizeof nm, "spread %s blk=%d nt=%d spread=%d grid=%d", #V, BLK, NT, SP, G);                   \
    report(nm, ms, (size_t)algo);                                                                            \
    check(nm);                                                                                               \
  }
#define RINGNC(V, BLK, NB, NBUF, G)                                                                           \
  {                                                                                                          \
    double ms = time_ms([&] { hipLaunchKernelGGL((k_ring_nc<V, BLK, NB, NBUF>), dim3(G), dim3(BLK), 0, 0, d, n, out, gtab); }); \
    char nm[96];                                                                                             \
    snprintf(nm, sizeof nm, "ringNC blk=%d nb=%d nbuf=%d grid=%d", BLK, NB, NBUF, G);                         \
    report(nm, ms, (size_t)algo);                                                                            \
  }
  RINGNC(F_P4A, 1024, 8, 2, 256)
  RINGNC(F_P4A, 1024, 8, 3, 256)
  RINGNC(F_P4A, 512, 8, 2, 256)
  RINGNC(F_P4A, 512, 8, 3, 256)
  RINGNC(F_P4A, 256, 8, 2, 256)
  RINGNC(F_P4A, 256, 8, 3, 256)
  RINGNC(F_P4A, 256, 8, 4, 256)
  for (int g : {256, 512, 768, 1024, 1536, 2048}) {
    char nm[64];
    snprintf(nm, sizeof nm, "span128 blk256 grid=%d", g);
    report(nm, time_ms([&] { hipLaunchKernelGGL(k_span<128>, dim3(g), dim3(256), 0, 0, d, bytes / 128, out); }), bytes);
  }
  std::vector<uint32_t> hct(1024);
  for (int jj = 0; jj < 8; jj++) for (int kk = 0; kk < 8; kk++) for (int vv = 0; vv < 16; vv++)
    hct[(jj * 8 + kk) * 16 + vv] = shift_bytes((uint32_t)vv << (4 * kk), (7 - jj) * 128);
  uint32_t* dct; CK(hipMalloc(&dct, 4096)); CK(hipMemcpy(dct, hct.data(), 4096, hipMemcpyHostToDevice));
#define ST8N(BLK, MODE, G)                                                                                   \
  {                                                                                                          \
    CK(hipMemset(out, 0, n * 4));                                                                            \
    double ms = time_ms([&] { hipLaunchKernelGGL((k_stripe8n<BLK, MODE>), dim3(G), dim3(BLK), 0, 0, d, n, out, dct); }); \
    char nm[96];                                                                                             \
    snprintf(nm, sizeof nm, "stripe8n blk=%d mode=%d grid=%d", BLK, MODE, G);                                 \
    report(nm, ms, (size_t)algo);                                                                            \
    if (MODE == 0) check(nm);                                                                                \
  }
  {
    for (size_t nn : {(size_t)2048, (size_t)262144, (size_t)524288, n}) {
      double ms = time_ms([&] { hipLaunchKernelGGL((k_stripe8n<512, 0>), dim3(256), dim3(512), 0, 0, d, nn, out, dct); });
      printf("stripe8n blk=512 n=%zu  %.4f ms  %.1f GB/s\n", nn, ms, nn * 1028.0 / ms / 1e6);
      ms = time_ms([&] { hipLaunchKernelGGL((k_stripe8n<512, 1>), dim3(256), dim3(512), 0, 0, d, nn, out, dct); });
      printf("stripe8n-memonly blk=512 n=%zu  %.4f ms  %.1f GB/s\n", nn, ms, nn * 1028.0 / ms / 1e6);
      ms = time_ms([&] { hipLaunchKernelGGL(k_span<128>, dim3(1024), dim3(256), 0, 0, d, nn * 8, out); });
      printf("span128 n=%zu  %.4f ms  %.1f GB/s\n", nn, ms, nn * 1024.0 / ms / 1e6);
    }
  }
#define MV(BLK, AS, BUF, G) { double ms = time_ms([&] { hipLaunchKernelGGL((k_memvar<BLK, AS, BUF>), dim3(G), dim3(BLK), 0, 0, d, n, out); }); \
    printf("memvar blk=%d assign=%d buf=%d grid=%d  %.4f ms  %.1f GB/s\n", BLK, AS, BUF, G, ms, bytes / ms / 1e6); }
  for (int rep = 0; rep < 2; rep++) {
  MV(512, 0, 2, 256) MV(512, 2, 2, 256) MV(1024, 0, 2, 256) MV(1024, 2, 2, 256) MV(256, 0, 2, 1024) MV(256, 0, 2, 256) MV(768, 2, 2, 256)
  }  if (mv_only) return 0;

  { double ms = time_ms([&] { hipLaunchKernelGGL(k_span<128>, dim3(256), dim3(512), 0, 0, d, bytes / 128, out); });
    printf("span128 blk512 grid256 %.4f ms %.1f GB/s\n", ms, bytes / ms / 1e6); }
#define COMP(V, BLK, ILP, G)                                                                                 \
  {                                                                                                          \
    const int W = 4096;                                                                                      \
    double ms = time_ms([&] { hipLaunchKernelGGL((k_compute<V, BLK, ILP, W>), dim3(G), dim3(BLK), 0, 0, d, n, out, gtab); }); \
    double eq = (double)G * BLK * ILP * W * 4;                                                               \
    char nm[96];                                                                                             \
    snprintf(nm, sizeof nm, "compute %s blk=%d ilp=%d grid=%d", #V, BLK, ILP, G);                            \
    report(nm, ms, (size_t)eq);                                                                              \
  }
  COMP(F_P4A, 1024, 1, 256)
  COMP(F_P4A, 1024, 2, 256)
  COMP(F_P4A, 1024, 4, 256)
  COMP(F_P4A, 512, 1, 256)
  COMP(F_P4A, 512, 2, 256)
  COMP(F_P4A, 512, 4, 256)
  COMP(F_P4A, 256, 4, 256)
  COMP(F_P4A, 256, 8, 256)
  COMP(F_P4C, 1024, 1, 256)
  COMP(F_P4C, 1024, 2, 256)
  COMP(F_S4R, 1024, 1, 256)
  COMP(F_S4R, 1024, 2, 256)
  COMP(F_S4R, 512, 2, 256)
  return 0;
}

// A/B: product library (C-ABI) vs the microbench stripe8n kernel on the same buffer, interleaved.
static int ab_main() {
  make_tables();
  const size_t n = 1u << 20, L = 1024, bytes = n * L;
  uint4* d;
  uint32_t *out1, *out2;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&out1, n * 4));
  CK(hipMalloc(&out2, n * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, d, bytes / 16, 0x1234ull);
  std::vector<uint32_t> hct(1024);
  for (int jj = 0; jj < 8; jj++) for (int kk = 0; kk < 8; kk++) for (int vv = 0; vv < 16; vv++)
    hct[(jj * 8 + kk) * 16 + vv] = shift_bytes((uint32_t)vv << (4 * kk), (7 - jj) * 128);
  uint32_t* dct; CK(hipMalloc(&dct, 4096)); CK(hipMemcpy(dct, hct.data(), 4096, hipMemcpyHostToDevice));
  CK(hipDeviceSynchronize());
  auto prod = [&] { if (annety_crc32_batch_fixed(d, n, L, L, out1, nullptr) != 0) { fprintf(stderr, "prod fail\n"); exit(1);} };
  auto mb = [&] { hipLaunchKernelGGL((k_stripe8n<512, 0>), dim3(256), dim3(512), 0, 0, d, n, out2, dct); };
  for (int round = 0; round < 4; round++) {
    double a = time_ms(prod, 10), b = time_ms(mb, 10);
    printf("round %d  product %.4f ms (%.1f GB/s)   microbench %.4f ms (%.1f GB/s)\n", round, a, (bytes + 4.0 * n) / a / 1e6, b,
           (bytes + 4.0 * n) / b / 1e6);
  }
  std::vector<uint32_t> h1(n), h2(n);
  CK(hipMemcpy(h1.data(), out1, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(h2.data(), out2, n * 4, hipMemcpyDeviceToHost));
  printf("outputs %s\n", h1 == h2 ? "identical" : "DIFFER");
  // back-to-back launches (no events between)
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int which = 0; which < 2; which++) {
    CK(hipEventRecord(e0));
    for (int r = 0; r < 50; r++) { if (which == 0) prod(); else mb(); }
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%s back-to-back x50: %.4f ms/launch (%.1f GB/s)\n", which == 0 ? "product" : "microbench", ms / 50, (bytes + 4.0 * n) / (ms / 50) / 1e6);
  }
  return 0;
}
