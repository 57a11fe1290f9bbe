// Device-side building blocks shared by the gfx950 checksum kernels (crc32_kernels.hip,
// crc32_arena.hip): the LDS-table line fold, the nibble-table GF(2) maps, lane-group reductions and
// the LDS-DMA image staging. Header-only; every kernel translation unit gets its own inline copies.
// The math is in crc32_math.h; DESIGN.md §2 describes the LDS image and the fold.
#pragma once

#include <hip/hip_runtime.h>

#include "crc32_kernels.h"
#include "crc32_math.h"

namespace annety_crc {
namespace {

constexpr int kBlock = 512;
// Threads per virtual workgroup (0 = off): the lane-groups of one 512-thread block are taken from
// two virtual blocks gridDim.x apart instead of one contiguous run (microbench/mb_crc.hip `mv`:
// 6.43 vs 6.17 TB/s for the same load/LDS structure).
constexpr int kVwg = 256;

// Lane-group index of this thread under the virtual-workgroup mapping (a bijection onto
// [0, gridDim.x * BLK / G) for VWG a multiple of G that divides BLK).
template <int BLK, int G, int VWG>
__device__ __forceinline__ size_t group_id() {
  if constexpr (VWG == 0 || VWG >= BLK) {
    return (blockIdx.x * (size_t)BLK + threadIdx.x) / G;
  } else {
    const size_t v = blockIdx.x + (size_t)gridDim.x * (threadIdx.x / VWG);
    return (v * VWG + threadIdx.x % VWG) / G;
  }
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

struct LaneCtx {
  uint32_t L0;     // (replica*8) in byte 0, pair 0 in byte 2
  uint32_t L1;     // (replica*8) in byte 0, pair 1 in byte 2
  uint32_t slot4;  // replica*4 for the 4-byte join tables
};

// Absorb one 32-bit word per chain, two chains at once. x = register ^ word (little-endian bytes
// b0..b3) becomes T3[b0]^T2[b1]^T1[b2]^T0[b3] ^ wnext, i.e. the register after the word, pre-xored with
// the chain's next word. The eight ds_read_b64 and their wait are ONE asm statement: the compiler cannot
// narrow them to ds_read_b32 (which would use the 32-bank rule and conflict 2-way), and it never sees a
// destination register before the data has landed. (With the reads and the wait as separate statements
// the allocator may copy a destination between them; under a 128-VGPR cap it did, and the copy picked
// up stale bits whenever the LDS was slower than the copy: DESIGN.md §7.2.)
__device__ __forceinline__ void word4x2(uint32_t& xa, uint32_t wa, uint32_t& xb, uint32_t wb, const LaneCtx& k) {
  const uint32_t a0 = __builtin_amdgcn_perm(xa, k.L0, 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(xa, k.L0, 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(xa, k.L1, 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(xa, k.L1, 0x0C020700u);
  const uint32_t b0 = __builtin_amdgcn_perm(xb, k.L0, 0x0C020400u);
  const uint32_t b1 = __builtin_amdgcn_perm(xb, k.L0, 0x0C020500u);
  const uint32_t b2 = __builtin_amdgcn_perm(xb, k.L1, 0x0C020600u);
  const uint32_t b3 = __builtin_amdgcn_perm(xb, k.L1, 0x0C020700u);
  uint2 u0, u1, u2, u3, v0, v1, v2, v3;
  asm volatile(
      "ds_read_b64 %0, %8\n\t"
      "ds_read_b64 %1, %9\n\t"
      "ds_read_b64 %2, %10\n\t"
      "ds_read_b64 %3, %11\n\t"
      "ds_read_b64 %4, %12\n\t"
      "ds_read_b64 %5, %13\n\t"
      "ds_read_b64 %6, %14\n\t"
      "ds_read_b64 %7, %15\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(u0), "=&v"(u1), "=&v"(u2), "=&v"(u3), "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
      : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(b0), "v"(b1), "v"(b2), "v"(b3));
  xa = xor3(xor3(u0.x, u1.y, u2.x), u3.y, wa);
  xb = xor3(xor3(v0.x, v1.y, v2.x), v3.y, wb);
}

// Four chains at once (two lines, two chains each): 16 ds_read_b64 in flight per wait.
__device__ __forceinline__ void word4x4(uint32_t& xa, uint32_t wa, uint32_t& xb, uint32_t wb, uint32_t& xc, uint32_t wc,
                                        uint32_t& xd, uint32_t wd, const LaneCtx& k) {
  uint32_t a[16];
  const uint32_t x[4] = {xa, xb, xc, xd};
#pragma unroll
  for (int c = 0; c < 4; c++) {
    a[4 * c + 0] = __builtin_amdgcn_perm(x[c], k.L0, 0x0C020400u);
    a[4 * c + 1] = __builtin_amdgcn_perm(x[c], k.L0, 0x0C020500u);
    a[4 * c + 2] = __builtin_amdgcn_perm(x[c], k.L1, 0x0C020600u);
    a[4 * c + 3] = __builtin_amdgcn_perm(x[c], k.L1, 0x0C020700u);
  }
  uint2 u[16];
  asm volatile(
      "ds_read_b64 %0, %16\n\tds_read_b64 %1, %17\n\tds_read_b64 %2, %18\n\tds_read_b64 %3, %19\n\t"
      "ds_read_b64 %4, %20\n\tds_read_b64 %5, %21\n\tds_read_b64 %6, %22\n\tds_read_b64 %7, %23\n\t"
      "ds_read_b64 %8, %24\n\tds_read_b64 %9, %25\n\tds_read_b64 %10, %26\n\tds_read_b64 %11, %27\n\t"
      "ds_read_b64 %12, %28\n\tds_read_b64 %13, %29\n\tds_read_b64 %14, %30\n\tds_read_b64 %15, %31\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(u[0]), "=&v"(u[1]), "=&v"(u[2]), "=&v"(u[3]), "=&v"(u[4]), "=&v"(u[5]), "=&v"(u[6]), "=&v"(u[7]),
        "=&v"(u[8]), "=&v"(u[9]), "=&v"(u[10]), "=&v"(u[11]), "=&v"(u[12]), "=&v"(u[13]), "=&v"(u[14]), "=&v"(u[15])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]), "v"(a[8]), "v"(a[9]),
        "v"(a[10]), "v"(a[11]), "v"(a[12]), "v"(a[13]), "v"(a[14]), "v"(a[15]));
  xa = xor3(xor3(u[0].x, u[1].y, u[2].x), u[3].y, wa);
  xb = xor3(xor3(u[4].x, u[5].y, u[6].x), u[7].y, wb);
  xc = xor3(xor3(u[8].x, u[9].y, u[10].x), u[11].y, wc);
  xd = xor3(xor3(u[12].x, u[13].y, u[14].x), u[15].y, wd);
}

// Apply a uniform nibble-table map (8 x 16 entries at LDS byte offset `off`, broadcast reads).
__device__ __forceinline__ uint32_t nibble_map_uniform(uint32_t s, const uint32_t* lds, uint32_t off);

// Absorb one 128-byte line (8 x 16 B) into register s: bytes 0-63 continue the lane's chain, bytes
// 64-127 start a fresh chain from 0; the two are joined with shift_64 (raw(A||B, s) =
// shift_64(raw(A, s)) ^ raw(B, 0)). Two chains double the LDS reads in flight per wave.
__device__ __forceinline__ uint32_t absorb_line(uint32_t s, const uint4 (&v)[8], const LaneCtx& k,
                                                const uint32_t* lds) {
  uint32_t xa = s ^ v[0].x, xb = v[4].x;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    word4x2(xa, v[i].y, xb, v[4 + i].y, k);
    word4x2(xa, v[i].z, xb, v[4 + i].z, k);
    word4x2(xa, v[i].w, xb, v[4 + i].w, k);
    word4x2(xa, i + 1 < 4 ? v[i + 1].x : 0u, xb, i + 1 < 4 ? v[5 + i].x : 0u, k);
  }
  return nibble_map_uniform(xa, lds, kLdsHalfOff) ^ xb;
}

// Two independent lines from register 0 (raw CRCs), folded together: twice the LDS reads per wait.
__device__ __forceinline__ void absorb_two_lines(const uint4 (&v)[8], const uint4 (&w)[8], const LaneCtx& k,
                                                 const uint32_t* lds, uint32_t& rv, uint32_t& rw);

// Apply a uniform nibble-table map (8 x 16 entries at LDS byte offset `off`, broadcast reads).
__device__ __forceinline__ uint32_t nibble_map_uniform(uint32_t s, const uint32_t* lds, uint32_t off) {
  const uint32_t* t = lds + off / 4;
  uint32_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++) r[k] = t[k * 16 + __builtin_amdgcn_ubfe(s, 4 * k, 4)];
  return xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), r[6] ^ r[7]);
}

__device__ __forceinline__ void absorb_two_lines(const uint4 (&v)[8], const uint4 (&w)[8], const LaneCtx& k,
                                                 const uint32_t* lds, uint32_t& rv, uint32_t& rw) {
  uint32_t xa = v[0].x, xb = v[4].x, xc = w[0].x, xd = w[4].x;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    word4x4(xa, v[i].y, xb, v[4 + i].y, xc, w[i].y, xd, w[4 + i].y, k);
    word4x4(xa, v[i].z, xb, v[4 + i].z, xc, w[i].z, xd, w[4 + i].z, k);
    word4x4(xa, v[i].w, xb, v[4 + i].w, xc, w[i].w, xd, w[4 + i].w, k);
    word4x4(xa, i + 1 < 4 ? v[i + 1].x : 0u, xb, i + 1 < 4 ? v[5 + i].x : 0u, xc, i + 1 < 4 ? w[i + 1].x : 0u, xd,
            i + 1 < 4 ? w[5 + i].x : 0u, k);
  }
  rv = nibble_map_uniform(xa, lds, kLdsHalfOff) ^ xb;
  rw = nibble_map_uniform(xc, lds, kLdsHalfOff) ^ xd;
}

// Map i of a set of T nibble-table maps stored [k][i][v] (k nibble position, v value): for one k the
// set's tables lie side by side, so lanes applying different maps spread over the banks
// ((16 i + v) mod 64) instead of all sharing the same 16 (a [i][k][v] layout cost the segment steps
// up to 8-way conflicts).
template <uint32_t T>
__device__ __forceinline__ uint32_t nibble_map_set(uint32_t s, const uint32_t* lds, uint32_t off, uint32_t i) {
  const uint32_t* t = lds + off / 4 + i * 16;
  uint32_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++) r[k] = t[k * T * 16 + __builtin_amdgcn_ubfe(s, 4 * k, 4)];
  return xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), r[6] ^ r[7]);
}

// Lane-position join: shift_{(G-1-j)*128}(s) from the replicated nibble tables (slot = lane & 31).
__device__ __forceinline__ uint32_t nibble_map_lane(uint32_t s, const uint32_t* lds, uint32_t slot4) {
  const char* b = reinterpret_cast<const char*>(lds) + kLdsJoinOff;
  uint32_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    r[k] = *reinterpret_cast<const uint32_t*>(b + k * 2048 + ((__builtin_amdgcn_ubfe(s, 4 * k, 4) << 7) | slot4));
  return xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), r[6] ^ r[7]);
}

// xor-reduce across the G lanes of a lane-group; the value is complete on lane j = G-1.
template <int G>
__device__ __forceinline__ uint32_t group_xor_reduce(uint32_t x) {
  if constexpr (G >= 2) x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);   // quad_perm 1,0,3,2
  if constexpr (G >= 4) x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);   // quad_perm 2,3,0,1
  if constexpr (G >= 8) x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, false);  // row_half_mirror
  if constexpr (G >= 16) x ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x140, 0xF, 0xF, false); // row_mirror
  if constexpr (G >= 32)  // row_bcast15 into rows 1 and 3 only
    x ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
  return x;
}

// Stage the LDS image with LDS-DMA (global_load_lds_dwordx4): each wave-instruction moves 1 KiB
// straight into LDS with no VGPR round trip, so the whole image is in flight at once.
// Parts: slicing tables (img_slice), the per-G join/round tables (img_group) and, for the
// variable-length kernel, the inverse-shift tables (img_extra).
// kBaseBytes: end of the group part (the extra part follows it; = kLdsCommonBytes for images with
// no group part). kStartBytes: stage only [kStartBytes, kBytes) (the rest is already in place).
template <uint32_t kBytes = kLdsImageBytes, int BLK = kBlock, uint32_t kBaseBytes = kLdsImageBytes,
          uint32_t kStartBytes = 0>
__device__ __forceinline__ void load_image(uint4* lds4, const uint4* __restrict__ img_common,
                                           const uint4* __restrict__ img_group,
                                           const uint4* __restrict__ img_extra = nullptr) {
  constexpr int kCommon = kLdsCommonBytes / 16;
  constexpr int kBase = kBaseBytes / 16;
  constexpr int kTotal = kBytes / 16;
  constexpr int kStart = kStartBytes / 16;
  constexpr int kChunks = (kTotal + 63) / 64;  // 1 KiB pieces (the last one may be partial)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int c = kStart / 64 + wave; c < kChunks; c += BLK / 64) {
    const int i = c * 64 + lane;
    if (i >= kStart && i < kTotal) {
      const uint4* src = i < kCommon ? img_common + i : (i < kBase ? img_group + (i - kCommon) : img_extra + (i - kBase));
      __builtin_amdgcn_global_load_lds(src, lds4 + c * 64, 16, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// 16-byte load through an address-space-1 pointer built from an integer address: the compiler
// emits global_load_dwordx4 (vmcnt only) instead of flat_load (vmcnt + lgkmcnt, which would make
// every LDS wait also wait for HBM).
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t clamp032(int32_t x) { return (uint32_t)min(max(x, 0), 32); }  // v_med3_i32
__device__ __forceinline__ uint4 gload16(uint64_t addr) {
  const __attribute__((address_space(1))) v4u32* p = (const __attribute__((address_space(1))) v4u32*)addr;
  const v4u32 x = *p;
  return make_uint4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ uint32_t gload4(uint64_t addr) {
  return *(const __attribute__((address_space(1))) uint32_t*)addr;
}
__device__ __forceinline__ uint32_t gload1(uint64_t addr) {
  return *(const __attribute__((address_space(1))) uint8_t*)addr;
}
// Global (not flat) stores: a flat store would also count in lgkmcnt, and every LDS wait of the fold
// (word4x2's s_waitcnt lgkmcnt(0)) would then wait for it.
__device__ __forceinline__ void gstore4(uint64_t addr, uint32_t v) { *(__attribute__((address_space(1))) uint32_t*)addr = v; }
__device__ __forceinline__ void gstore1(uint64_t addr, uint32_t v) {
  *(__attribute__((address_space(1))) uint8_t*)addr = (uint8_t)v;
}
// (any byte address: the hardware runs unaligned global stores, microbench/ua_store_mb.hip - exact, 0.96-0.98 of the
// aligned rate for 16-byte stores)
__device__ __forceinline__ void gstore2(uint64_t addr, uint32_t v) {
  *(__attribute__((address_space(1))) uint16_t*)addr = (uint16_t)v;
}
__device__ __forceinline__ void gstore8(uint64_t addr, uint64_t v) { *(__attribute__((address_space(1))) uint64_t*)addr = v; }
__device__ __forceinline__ void gstore16(uint64_t addr, uint4 v) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 x;
  x.x = v.x;
  x.y = v.y;
  x.z = v.z;
  x.w = v.w;
  *(__attribute__((address_space(1))) u32x4*)addr = x;
}
// Nontemporal 16-byte store, as an asm statement: beside a temporal store of the same value and address in the
// other arm of a branch, the compiler merged the two and dropped the nontemporal flag. (The waitcnt pass does not
// count an asm store; that only makes its later vmcnt waits stricter, and nothing reads these bytes back.)
__device__ __forceinline__ void gstore16_nt(uint64_t addr, uint4 v) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 x;
  x.x = v.x;
  x.y = v.y;
  x.z = v.z;
  x.w = v.w;
  asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(addr), "v"(x) : "memory");
}

// Keep bytes [lo, hi) of N 16-byte chunks (N = 4: a half line), zero the rest, from an image's chunk masks at LDS
// byte offset `off` (crc32_math.h kLdsW8MaskOff, kLdsStitchMaskOff: KEEP_FROM[a] = bytes [a, 16), then KEEP_TO[b] =
// bytes [0, b)): per chunk two ds_read_b128 and four ands, against mask_line's per-word shifts.
template <int N>
__device__ __forceinline__ void mask_chunks(uint4 (&v)[N], int32_t lo, int32_t hi, const uint32_t* lds,
                                            uint32_t off = kLdsW8MaskOff) {
  const uint4* t = reinterpret_cast<const uint4*>(lds + off / 4);
#pragma unroll
  for (int i = 0; i < N; i++) {
    const uint4 a = t[min(max(lo - 16 * i, 0), 16)], b = t[17 + min(max(hi - 16 * i, 0), 16)];
    v[i].x &= a.x & b.x;
    v[i].y &= a.y & b.y;
    v[i].z &= a.z & b.z;
    v[i].w &= a.w & b.w;
  }
}

// Nontemporal 16-byte load from scalar base g (an absolute global address, wave-uniform) + lane offset off: the
// base goes straight to the instruction's SGPR pair (a base rebuilt from a kernel pointer as ptr + (g - ptr) cost
// six scalar adds per load).
__device__ __forceinline__ uint4 gload16_nt(uint64_t g, uint32_t off) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const __attribute__((address_space(1))) u32x4* p = (const __attribute__((address_space(1))) u32x4*)(g + off);
  const u32x4 x = __builtin_nontemporal_load(p);
  return make_uint4(x.x, x.y, x.z, x.w);
}

// lane ^ 8 (DPP row_xmask:8 inside each row of 16)
__device__ __forceinline__ int32_t lane_xor8(int32_t x) { return __builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, false); }
// shift_{-m}, m in [0, 128): U_hi[m >> 4] o U_lo[m & 15] from the w8 image (crc32_math.h kLdsW8UnshiftOff)
__device__ __forceinline__ uint32_t w8_unshift(uint32_t t, uint32_t m, const uint32_t* lds) {
  t = nibble_map_uniform(t, lds, kLdsW8UnshiftOff + (m & 15u) * 512);
  return nibble_map_uniform(t, lds, kLdsW8UnshiftOff + 8192 + (m >> 4) * 512);
}
// shift_{(7-j)*128} from the w8 image's unreplicated join tables
__device__ __forceinline__ uint32_t w8_join(uint32_t s, const uint32_t* lds, uint32_t j) {
  const uint32_t* t = lds + kLdsW8JoinOff / 4 + j;
  uint32_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++) r[k] = t[k * 128 + __builtin_amdgcn_ubfe(s, 4 * k, 4) * 8];
  return xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), r[6] ^ r[7]);
}

// The streaming loops raise their wave priority while they issue the next task's loads, so the
// other wave on the SIMD (in its fold) does not delay them: config-1 kernel -0.5..1.0 %, arena line
// pass -1.5 % (profiles/r02/setprio_ab.log; priority 3 measured the same as 1); bench steps, two passes
// each: config 1 -0.9..-1.0 %, config 2 -0.3..-0.6 %, config 3 -0.8 % and -6.3 % (setprio_bench_ab.log).
#ifndef ANNETY_PRIO
#define ANNETY_PRIO 1
#endif
#define ANNETY_PRIO_HI() do { if constexpr (ANNETY_PRIO) __builtin_amdgcn_s_setprio(ANNETY_PRIO); } while (0)
#define ANNETY_PRIO_LO() do { if constexpr (ANNETY_PRIO) __builtin_amdgcn_s_setprio(0); } while (0)

// Coalesced loads for a wave's 8 KiB (64 consecutive 128-byte lines, line m = 8 b + j: block b, line j):
// load i covers block i whole, 16 B per lane, lane l reading chunk 4 l3 + 2 l5 + l4 of line j = l & 7 (lk =
// bit k of l). Every load is a contiguous 1 KiB, so it can be nontemporal (per-line loads, which touch 64 lines
// per instruction, run 2.4x slower nontemporal). coalesced_lane_offset() is that lane's byte offset inside a
// block. transpose_blocks() then swaps register bit 0 with lane bit 4 (permlane16) and register bit 1 with lane
// bit 5 (permlane32), one swap per dword pair: lane l holds half l3 of line j of block 2 l5 + l4 in v[0..3] and
// of block 4 + 2 l5 + l4 in v[4..7], ready for fold_halves(). DESIGN.md §2.3.
__device__ __forceinline__ uint32_t coalesced_lane_offset(uint32_t l) {
  return 128u * (l & 7u) + 16u * (4u * ((l >> 3) & 1u) + 2u * ((l >> 5) & 1u) + ((l >> 4) & 1u));
}
template <int D>
__device__ __forceinline__ void swap_stage(uint4 (&v)[8]) {
#pragma unroll
  for (int r = 0; r < 8; r++) {
    if (r & D) continue;
    uint32_t* a = reinterpret_cast<uint32_t*>(&v[r]);
    uint32_t* b = reinterpret_cast<uint32_t*>(&v[r | D]);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if constexpr (D == 1) {
        const auto p = __builtin_amdgcn_permlane16_swap(a[q], b[q], false, false);
        a[q] = p[0];
        b[q] = p[1];
      } else {
        const auto p = __builtin_amdgcn_permlane32_swap(a[q], b[q], false, false);
        a[q] = p[0];
        b[q] = p[1];
      }
    }
  }
}
__device__ __forceinline__ void transpose_blocks(uint4 (&v)[8]) {
  swap_stage<1>(v);
  swap_stage<2>(v);
}
// shift_64 through the byte tables at LDS byte offset `off` (kLdsByteMapBytes): 4 lookups at 2 VALU per
// address against the nibble map's 8; the lanes' random bytes cost 3-4-way bank conflicts, which the LDS
// has room for. microbench/bytemap_mb.hip: config 1 172.5-175.0 us against 175.6-179.9 with the nibble map.
// (The same 4-table form serves any shift whose byte tables sit at `off`: crc32_fixed32_nt_kernel's round map.)
__device__ __forceinline__ uint32_t byte_map64(uint32_t x, const uint32_t* lds, uint32_t off) {
  const uint32_t* t = lds + off / 4;
  return xor3(t[x & 255], t[256 + ((x >> 8) & 255)], t[512 + ((x >> 16) & 255)]) ^ t[768 + (x >> 24)];
}
// After transpose_blocks: the raw CRC (register 0) of line l & 7 of block 4 l3 + 2 l5 + l4. The two 64-byte
// chains v[0..3] and v[4..7] are half l3 of two lines; the halves meet across lane bit 3 (DPP row_ror:8 =
// lane ^ 8): lanes with l3 = 0 keep their first block's line, lanes with l3 = 1 their second block's,
// raw(line) = shift_64(raw(first half)) ^ raw(second half), shift_64 from the byte tables at `bm_off`.
__device__ __forceinline__ uint32_t fold_halves(const uint4 (&v)[8], const LaneCtx& k, const uint32_t* lds,
                                                uint32_t l3, uint32_t bm_off) {
  uint32_t xa = v[0].x, xb = v[4].x;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    word4x2(xa, v[i].y, xb, v[4 + i].y, k);
    word4x2(xa, v[i].z, xb, v[4 + i].z, k);
    word4x2(xa, v[i].w, xb, v[4 + i].w, k);
    word4x2(xa, i + 1 < 4 ? v[i + 1].x : 0u, xb, i + 1 < 4 ? v[5 + i].x : 0u, k);
  }
  const uint32_t send = l3 ? xa : xb;
  const uint32_t got = (uint32_t)__builtin_amdgcn_mov_dpp((int)send, 0x128, 0xF, 0xF, false);
  const uint32_t first = l3 ? got : xa, second = l3 ? xb : got;
  return byte_map64(first, lds, bm_off) ^ second;
}
// Block of a lane's line after fold_halves.
__device__ __forceinline__ uint32_t folded_block(uint32_t l) {
  return 4u * ((l >> 3) & 1u) + 2u * ((l >> 5) & 1u) + ((l >> 4) & 1u);
}

// Keep bytes [lo8/8, hi8/8) of a line (N = 8) or half line (N = 4), zero the rest (branch-free, per
// 32-bit word).
template <int N>
__device__ __forceinline__ void mask_line(uint4 (&v)[N], int32_t lo8, int32_t hi8) {
#pragma unroll
  for (int i = 0; i < N; i++) {
    uint32_t* w = reinterpret_cast<uint32_t*>(&v[i]);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int32_t p8 = (i * 16 + q * 4) * 8;
      const uint32_t keep_lo = (uint32_t)(0xFFFFFFFFull << clamp032(lo8 - p8));
      const uint32_t keep_hi = (uint32_t)(0xFFFFFFFFull >> clamp032(p8 + 32 - hi8));
      w[q] &= keep_lo & keep_hi;
    }
  }
}

// shift_{(7-g)*1024} for the leader lane of group g (k, v, g layout: conflict-free for the 8 leaders).
__device__ __forceinline__ uint32_t sb_join(uint32_t s, const uint32_t* lds, uint32_t g) {
  const uint32_t* t = lds + kLdsSbJoinOff / 4 + g;
  uint32_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++) r[k] = t[k * 128 + __builtin_amdgcn_ubfe(s, 4 * k, 4) * 8];
  return xor3(xor3(r[0], r[1], r[2]), xor3(r[3], r[4], r[5]), r[6] ^ r[7]);
}

// This call's extent from the launch_extent partials (ws + 8 + 4b: {lo, hi, sum, bad} of block b), reduced
// by the calling wave; every wave computes the same values.
__device__ __forceinline__ void extent_of(const uint64_t* ws, uint32_t parts, uint64_t& lo, uint64_t& hi,
                                          uint64_t& sum, uint64_t& bad) {
  lo = ~0ull;
  hi = sum = bad = 0;
  for (uint32_t b = threadIdx.x & 63; b < parts; b += 64) {
    const uint64_t* q = ws + 8 + 4 * (size_t)b;
    lo = min(lo, q[0]);
    hi = max(hi, q[1]);
    sum += q[2];
    bad |= q[3];
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    lo = min(lo, (uint64_t)__shfl_xor((unsigned long long)lo, d));
    hi = max(hi, (uint64_t)__shfl_xor((unsigned long long)hi, d));
    sum += (uint64_t)__shfl_xor((unsigned long long)sum, d);
    bad |= (uint64_t)__shfl_xor((unsigned long long)bad, d);
  }
}

// AutoChoice (crc32_kernels.h): true if the device picks the arena path for this call, with sp = the span of the
// batch's payload bytes. Called by whole waves (extent_of reduces across the wave); every wave of every launch of
// the call gets the same answer from the same partials.
__device__ __forceinline__ bool choose_arena(const AutoChoice& c, ArenaSpan& sp) {
  uint64_t lo, hi, sum, bad;
  extent_of(c.ws, c.parts, lo, hi, sum, bad);
  // (wave-uniform after the reduction: into scalar registers, so the span and the geometry derived from it stay
  // out of the VGPRs of the kernels that use them)
  auto uni = [](uint64_t x) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  };
  lo = uni(lo);
  hi = uni(hi);
  sum = uni(sum);
  bad = uni(bad);
  if (!(sum > 0 && hi > lo && bad == 0 && sum * 3 >= (hi - lo) * 2 && hi - lo < (32ull << 30))) return false;
  sp = arena_span(c.base + lo, c.base + hi);
  return arena_geom_of(sp.fs1 - sp.fs0, c.blocks).words <= c.cap_words;
}

}  // namespace
}  // namespace annety_crc
