// MI355X (gfx950) batch kernels for annety's checksum path (include/Crc32c.h:41-82, src/Crc32c.cc).
//
// Shape of the hot kernel:
//   * one workgroup of 512 lanes per CU (the 144.5 KiB LDS image leaves room for exactly one);
//   * a payload is owned by a lane-group of G lanes (G = 1..32); per round each lane reads one
//     128-byte line (8 back-to-back global_load_dwordx4), so a wave streams G*128*64/G = 8 KiB of
//     contiguous payload per round - the access shape that reaches the HBM roof on this chip;
//   * each lane folds its line through slicing-by-4 tables held in LDS as 32-way replicated paired
//     slots: one v_perm_b32 builds the address, one ds_read_b64 fetches two tables, no bank conflicts;
//   * lanes' partial registers are re-joined with the linear map shift_{(G-1-j)*128} (LDS nibble
//     tables, conflict-free) and a DPP xor-reduction; lane G-1 writes the digest.
// No MFMA: the work is a byte-indexed table lookup, not a contraction.
#include <hip/hip_runtime.h>

#include "crc32_kernels.h"
#include "crc32_math.h"

namespace annety_crc {
namespace {

constexpr int kBlock = 512;

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

struct LaneCtx {
  uint32_t L0;     // (replica*8) in byte 0, pair 0 in byte 2
  uint32_t L1;     // (replica*8) in byte 0, pair 1 in byte 2
  uint32_t slot4;  // replica*4 for the 4-byte join tables
};

// Absorb one 32-bit word. x = register ^ word (little-endian bytes b0..b3). Returns
// T3[b0]^T2[b1]^T1[b2]^T0[b3] ^ wnext, i.e. the register after the word, pre-xored with the next word.
// The four ds_read_b64 are issued back-to-back through inline asm so the compiler cannot narrow them to
// ds_read_b32 (which would use the 32-bank rule and conflict 2-way); the wait is tied to the results.
__device__ __forceinline__ uint32_t word4(uint32_t x, uint32_t wnext, const LaneCtx& k) {
  const uint32_t a0 = __builtin_amdgcn_perm(x, k.L0, 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(x, k.L0, 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(x, k.L1, 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(x, k.L1, 0x0C020700u);
  uint2 v0, v1, v2, v3;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v0) : "v"(a0));
  asm volatile("ds_read_b64 %0, %1" : "=v"(v1) : "v"(a1));
  asm volatile("ds_read_b64 %0, %1" : "=v"(v2) : "v"(a2));
  asm volatile("ds_read_b64 %0, %1" : "=v"(v3) : "v"(a3));
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));
  return xor3(xor3(v0.x, v1.y, v2.x), v3.y, wnext);
}

// Absorb one 128-byte line (8 x 16 B) into register s.
__device__ __forceinline__ uint32_t absorb_line(uint32_t s, const uint4 (&v)[8], const LaneCtx& k) {
  uint32_t x = s ^ v[0].x;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x = word4(x, v[i].y, k);
    x = word4(x, v[i].z, k);
    x = word4(x, v[i].w, k);
    x = word4(x, i + 1 < 8 ? v[i + 1].x : 0u, k);
  }
  return x;
}

// Apply a uniform nibble-table map (8 x 16 entries at LDS byte offset `off`, broadcast reads).
__device__ __forceinline__ uint32_t nibble_map_uniform(uint32_t s, const uint32_t* lds, uint32_t off) {
  const uint32_t* t = lds + off / 4;
  uint32_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++) r[k] = t[k * 16 + __builtin_amdgcn_ubfe(s, 4 * k, 4)];
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
// straight into LDS with no VGPR round trip, so the whole 144.5 KiB is in flight at once.
__device__ __forceinline__ void load_image(uint4* lds4, const uint4* __restrict__ img_slice,
                                           const uint4* __restrict__ img_group) {
  constexpr int kSlice = kLdsSliceBytes / 16;
  constexpr int kTotal = kLdsImageBytes / 16;  // 9248 x 16 B
  constexpr int kChunks = (kTotal + 63) / 64;   // 1 KiB pieces (the last one is half)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int c = wave; c < kChunks; c += kBlock / 64) {
    const int i = c * 64 + lane;
    if (i < kTotal) {
      const uint4* src = i < kSlice ? img_slice + i : img_group + (i - kSlice);
      __builtin_amdgcn_global_load_lds(src, lds4 + c * 64, 16, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Fixed-length batch: payload p = base + p*stride, `len_blocks` 16-byte blocks, 16-byte aligned.
// Chunks are aligned to the payload END (virtual leading zero blocks pad the first round), so every
// lane's last chunk ends (G-1-j)*128 bytes before the payload end and the join maps are constants.
//   FULL  : len is a multiple of G*128 (no virtual blocks)
//   RAW   : crc32_update semantics - no init injection, no final xor; state_in folded in by the writer
template <int G, bool FULL, bool RAW>
__global__ __launch_bounds__(kBlock) void crc32_fixed_kernel(const uint8_t* __restrict__ base, size_t n,
                                                             uint32_t len_blocks, size_t stride, uint32_t rounds,
                                                             uint32_t vlead, const uint4* __restrict__ img_slice,
                                                             const uint4* __restrict__ img_group,
                                                             const ShiftCols raw_shift_cols,
                                                             uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsImageBytes / 16];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);

  const uint32_t j = threadIdx.x & (G - 1);
  const size_t gid = (blockIdx.x * (size_t)kBlock + threadIdx.x) / G;
  const size_t ngroups = ((size_t)gridDim.x * kBlock) / G;
  const size_t ntasks = gid < n ? (n - 1 - gid) / ngroups + 1 : 0;

  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;

  // step = (task t, round r); loads run one step ahead of the compute (A/B double buffer)
  auto load_step = [&](size_t t, uint32_t r, uint4 (&v)[8]) {
    const uint8_t* p = base + (gid + t * ngroups) * stride;
    const uint32_t c = r * G + j;  // virtual chunk index of this lane
    if constexpr (FULL) {
      const uint4* s = reinterpret_cast<const uint4*>(p + (size_t)c * kChunkBytes);
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = s[i];
    } else {
      const int64_t b0 = (int64_t)c * 8 - (int64_t)vlead;  // real block index of v[0]
      const uint4* s = reinterpret_cast<const uint4*>(p);
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = (b0 + i >= 0) ? s[b0 + i] : make_uint4(0, 0, 0, 0);
    }
  };

  uint4 A[8], B[8];
  if (ntasks > 0) load_step(0, 0, A);  // first line in flight while the LDS image is staged
  load_image(lds4, img_slice, img_group);
  __syncthreads();

  const size_t nsteps = ntasks * rounds;
  size_t t_ld = 0, t_c = 0;
  uint32_t r_ld = 0, r_c = 0;
  auto advance = [&](size_t& t, uint32_t& r) {
    if (++r == rounds) {
      r = 0;
      ++t;
    }
  };
  advance(t_ld, r_ld);  // next step to load = step 1
  uint32_t s = 0;

  auto compute_step = [&](uint4 (&v)[8]) {
    uint32_t sin = 0;
    if (r_c > 0) {
      if constexpr (G > 1) sin = nibble_map_uniform(s, lds, kLdsRoundOff);
      else sin = s;
    }
    if constexpr (!RAW) {
      // init 0xFFFFFFFF == complementing the first 32 bits of the payload (the lane's register is 0
      // until the line holding payload byte 0), so it is folded into the data instead of the state.
      if constexpr (FULL) {
        v[0].x ^= (r_c == 0 && j == 0) ? kInit : 0u;
      } else {
        const uint32_t first_blk = (r_c * G + j == (vlead >> 3)) ? (vlead & 7u) : 8u;
#pragma unroll
        for (int i = 0; i < 8; i++) v[i].x ^= ((uint32_t)i == first_blk) ? kInit : 0u;
      }
    }
    s = absorb_line(sin, v, k);
    if (r_c == rounds - 1) {
      uint32_t t = s;
      if constexpr (G > 1) t = group_xor_reduce<G>(nibble_map_lane(s, lds, k.slot4));
      if (j == G - 1) {
        const size_t p = gid + t_c * ngroups;
        if constexpr (RAW) {
          // raw(M, s0) = shift_len(s0) ^ raw(M, 0)
          uint32_t s0 = out[p], sh = 0;
#pragma unroll
          for (int i = 0; i < 32; i++) sh ^= (0u - ((s0 >> i) & 1u)) & raw_shift_cols.c[i];
          out[p] = t ^ sh;
        } else {
          out[p] = ~t;
        }
      }
      s = 0;
    }
    advance(t_c, r_c);
  };

  for (size_t q = 0; q < nsteps; q += 2) {
    if (q + 1 < nsteps) load_step(t_ld, r_ld, B);
    advance(t_ld, r_ld);
    __builtin_amdgcn_sched_barrier(0);
    compute_step(A);
    if (q + 2 < nsteps) load_step(t_ld, r_ld, A);
    advance(t_ld, r_ld);
    __builtin_amdgcn_sched_barrier(0);
    if (q + 1 < nsteps) compute_step(B);
  }
}

// Single-round fast path (payload = exactly G lines, 16-byte aligned; BASELINE config 1 is G = 8):
// each step is one whole payload per lane-group, so there is no round state, and the per-lane line
// pointer advances by a constant per task. Loads run one task ahead (A/B double buffer).
template <int G>
__global__ __launch_bounds__(kBlock) void crc32_oneround_kernel(const uint8_t* __restrict__ base, size_t n,
                                                                size_t stride, const uint4* __restrict__ img_slice,
                                                                const uint4* __restrict__ img_group,
                                                                uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsImageBytes / 16];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);

  const uint32_t j = threadIdx.x & (G - 1);
  const size_t gid = (blockIdx.x * (size_t)kBlock + threadIdx.x) / G;
  const size_t ngroups = ((size_t)gridDim.x * kBlock) / G;
  const int ntasks = gid < n ? (int)((n - 1 - gid) / ngroups + 1) : 0;
  const size_t pstep = ngroups * stride;  // bytes between this group's consecutive payloads

  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;
  const uint32_t sinit = j == 0 ? kInit : 0u;  // init == complement of the payload's first word

  const uint8_t* lp = base + gid * stride + (size_t)j * kChunkBytes;
  uint32_t* op = out + gid;
  uint4 A[8], B[8];
  if (ntasks > 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) A[i] = reinterpret_cast<const uint4*>(lp)[i];
  }
  load_image(lds4, img_slice, img_group);
  __syncthreads();

  auto finish = [&](uint32_t s) {
    uint32_t t = s;
    if constexpr (G > 1) t = group_xor_reduce<G>(nibble_map_lane(s, lds, k.slot4));
    if (j == G - 1) *op = ~t;
    op += ngroups;
  };
  for (int t = 0; t < ntasks; t += 2) {
    if (t + 1 < ntasks) {
      const uint4* s = reinterpret_cast<const uint4*>(lp + pstep);
#pragma unroll
      for (int i = 0; i < 8; i++) B[i] = s[i];
    }
    __builtin_amdgcn_sched_barrier(0);
    finish(absorb_line(sinit, A, k));
    if (t + 2 < ntasks) {
      const uint4* s = reinterpret_cast<const uint4*>(lp + 2 * pstep);
#pragma unroll
      for (int i = 0; i < 8; i++) A[i] = s[i];
    }
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < ntasks) finish(absorb_line(sinit, B, k));
    lp += 2 * pstep;
  }
}

// ---------------------------------------------------------------------------------------------
// General kernel: any alignment, any length (variable-length batches and odd fixed shapes).
// Lines are the 128-byte lines of ABSOLUTE device memory, so every load is aligned and never leaves
// the 128-byte line (hence the page) of a valid byte. Bytes of the first/last line outside the payload
// are zeroed; leading zeros are free (the lane register is 0 there), the trailing zeros of the last
// line are removed after the join by one inverse shift unshift_{over} (64 KiB of nibble tables in
// global memory, L2-resident), over = bytes between the payload end and its last line end.
// Lines are assigned end-aligned over rounds of G lanes, exactly like the fixed kernel.
// `order` (optional) lists payload indices, e.g. grouped by length class so a wave's payloads finish
// together.
template <int G>
__global__ __launch_bounds__(kBlock) void crc32_var_kernel(const uint8_t* __restrict__ base, size_t n,
                                                           const uint64_t* __restrict__ d_off,
                                                           const uint32_t* __restrict__ d_len, uint64_t fstride,
                                                           uint32_t flen, const uint32_t* __restrict__ order,
                                                           const uint4* __restrict__ img_slice,
                                                           const uint4* __restrict__ img_group,
                                                           const uint32_t* __restrict__ unshift,
                                                           const uint32_t* __restrict__ short_init,
                                                           uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsImageBytes / 16];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);

  const uint32_t j = threadIdx.x & (G - 1);
  const size_t gid = (blockIdx.x * (size_t)kBlock + threadIdx.x) / G;
  const size_t ngroups = ((size_t)gridDim.x * kBlock) / G;

  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;

  load_image(lds4, img_slice, img_group);
  __syncthreads();

  for (size_t task = gid; task < n; task += ngroups) {
    const size_t p = order ? order[task] : task;
    const uint64_t off = d_off ? d_off[p] : (uint64_t)p * fstride;
    const uint32_t len = d_len ? d_len[p] : flen;
    if (len == 0) {
      if (j == G - 1) out[p] = 0u;
      continue;
    }
    const uint64_t a = (uint64_t)(uintptr_t)(base + off);
    const uint64_t e = a + len;
    const uint64_t line0 = a >> 7, line1 = (e - 1) >> 7;
    const uint32_t nlines = (uint32_t)(line1 - line0 + 1);
    const uint32_t rounds = (nlines + G - 1) / G;
    const uint32_t vlead = rounds * G - nlines;       // virtual leading lines
    const uint32_t lead = (uint32_t)(a & 127);        // payload start within its first line
    const uint32_t tailend = (uint32_t)(((e - 1) & 127) + 1);  // payload end within its last line
    const uint32_t over = 128 - tailend;
    uint32_t s = 0;
    for (uint32_t r = 0; r < rounds; r++) {
      if (r > 0) {
        if constexpr (G > 1) s = nibble_map_uniform(s, lds, kLdsRoundOff);
      }
      const int64_t li = (int64_t)(r * G + j) - (int64_t)vlead;  // real line index of this lane
      uint4 v[8];
      if (li >= 0) {
        const uint4* src = reinterpret_cast<const uint4*>((line0 + (uint64_t)li) << 7);
#pragma unroll
        for (int i = 0; i < 8; i++) v[i] = src[i];
        const bool first = li == 0, last = (uint32_t)li == nlines - 1;
        // init 0xFFFFFFFF == complement of payload bytes [0, 4) (len >= 4); they may straddle lines
        const int64_t lbase = (int64_t)li * 128 - (int64_t)lead;  // payload offset of line byte 0
        const bool has_init = len >= 4 && lbase < 4;
        if (first || last || has_init) {
          const int32_t lo = first ? (int32_t)lead : 0;
          const int32_t hi = last ? (int32_t)tailend : 128;
#pragma unroll
          for (int i = 0; i < 8; i++) {
            uint32_t* w = reinterpret_cast<uint32_t*>(&v[i]);
#pragma unroll
            for (int q = 0; q < 4; q++) {
              const int32_t pos = i * 16 + q * 4;
              // keep bytes with lo <= pos+b < hi
              const int32_t kb = min(max(lo - pos, 0), 4), ke = min(max(hi - pos, 0), 4);
              const uint32_t keep = ke > kb ? ((0xFFFFFFFFu >> (8 * (4 - (ke - kb)))) << (8 * kb)) : 0u;
              // complement payload bytes [0, 4): line positions [-lbase, 4 - lbase)
              const int32_t ib = min(max((int32_t)(-lbase) - pos, 0), 4);
              const int32_t ie = min(max((int32_t)(4 - lbase) - pos, 0), 4);
              const uint32_t inv = (has_init && ie > ib) ? ((0xFFFFFFFFu >> (8 * (4 - (ie - ib)))) << (8 * ib)) : 0u;
              w[q] = (w[q] & keep) ^ inv;
            }
          }
        }
        s = absorb_line(s, v, k);
      }
    }
    uint32_t t = s;
    if constexpr (G > 1) t = group_xor_reduce<G>(nibble_map_lane(s, lds, k.slot4));
    if (j == G - 1) {
      // remove the `over` trailing zero bytes of the last line
      if (over) {
        const uint32_t* u = unshift + over * 128;
        uint32_t r8 = 0;
#pragma unroll
        for (int kk = 0; kk < 8; kk++) r8 ^= u[kk * 16 + ((t >> (4 * kk)) & 15u)];
        t = r8;
      }
      if (len < 4) t ^= short_init[len];  // shift_len(0xFFFFFFFF): init not expressible as complement
      out[p] = ~t;
    }
  }
}

template <int G>
hipError_t launch_var_g(const VarLaunch& a, hipStream_t stream) {
  const size_t lanes = a.n * (size_t)G;
  size_t blocks = (lanes + kBlock - 1) / kBlock;
  if (blocks > a.max_blocks) blocks = a.max_blocks;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((crc32_var_kernel<G>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                     static_cast<const uint8_t*>(a.base), a.n, a.off, a.len, a.fixed_stride, a.fixed_len, a.order,
                     static_cast<const uint4*>(a.img_slice), static_cast<const uint4*>(a.img_group), a.unshift,
                     a.short_init, a.out);
  return hipGetLastError();
}

template <int G, bool FULL, bool RAW>
hipError_t launch_g(const FixedLaunch& a, hipStream_t stream) {
  const size_t lanes = a.n * (size_t)G;
  size_t blocks = (lanes + kBlock - 1) / kBlock;
  if (blocks > a.max_blocks) blocks = a.max_blocks;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((crc32_fixed_kernel<G, FULL, RAW>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                     static_cast<const uint8_t*>(a.base), a.n, a.len_blocks, a.stride, a.rounds, a.vlead,
                     static_cast<const uint4*>(a.img_slice), static_cast<const uint4*>(a.img_group), a.raw_shift_cols,
                     a.out);
  return hipGetLastError();
}

template <int G>
hipError_t launch_one_g(const FixedLaunch& a, hipStream_t stream) {
  const size_t lanes = a.n * (size_t)G;
  size_t blocks = (lanes + kBlock - 1) / kBlock;
  if (blocks > a.max_blocks) blocks = a.max_blocks;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((crc32_oneround_kernel<G>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                     static_cast<const uint8_t*>(a.base), a.n, a.stride, static_cast<const uint4*>(a.img_slice),
                     static_cast<const uint4*>(a.img_group), a.out);
  return hipGetLastError();
}

hipError_t launch_one(const FixedLaunch& a, hipStream_t stream) {
  switch (a.group) {
    case 1: return launch_one_g<1>(a, stream);
    case 2: return launch_one_g<2>(a, stream);
    case 4: return launch_one_g<4>(a, stream);
    case 8: return launch_one_g<8>(a, stream);
    case 16: return launch_one_g<16>(a, stream);
    case 32: return launch_one_g<32>(a, stream);
    default: return hipErrorInvalidValue;
  }
}

template <bool FULL, bool RAW>
hipError_t launch_full(const FixedLaunch& a, hipStream_t stream) {
  switch (a.group) {
    case 1: return launch_g<1, FULL, RAW>(a, stream);
    case 2: return launch_g<2, FULL, RAW>(a, stream);
    case 4: return launch_g<4, FULL, RAW>(a, stream);
    case 8: return launch_g<8, FULL, RAW>(a, stream);
    case 16: return launch_g<16, FULL, RAW>(a, stream);
    case 32: return launch_g<32, FULL, RAW>(a, stream);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t launch_fixed(const FixedLaunch& a, hipStream_t stream) {
  if (!a.raw && a.full && a.rounds == 1) return launch_one(a, stream);
  if (a.raw) return a.full ? launch_full<true, true>(a, stream) : launch_full<false, true>(a, stream);
  return a.full ? launch_full<true, false>(a, stream) : launch_full<false, false>(a, stream);
}

hipError_t launch_var(const VarLaunch& a, hipStream_t stream) {
  switch (a.group) {
    case 1: return launch_var_g<1>(a, stream);
    case 2: return launch_var_g<2>(a, stream);
    case 4: return launch_var_g<4>(a, stream);
    case 8: return launch_var_g<8>(a, stream);
    case 16: return launch_var_g<16>(a, stream);
    case 32: return launch_var_g<32>(a, stream);
    default: return hipErrorInvalidValue;
  }
}

int fixed_kernel_block() { return kBlock; }

}  // namespace annety_crc
