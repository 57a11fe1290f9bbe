// MI355X (gfx950) batch kernels for annety's checksum path (include/Crc32c.h:41-82, src/Crc32c.cc).
//
// Shape of the hot kernel:
//   * one workgroup of 512 lanes per CU (the 144.5 KiB LDS image leaves room for exactly one);
//   * a payload is owned by a lane-group of G lanes (G = 1..32); per round each lane folds one 128-byte
//     line, and a wave streams 8 KiB of contiguous payload per round. The per-line kernels read a lane's
//     line as 8 back-to-back global_load_dwordx4; the nontemporal kernels (crc32_onekib_nt_kernel,
//     crc32_fixed32_nt_kernel) read 8 coalesced 1 KiB pieces and transpose them in registers;
//   * each lane folds its line through slicing-by-4 tables held in LDS as 32-way replicated paired
//     slots: one v_perm_b32 builds the address, one ds_read_b64 fetches two tables, no bank conflicts;
//   * lanes' partial registers are re-joined with the linear map shift_{(G-1-j)*128} (LDS nibble
//     tables, conflict-free) and a DPP xor-reduction; lane G-1 writes the digest.
// No MFMA: the work is a byte-indexed table lookup, not a contraction.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "crc32_device.h"
#include "crc32_kernels.h"
#include "crc32_math.h"

namespace annety_crc {
namespace {

// Fixed-length batch: payload p = base + p*stride, 16-byte aligned, `rounds` rounds of G lines per payload.
// Chunks are aligned to the payload END (virtual leading zero blocks pad the first round), so every
// lane's last chunk ends (G-1-j)*128 bytes before the payload end and the join maps are constants.
//   FULL  : len is a multiple of G*128 (no virtual blocks)
//   RAW   : crc32_update semantics - no init injection, no final xor; state_in folded in by the writer
template <int G, bool FULL, bool RAW, int VWG = kVwg>
__global__ __launch_bounds__(kBlock) void crc32_fixed_kernel(const uint8_t* __restrict__ base, size_t n,
                                                             size_t stride, uint32_t rounds,
                                                             uint32_t vlead, const uint4* __restrict__ img_slice,
                                                             const uint4* __restrict__ img_group,
                                                             const ShiftCols raw_shift_cols,
                                                             uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsImageBytes / 16];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);

  const uint32_t j = threadIdx.x & (G - 1);
  const size_t gid = group_id<kBlock, G, VWG>();
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
    s = absorb_line(sin, v, k, lds);
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

  // unconditional loads (a step past the end re-reads step 0's line): see crc32_oneround_kernel
  for (size_t q = 0; q < nsteps; q += 2) {
    ANNETY_PRIO_HI();
    {
      const bool ok = q + 1 < nsteps;
      load_step(ok ? t_ld : 0, ok ? r_ld : 0u, B);
    }
    advance(t_ld, r_ld);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    compute_step(A);
    ANNETY_PRIO_HI();
    {
      const bool ok = q + 2 < nsteps;
      load_step(ok ? t_ld : 0, ok ? r_ld : 0u, A);
    }
    advance(t_ld, r_ld);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    if (q + 1 < nsteps) compute_step(B);
  }
}

// Single-round fast path (payload = exactly G lines, 16-byte aligned; BASELINE config 1 is G = 8):
// each step is one whole payload per lane-group, so there is no round state, and the per-lane line
// pointer advances by a constant per task. Loads run one task ahead (A/B double buffer). The arena line
// pass (crc32_arena_lines.h) is this loop with suffix-CRC outputs instead of digests.
template <int G, int BLK = kBlock, int VWG = kVwg>
__global__ __launch_bounds__(BLK) void crc32_oneround_kernel(const uint8_t* __restrict__ base, size_t n,
                                                                size_t stride, const uint4* __restrict__ img_slice,
                                                                const uint4* __restrict__ img_group,
                                                                uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsImageBytes / 16];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);

  const uint32_t j = threadIdx.x & (G - 1);
  const size_t gid = group_id<BLK, G, VWG>();
  const size_t ngroups = ((size_t)gridDim.x * BLK) / G;
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
  load_image<kLdsImageBytes, BLK>(lds4, img_slice, img_group);
  __syncthreads();

  auto finish = [&](uint32_t s) {
    uint32_t t = s;
    if constexpr (G > 1) t = group_xor_reduce<G>(nibble_map_lane(s, lds, k.slot4));
    if (j == G - 1) *op = ~t;
    op += ngroups;
  };
  // Loads are unconditional (past the last task a group re-reads its current line, an L2 hit): with the
  // next task's loads behind a branch the waitcnt pass merges the two paths and waits vmcnt(0) before
  // every fold, which serialises the A/B double buffer.
  for (int t = 0; t < ntasks; t += 2) {
    ANNETY_PRIO_HI();
    {
      const uint4* s = reinterpret_cast<const uint4*>(t + 1 < ntasks ? lp + pstep : lp);
#pragma unroll
      for (int i = 0; i < 8; i++) B[i] = s[i];
    }
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    finish(absorb_line(sinit, A, k, lds));
    ANNETY_PRIO_HI();
    {
      const uint4* s = reinterpret_cast<const uint4*>(t + 2 < ntasks ? lp + 2 * pstep : lp);
#pragma unroll
      for (int i = 0; i < 8; i++) A[i] = s[i];
    }
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    if (t + 1 < ntasks) finish(absorb_line(sinit, B, k, lds));
    lp += 2 * pstep;
  }
}

// Contiguous 1 KiB payloads (stride 1024, n a multiple of 8: BASELINE configs 1 and 4): the one-round
// kernel's work with coalesced nontemporal loads. A wave's task is 8 consecutive payloads (8 KiB); load i reads
// payload i whole (1 KiB contiguous, 16 B per lane) and transpose_blocks() / fold_halves() (crc32_device.h)
// bring each lane one line, of payload folded_block(lane). Same box, alternating: 167-169 us per 1 GiB launch
// against 180 us for crc32_oneround_kernel<8> (microbench/nt_mb.hip). Addresses are one scalar base per task
// plus immediate offsets: with a runtime stride the per-load scalar arithmetic cost 7 us of it.
template <int BLK = kBlock, int VWG = kVwg>
__global__ __launch_bounds__(BLK) void crc32_onekib_nt_kernel(const uint8_t* __restrict__ base, size_t n,
                                                              const uint4* __restrict__ img_slice,
                                                              const uint4* __restrict__ img_group,
                                                              const uint4* __restrict__ img_bytemap,
                                                              uint32_t* __restrict__ out) {
  static_assert(BLK % 64 == 0 && (VWG == 0 || VWG % 64 == 0), "a wave's lanes must be 8 consecutive lane groups");
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsFixedNtImageBytes / 16];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  const uint32_t l = threadIdx.x & 63, j = l & 7, l3 = (l >> 3) & 1;
  const size_t gid = group_id<BLK, 8, VWG>();
  // the wave's first payload (its 8 lane groups are 8 consecutive groups), wave-uniform
  const size_t p0 = ((size_t)__builtin_amdgcn_readfirstlane((uint32_t)(gid >> 32)) << 32) |
                    (size_t)(__builtin_amdgcn_readfirstlane((uint32_t)gid) & ~7u);
  const size_t ngroups = ((size_t)gridDim.x * BLK) / 8;
  const int ntasks = p0 < n ? (int)((n - 1 - p0) / ngroups + 1) : 0;
  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;
  const uint32_t lane_off = coalesced_lane_offset(l);
  const uint32_t sinit = (j == 0 && l3 == 0) ? kInit : 0u;  // the payloads' first words (line 0, half 0)
  const uint8_t* wp = base + p0 * 1024 + lane_off;
  const size_t pstep = ngroups * 1024;
  uint32_t* op = out + p0 + folded_block(l);
  auto load = [&](const uint8_t* a, uint4 (&v)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const v4u32 x = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(a + 1024 * i));
      v[i] = make_uint4(x.x, x.y, x.z, x.w);
    }
  };
  uint4 A[8], B[8];
  if (ntasks > 0) load(wp, A);
  load_image<kLdsFixedNtImageBytes, BLK, kLdsImageBytes>(lds4, img_slice, img_group, img_bytemap);
  __syncthreads();
  auto finish = [&](uint4 (&v)[8]) __attribute__((always_inline)) {
    transpose_blocks(v);
    v[0].x ^= sinit;
    v[4].x ^= sinit;
    const uint32_t c =
        group_xor_reduce<8>(nibble_map_lane(fold_halves(v, k, lds, l3, kLdsImageBytes), lds, k.slot4));
    if (j == 7) *op = ~c;
    op += ngroups;
  };
  // unconditional loads, as in crc32_oneround_kernel (past the last task a wave re-reads its current one)
  for (int t = 0; t < ntasks; t += 2) {
    ANNETY_PRIO_HI();
    load(t + 1 < ntasks ? wp + pstep : wp, B);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    finish(A);
    ANNETY_PRIO_HI();
    load(t + 2 < ntasks ? wp + 2 * pstep : wp, A);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    if (t + 1 < ntasks) finish(B);
    wp += 2 * pstep;
  }
}

// G = 32 fixed batches whose length is a multiple of 4 KiB (n even; the long-payload split's 64 KiB segments
// of config 2): crc32_fixed_kernel<32, true, false>'s rounds with coalesced nontemporal loads. A wave = two
// lane groups (lanes 0-31 and 32-63, payloads g0 and g0 + 1); a round reads 4 KiB of each. Load i covers
// block blk_of(i) of the wave's 8 KiB (group = bit 2, block of the 4 KiB = bits 0-1), chosen so that after
// transpose_blocks() / fold_halves() lane l holds line j = 8 (2 l3 + l4) + (l & 7) of its own group's round:
// the groups stay the two half-waves (group_xor_reduce<32> as before) and the join takes slot j. The round
// register enters the chains that fold the first halves: a lane with l3 = 0 folds the first half of its own line
// (chain a) and of its partner's (lane ^ 8, chain b), so it injects its own and the partner's register.
template <int BLK = kBlock, int VWG = kVwg>
__global__ __launch_bounds__(BLK) void crc32_fixed32_nt_kernel(const uint8_t* __restrict__ base, size_t n,
                                                               size_t stride, uint32_t rounds,
                                                               const uint4* __restrict__ img_slice,
                                                               const uint4* __restrict__ img_group,
                                                               const uint4* __restrict__ img_bytemap,
                                                               uint32_t* __restrict__ out) {
  static_assert(BLK % 64 == 0 && (VWG == 0 || VWG % 64 == 0), "a wave's lanes must be 2 consecutive lane groups");
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsFixed32NtImageBytes / 16];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  const uint32_t l = threadIdx.x & 63, l3 = (l >> 3) & 1, l4 = (l >> 4) & 1;
  const size_t gid = group_id<BLK, 32, VWG>();
  const size_t g0 = ((size_t)__builtin_amdgcn_readfirstlane((uint32_t)(gid >> 32)) << 32) |
                    (size_t)(__builtin_amdgcn_readfirstlane((uint32_t)gid) & ~1u);
  const size_t ngroups = ((size_t)gridDim.x * BLK) / 32;
  const size_t ntasks = g0 < n ? (n - 1 - g0) / ngroups + 1 : 0;  // the same for both groups (n, g0 even)
  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  const uint32_t jl = 8 * (2 * l3 + l4) + (l & 7);  // this lane's line of the round
  k.slot4 = jl << 2;
  const uint32_t lane_off = coalesced_lane_offset(l);
  const uint32_t sinit = (l & 31) == 0 ? kInit : 0u;  // line 0, half 0, chunk 0 of each payload (lanes 0, 32)
  // load i -> block blk_of(i): group (i >> 1) & 1, block 2 (i >> 2) + (i & 1) of that group's 4 KiB
  auto load_step = [&](size_t t, uint32_t r, uint4 (&v)[8]) __attribute__((always_inline)) {
    const uint8_t* b0 = base + (g0 + t * ngroups) * stride + (size_t)r * 4096 + lane_off;
    const uint8_t* b1 = b0 + stride;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint8_t* a = (((i >> 1) & 1) ? b1 : b0) + 1024 * (2 * (i >> 2) + (i & 1));
      const v4u32 x = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(a));
      v[i] = make_uint4(x.x, x.y, x.z, x.w);
    }
  };
  uint4 A[8], B[8];
  if (ntasks > 0) load_step(0, 0, A);
  load_image<kLdsFixed32NtImageBytes, BLK, kLdsImageBytes>(lds4, img_slice, img_group, img_bytemap);
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
  advance(t_ld, r_ld);
  uint32_t s = 0;
  auto compute_step = [&](uint4 (&v)[8]) __attribute__((always_inline)) {
    transpose_blocks(v);
    uint32_t sin = 0;
    if (r_c > 0) sin = byte_map64(s, lds, kLdsFixedNtImageBytes);  // shift_{31*128}
    const uint32_t sp = (uint32_t)__builtin_amdgcn_mov_dpp((int)sin, 0x128, 0xF, 0xF, false);  // lane ^ 8's
    v[0].x ^= l3 ? 0u : (r_c == 0 ? sinit : sin);
    v[4].x ^= l3 ? 0u : sp;
    s = fold_halves(v, k, lds, l3, kLdsImageBytes);
    if (r_c == rounds - 1) {
      const uint32_t c = group_xor_reduce<32>(nibble_map_lane(s, lds, k.slot4));
      if ((l & 31) == 31) out[g0 + (l >> 5) + t_c * ngroups] = ~c;
      s = 0;
    }
    advance(t_c, r_c);
  };
  for (size_t q = 0; q < nsteps; q += 2) {
    ANNETY_PRIO_HI();
    {
      const bool ok = q + 1 < nsteps;
      load_step(ok ? t_ld : 0, ok ? r_ld : 0u, B);
    }
    advance(t_ld, r_ld);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    compute_step(A);
    ANNETY_PRIO_HI();
    {
      const bool ok = q + 2 < nsteps;
      load_step(ok ? t_ld : 0, ok ? r_ld : 0u, A);
    }
    advance(t_ld, r_ld);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    if (q + 1 < nsteps) compute_step(B);
  }
}

// ---------------------------------------------------------------------------------------------
// General kernel: any alignment, any length (variable-length batches and odd fixed shapes).
// Lines are the 128-byte lines of ABSOLUTE device memory, so every load is aligned and never leaves
// the 128-byte line (hence the page) of a valid byte. Bytes of the first/last line outside the payload
// are zeroed; leading zeros are free (the lane register is 0 there), the trailing zeros of the last
// line are removed after the join by one inverse shift unshift_{over} (64 KiB of nibble tables in
// global memory, L2-resident), over = bytes between the payload end and its last line end.
// Lines are assigned end-aligned over rounds of G lanes, exactly like the fixed kernel, and the
// (task, round) steps are double-buffered across task boundaries.
// `order`/`range` (optional) select the tasks: order[range[0] .. range[1]) are payload indices sorted
// by line count (crc32_bucket_place, crc32_arena.hip), so the payloads of a wave finish together and each length
// class runs with its own G. Zero-length payloads never reach this kernel (the bucket pass writes 0).
struct VarTask {
  uint64_t line0;    // absolute index of the payload's first 128-byte line
  uint32_t nlines, rounds, vlead, lead, tailend, len, p;
  uint32_t state;    // update mode: the register before this payload (crc32_update semantics)
  bool valid;
};

// Raw task descriptor: {absolute start address lo, hi, length, payload index}. In sorted mode the
// bucket pass writes them contiguously, so a task costs one 16-byte load and no dependent chain.
template <int G>
__device__ __forceinline__ VarTask decode_task(uint4 d, bool valid) {
  VarTask k{};
  k.valid = valid;
  if (!valid) return k;
  const uint64_t a = ((uint64_t)d.y << 32) | d.x;
  const uint32_t len = d.z;
  const uint64_t e = a + len;  // len > 0
  k.line0 = a >> 7;
  k.nlines = (uint32_t)(((e - 1) >> 7) - k.line0 + 1);
  k.rounds = (k.nlines + G - 1) / G;
  k.vlead = k.rounds * G - k.nlines;
  k.lead = (uint32_t)(a & 127);
  k.tailend = (uint32_t)(((e - 1) & 127) + 1);
  k.len = len;
  k.p = d.w;
  return k;
}

// Branch-free descriptor fetch: past the end it re-reads the last entry (validity is tracked apart),
// so the compiler never has to wait on the load to merge two paths.
template <bool SORTED>
__device__ __forceinline__ uint4 raw_task(size_t t, size_t end, const uint8_t* base, const uint4* desc,
                                          uint64_t fstride, uint32_t flen) {
  const size_t tc = t < end ? t : (end ? end - 1 : 0);
  if constexpr (SORTED) {
    return desc[tc];
  } else {
    const uint64_t a = (uint64_t)(uintptr_t)(base + (uint64_t)tc * fstride);
    return make_uint4((uint32_t)a, (uint32_t)(a >> 32), flen, (uint32_t)tc);
  }
}

//   UPD: crc32_update semantics (include/Crc32c.h:71-82): out[p] holds the register before payload p on
//        entry and after it on exit (no init, no final xor). The entry register s is injected like the
//        init: raw(M, s) = raw(M ^ (s as payload bytes 0..3, little-endian), 0) when len >= 4, and
//        shift_len(s) ^ raw(M, 0) below that.
//   PROBE (microbench only; product = 0): bit 0 drops the byte masks, bit 1 the unshift - wrong
//        digests, used to measure what those stages cost (microbench/ab3.hip).
//   STAGE: which parts of the LDS image this call stages - 2 = all of it, and none when the block has no
//        task (a kernel of its own); 1 = all of it always; 0 = only the G-specific group part (the later
//        length classes of crc32_var_sorted_kernel, whose first class staged the rest).
template <int G, bool SORTED, bool UPD, int VWG, int PROBE, int STAGE>
__device__ __forceinline__ void var_class(uint4* lds4, const uint8_t* __restrict__ base, size_t n, uint64_t fstride,
                                          uint32_t flen, const uint4* __restrict__ desc,
                                          const uint32_t* __restrict__ range, const uint4* __restrict__ img_slice,
                                          const uint4* __restrict__ img_group, const uint4* __restrict__ img_unshift,
                                          uint32_t* __restrict__ out) {
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);

  const uint32_t j = threadIdx.x & (G - 1);
  const size_t gid = group_id<kBlock, G, VWG>();
  const size_t ngroups = ((size_t)gridDim.x * kBlock) / G;
  const size_t t_begin = range ? range[0] : 0;
  const size_t t_end = range ? range[1] : n;

  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;

  auto raw = [&](size_t t) { return raw_task<SORTED>(t, t_end, base, desc, fstride, flen); };
  // Loads are unconditional (clamped to a harmless valid line for virtual lines and finished groups)
  // and every step runs the same instruction sequence, so the compiler's vmcnt bookkeeping stays exact.
  const uint64_t safe_line = (uint64_t)(uintptr_t)base >> 7;
  auto load = [&](const VarTask& tk, uint32_t r, uint4 (&v)[8]) {
    const int64_t li = (int64_t)(r * G + j) - (int64_t)tk.vlead;
    const uint64_t line = tk.valid ? tk.line0 + (uint64_t)(li > 0 ? li : 0) : safe_line;
    const uint64_t src = line << 7;
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = gload16(src + 16 * i);
  };

  // Software pipeline over steps q = (task, round):
  //   step q computes  (dec0, r0) on the buffer loaded at q-1,
  //          loads     (dec1, r1) = step q+1, decoded from the descriptor fetched at q-1,
  //          fetches   the raw descriptor of step q+2's task.
  size_t t0 = t_begin + gid;
  // a block with no task (an empty length class of the sorted path, or fewer tasks than lane groups)
  // leaves before its first descriptor load and the image staging
  if (!__syncthreads_or(t0 < t_end)) {
    if constexpr (STAGE == 1) {
      load_image<kLdsVarImageBytes>(lds4, img_slice, img_group, img_unshift);
      __syncthreads();
    }
    return;
  }
  VarTask dec0 = decode_task<G>(raw(t0), t0 < t_end);
  if constexpr (UPD) dec0.state = dec0.valid ? out[dec0.p] : 0u;
  uint32_t r0 = 0;
  size_t t1 = dec0.rounds > 1 ? t0 : t0 + ngroups;
  uint32_t r1 = dec0.rounds > 1 ? 1u : 0u;
  uint4 d1 = raw(t1);

  uint4 A[8], B[8];
  load(dec0, r0, A);
  if constexpr (STAGE == 0)
    load_image<kLdsImageBytes, kBlock, kLdsImageBytes, kLdsCommonBytes>(lds4, img_slice, img_group);
  else
    load_image<kLdsVarImageBytes>(lds4, img_slice, img_group, img_unshift);
  __syncthreads();

  uint32_t s = 0;
  auto compute = [&](uint4 (&v)[8], const VarTask& cur, uint32_t r_c) {
    if (r_c > 0) {
      if constexpr (G > 1) s = nibble_map_uniform(s, lds, kLdsRoundOff);
    }
    const int64_t li = (int64_t)(r_c * G + j) - (int64_t)cur.vlead;  // real line index of this lane
    if (cur.valid && li >= 0) {
      // Byte masks of the payload's first and last line, branch-free per word (SIMT runs this block for
      // the whole wave whenever one lane needs it, so it must be cheap):
      //   lead side: keep bytes >= A, complement bytes [A, B)   -> w = keepA & (w ^ ~keepB)
      //     (the init 0xFFFFFFFF is the complement of payload bytes [0, 4) when len >= 4; if the first
      //      line holds fewer than 4 payload bytes the rest spills into the second line)
      //   tail side: keep bytes < hi                            -> w &= keepH
      const bool first = li == 0, last = (uint32_t)li == cur.nlines - 1;
      const bool spill = li == 1 && cur.lead > 124 && cur.len >= 4;
      if ((PROBE & 1) == 0 && (first || spill)) {
        const int32_t A8 = first ? (int32_t)cur.lead * 8 : 0;
        if constexpr (UPD) {
          // the register's bytes land at payload bytes 0..3, i.e. line bit offset S8 (< 0 on the spill line)
          const int32_t S8 = ((int32_t)cur.lead - (first ? 0 : 128)) * 8;
          const uint32_t reg = cur.len < 4 ? 0u : cur.state;
#pragma unroll
          for (int i = 0; i < 8; i++) {
            uint32_t* w = reinterpret_cast<uint32_t*>(&v[i]);
#pragma unroll
            for (int q = 0; q < 4; q++) {
              const int32_t p8 = (i * 16 + q * 4) * 8;
              const uint32_t keepA = (uint32_t)(0xFFFFFFFFull << clamp032(A8 - p8));
              const int32_t x = S8 - p8;  // bit offset of register byte 0 inside this word
              const uint32_t sw = x >= 32 || x <= -32 ? 0u : (x >= 0 ? reg << x : reg >> -x);
              w[q] = (keepA & w[q]) ^ sw;
            }
          }
        } else {
          const int32_t B8 = cur.len < 4 ? A8 : ((int32_t)cur.lead + 4 - (first ? 0 : 128)) * 8;
#pragma unroll
          for (int i = 0; i < 8; i++) {
            uint32_t* w = reinterpret_cast<uint32_t*>(&v[i]);
#pragma unroll
            for (int q = 0; q < 4; q++) {
              const int32_t p8 = (i * 16 + q * 4) * 8;
              const uint32_t keepA = (uint32_t)(0xFFFFFFFFull << clamp032(A8 - p8));
              const uint32_t keepB = (uint32_t)(0xFFFFFFFFull << clamp032(B8 - p8));
              w[q] = keepA & (w[q] ^ ~keepB);
            }
          }
        }
      }
      if ((PROBE & 1) == 0 && last) {
        const int32_t H8 = (int32_t)cur.tailend * 8;
#pragma unroll
        for (int i = 0; i < 8; i++) {
          uint32_t* w = reinterpret_cast<uint32_t*>(&v[i]);
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const int32_t p8 = (i * 16 + q * 4) * 8;
            w[q] &= (uint32_t)(0xFFFFFFFFull >> clamp032(p8 + 32 - H8));
          }
        }
      }
      s = absorb_line(s, v, k, lds);
    }
    if (r_c == cur.rounds - 1) {
      uint32_t t = s;
      if constexpr (G > 1) t = group_xor_reduce<G>(nibble_map_lane(s, lds, k.slot4));
      if (cur.valid && j == G - 1) {
        const uint32_t over = 128 - cur.tailend;  // trailing zero bytes of the last line
        if ((PROBE & 2) == 0 && over) {  // shift_{-over} = U_hi[over >> 4] o U_lo[over & 15], both from LDS
          t = nibble_map_uniform(t, lds, kLdsUnshiftOff + (over & 15u) * 512);
          t = nibble_map_uniform(t, lds, kLdsUnshiftOff + 8192 + (over >> 4) * 512);
        }
        if constexpr (UPD) {
          if (cur.len < 4) t ^= shift_bits(cur.state, 8u * cur.len);  // <= 24 bit steps
          out[cur.p] = t;
        } else {
          if (cur.len < 4) {  // shift_len(0xFFFFFFFF): init not expressible as a complement (constants)
            constexpr uint32_t k1 = shift_bits(kInit, 8), k2 = shift_bits(kInit, 16), k3 = shift_bits(kInit, 24);
            t ^= cur.len == 1 ? k1 : (cur.len == 2 ? k2 : k3);
          }
          out[cur.p] = ~t;
        }
      }
      s = 0;
    }
  };

  auto step = [&](uint4 (&cur_buf)[8], uint4 (&nxt_buf)[8]) {
    VarTask dec1 = decode_task<G>(d1, t1 < t_end);
    if constexpr (UPD) dec1.state = dec1.valid ? out[dec1.p] : 0u;  // read one step before it is used
    const bool more = r1 + 1 < dec1.rounds;
    const size_t t2 = more ? t1 : t1 + ngroups;
    const uint32_t r2 = more ? r1 + 1 : 0u;
    const uint4 d2 = raw(t2);
    load(dec1, r1, nxt_buf);
    __builtin_amdgcn_sched_barrier(0);
    compute(cur_buf, dec0, r0);
    dec0 = dec1;
    r0 = r1;
    t1 = t2;
    r1 = r2;
    d1 = d2;
  };

  // (three buffers, two steps' loads in flight, measured no faster on the small class: DESIGN.md §7.2)
  while (dec0.valid) {
    step(A, B);
    step(B, A);  // harmless when the group ran out of work on the first half: nothing is stored
  }
}

// Byte masks of one half-line (bytes [64 h, 64 h + 64) of a payload line, h = the lane's l3), for the line with
// real index li (var_class's masks, per half): li < 0 = virtual (zero), li = 0 the first line (bytes before the
// payload dropped, the init or the caller's register on payload bytes 0..3), li = 1 the spill line when the
// first holds fewer than 4 payload bytes, li = nlines - 1 the last (bytes after the payload dropped).
//   keep bits [A8, H8) of the line; non-UPD: complement bits [A8, B8) (the init); UPD: xor the register at S8.
struct HalfMask {
  int32_t A8, B8, H8, S8;
  uint32_t reg;
  uint32_t need;  // some byte of the line changes
};
template <bool UPD>
__device__ __forceinline__ HalfMask half_mask(int32_t li, const VarTask& cur) {
  HalfMask m;
  const bool first = li == 0;
  const bool spill = li == 1 && cur.lead > 124 && cur.len >= 4;
  m.A8 = li < 0 ? 1024 : (first ? (int32_t)cur.lead * 8 : 0);
  m.H8 = li == (int32_t)cur.nlines - 1 ? (int32_t)cur.tailend * 8 : 1024;
  m.S8 = first || spill ? ((int32_t)cur.lead - (first ? 0 : 128)) * 8 : 4096;  // register byte 0 (UPD)
  m.reg = cur.len < 4 ? 0u : cur.state;
  m.B8 = first || spill ? (cur.len < 4 ? m.A8 : ((int32_t)cur.lead + 4 - (first ? 0 : 128)) * 8) : m.A8;
  m.need = (li < 2 || li >= (int32_t)cur.nlines - 1) ? 1u : 0u;
  return m;
}
template <bool UPD, int O>
__device__ __forceinline__ void apply_half_mask(uint4 (&v)[8], const HalfMask& m, uint32_t h) {
  const int32_t base8 = (int32_t)h * 512;  // bit offset of the half in its line
#pragma unroll
  for (int i = 0; i < 4; i++) {
    uint32_t* w = reinterpret_cast<uint32_t*>(&v[O + i]);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int32_t p8 = base8 + (i * 16 + q * 4) * 8;
      const uint32_t keepA = (uint32_t)(0xFFFFFFFFull << clamp032(m.A8 - p8));
      const uint32_t keepH = (uint32_t)(0xFFFFFFFFull >> clamp032(p8 + 32 - m.H8));
      if constexpr (UPD) {
        const int32_t x = m.S8 - p8;
        const uint32_t sw = x >= 32 || x <= -32 ? 0u : (x >= 0 ? m.reg << x : m.reg >> -x);
        w[q] = (keepA & keepH & w[q]) ^ sw;
      } else {
        const uint32_t keepB = (uint32_t)(0xFFFFFFFFull << clamp032(m.B8 - p8));
        w[q] = keepA & keepH & (w[q] ^ ~keepB);
      }
    }
  }
}
template <bool UPD, int O>
__device__ __forceinline__ void mask_half(uint4 (&v)[8], int32_t li, const VarTask& cur, uint32_t h) {
  apply_half_mask<UPD, O>(v, half_mask<UPD>(li, cur), h);
}
[[maybe_unused]] __device__ __forceinline__ int32_t lane_xor8(int32_t x) { return __builtin_amdgcn_mov_dpp(x, 0x128, 0xF, 0xF, false); }

// The G = 32 and G = 16 length classes with coalesced nontemporal loads (crc32_fixed32_nt_kernel's access
// shape on the sorted descriptors). A wave holds NG = 64 / G lane groups, each stepping through its own
// (payload, round) sequence exactly like var_class<G>; per step a group's round is G consecutive absolute lines,
// read as 1 KiB pieces: load i covers piece 2 (i >> 2) + (i & 1) of group (i >> 1) & 1 (G = 32) or piece i >> 2
// of group i & 3 (G = 16), with the groups' line bases broadcast from their first lanes. A lane's line index is
// clamped to its payload's lines (virtual lines of the first round re-read the first line and are masked to
// zero; a group without a task reads one line of the buffer). After transpose_blocks lane l holds half l3 of
// lines jA and jA + G/2 of its group's round (jA = 8 l4 + (l & 7) for G = 32, l & 7 for G = 16); both halves
// are masked where they hold a payload edge, the round register enters the first halves, and the half join
// leaves lane l the register of line jl = jA + (G/2) l3 (nibble-table half join: the var image has no byte
// tables). STAGE as var_class (1: the whole image, also for a block without work; 0: the group part only).
template <int G, bool UPD, int STAGE>
__device__ __forceinline__ void var_class_nt(uint4* lds4, const uint8_t* __restrict__ base,
                                             const uint4* __restrict__ desc, const uint32_t* __restrict__ range,
                                             const uint4* __restrict__ img_slice, const uint4* __restrict__ img_group,
                                             const uint4* __restrict__ img_unshift, uint32_t* __restrict__ out) {
  static_assert(G == 16 || G == 32, "two or four lane groups per wave");
  constexpr int NG = 64 / G;
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  const uint32_t l = threadIdx.x & 63, l3 = (l >> 3) & 1, l4 = (l >> 4) & 1;
  const size_t gid = group_id<kBlock, G, kVwg>();
  const size_t ngroups = ((size_t)gridDim.x * kBlock) / G;
  const size_t t_begin = range[0], t_end = range[1];
  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  const uint32_t jA = (G == 32 ? 8 * l4 : 0u) + (l & 7);  // line of v[0..3]; v[4..7] holds line jA + G/2
  const uint32_t jl = jA + (G / 2) * l3;
  k.slot4 = jl << 2;
  const uint32_t chunk = 16u * (4u * l3 + 2u * ((l >> 5) & 1u) + l4);  // coalesced_lane_offset without the line
  const uint64_t b0 = (uint64_t)(uintptr_t)base;
  const uint64_t safe_line = b0 >> 7;

  auto raw = [&](size_t t) { return raw_task<true>(t, t_end, base, desc, 0, 0); };
  auto load = [&](const VarTask& tk, uint32_t r, uint4 (&v)[8]) {
    const int32_t rel0 = (int32_t)(r * G) - (int32_t)tk.vlead;
    const int32_t rmax = tk.valid ? (int32_t)tk.nlines - 1 : 0;
    const uint64_t ln0 = tk.valid ? tk.line0 : safe_line;
    const uint32_t lo = (uint32_t)ln0, hi = (uint32_t)(ln0 >> 32);
    int32_t rel_g[NG], max_g[NG];
    uint64_t ln_g[NG];
#pragma unroll
    for (int g = 0; g < NG; g++) {
      rel_g[g] = __builtin_amdgcn_readlane(rel0, g * G);
      max_g[g] = __builtin_amdgcn_readlane(rmax, g * G);
      ln_g[g] = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, g * G) << 32) |
                (uint32_t)__builtin_amdgcn_readlane((int)lo, g * G);
    }
    // branch-free (a scalar branch between two load sequences made the compiler drain the loads at the merge:
    // 284 us against 222 per config-3 call): per group a scalar base at its payload's first line, per lane a
    // 32-bit offset of its clamped line
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int g = G == 32 ? (i >> 1) & 1 : i & 3;
      const int piece = G == 32 ? 2 * (i >> 2) + (i & 1) : i >> 2;
      const int32_t rel = min(max(rel_g[g] + 8 * piece + (int32_t)(l & 7), 0), max_g[g]);
      const uint8_t* gb = base + ((ln_g[g] << 7) - b0);
      const v4u32 x = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(gb + ((uint32_t)rel * 128u + chunk)));
      v[i] = make_uint4(x.x, x.y, x.z, x.w);
    }
  };

  size_t t0 = t_begin + gid;
  if (!__syncthreads_or(t0 < t_end)) {  // the block has no task of this class
    if constexpr (STAGE == 1) {  // (the next classes stage only their group part)
      load_image<kLdsVarImageBytes>(lds4, img_slice, img_group, img_unshift);
      __syncthreads();
    }
    return;
  }
  VarTask dec0 = decode_task<G>(raw(t0), t0 < t_end);
  if constexpr (UPD) dec0.state = dec0.valid ? out[dec0.p] : 0u;
  uint32_t r0 = 0;
  size_t t1 = dec0.rounds > 1 ? t0 : t0 + ngroups;
  uint32_t r1 = dec0.rounds > 1 ? 1u : 0u;
  uint4 d1 = raw(t1);

  uint4 A[8], B[8];
  load(dec0, r0, A);
  if constexpr (STAGE == 0)
    load_image<kLdsImageBytes, kBlock, kLdsImageBytes, kLdsCommonBytes>(lds4, img_slice, img_group);
  else
    load_image<kLdsVarImageBytes>(lds4, img_slice, img_group, img_unshift);
  __syncthreads();

  uint32_t s = 0;
  auto compute = [&](uint4 (&v)[8], const VarTask& cur, uint32_t r_c) {
    transpose_blocks(v);
    const int32_t liA = (int32_t)(r_c * G + jA) - (int32_t)cur.vlead;
    const int32_t liB = liA + G / 2;
    const int32_t last = (int32_t)cur.nlines - 1;
    // virtual lines of a first round: zeroed by selects (cheap); the payload's first, spill and last lines:
    // the byte masks, on the one half-branch that holds them (a first round with both halves' general masks
    // cost twice the VALU of the whole fold)
    if (liA < 0 || liB < 0) {
#pragma unroll
      for (int i = 0; i < 4; i++) {
        v[i] = liA < 0 ? make_uint4(0u, 0u, 0u, 0u) : v[i];
        v[4 + i] = liB < 0 ? make_uint4(0u, 0u, 0u, 0u) : v[4 + i];
      }
    }
    const bool spill = cur.lead > 124 && cur.len >= 4;
    if (liA == 0 || (liA == 1 && spill) || liA == last) mask_half<UPD, 0>(v, liA, cur, l3);
    if (liB == 0 || (liB == 1 && spill) || liB == last) mask_half<UPD, 4>(v, liB, cur, l3);
    // the round register (shift_{(G-1)*128} of the lane's register, 0 at a payload's first round) enters the
    // first half of its line: lanes with l3 = 0 fold the first halves of their own line and of lane ^ 8's
    const uint32_t sin = nibble_map_uniform(s, lds, kLdsRoundOff);
    const uint32_t sp = (uint32_t)__builtin_amdgcn_mov_dpp((int)sin, 0x128, 0xF, 0xF, false);  // lane ^ 8's
    v[0].x ^= l3 ? 0u : sin;
    v[4].x ^= l3 ? 0u : sp;
    {
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
      s = nibble_map_uniform(first, lds, kLdsHalfOff) ^ second;  // shift_64
    }
    if (r_c == cur.rounds - 1) {
      uint32_t t = group_xor_reduce<G>(nibble_map_lane(s, lds, k.slot4));
      if (cur.valid && (l & (G - 1)) == G - 1) {
        const uint32_t over = 128 - cur.tailend;  // trailing zero bytes of the last line
        if (over) {
          t = nibble_map_uniform(t, lds, kLdsUnshiftOff + (over & 15u) * 512);
          t = nibble_map_uniform(t, lds, kLdsUnshiftOff + 8192 + (over >> 4) * 512);
        }
        if constexpr (UPD) {
          if (cur.len < 4) t ^= shift_bits(cur.state, 8u * cur.len);
          out[cur.p] = t;
        } else {
          if (cur.len < 4) {
            constexpr uint32_t k1 = shift_bits(kInit, 8), k2 = shift_bits(kInit, 16), k3 = shift_bits(kInit, 24);
            t ^= cur.len == 1 ? k1 : (cur.len == 2 ? k2 : k3);
          }
          out[cur.p] = ~t;
        }
      }
      s = 0;
    }
  };

  auto step = [&](uint4 (&cur_buf)[8], uint4 (&nxt_buf)[8]) {
    // every group of the wave still in its task (r1 > 0): its descriptor is decoded already (no load in the
    // branch, so the loads in flight are not drained at the merge; update mode decodes every step, since it
    // loads the register there)
    VarTask dec1 = dec0;
    if (UPD || __builtin_amdgcn_ballot_w64(r1 == 0) != 0) {
      dec1 = decode_task<G>(d1, t1 < t_end);
      if constexpr (UPD) dec1.state = dec1.valid ? out[dec1.p] : 0u;
    }
    const bool more = r1 + 1 < dec1.rounds;
    const size_t t2 = more ? t1 : t1 + ngroups;
    const uint32_t r2 = more ? r1 + 1 : 0u;
    const uint4 d2 = raw(t2);
    ANNETY_PRIO_HI();
    load(dec1, r1, nxt_buf);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    compute(cur_buf, dec0, r0);
    dec0 = dec1;
    r0 = r1;
    t1 = t2;
    r1 = r2;
    d1 = d2;
  };

  // wave-uniform loop: the loads and the cross-lane steps need every group (a finished group reads one
  // line of the buffer and stores nothing)
  while (__builtin_amdgcn_ballot_w64(dec0.valid) != 0) {
    step(A, B);
    step(B, A);
  }
}

// The small class (< 24 lines) with coalesced nontemporal loads, at G = 8: a wave's eight lane groups (lanes
// 8m..8m+7) each step through their own (payload, round) sequence, a round being 8 consecutive absolute lines =
// 1 KiB = exactly one load. Load i reads the round of lane group m(i) = (i >> 2) + 2 (i & 1) + 4 ((i >> 1) & 1)
// (its line base broadcast from lane 8 m(i)), so that after transpose_blocks and the half join lane l holds
// line l & 7 of its own group's round (crc32_onekib_nt_kernel's layout). Before the join a lane holds half l3 of
// line l & 7 of two groups: its own and lane ^ 8's; the masks of the partner's line come over DPP.
template <bool UPD>
__device__ __forceinline__ void var_class_nt8(uint4* lds4, const uint8_t* __restrict__ base,
                                              const uint4* __restrict__ desc, const uint32_t* __restrict__ range,
                                              const uint4* __restrict__ img_slice, const uint4* __restrict__ img_group,
                                              uint32_t* __restrict__ out) {
  constexpr int G = 8;
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  const uint32_t l = threadIdx.x & 63, l3 = (l >> 3) & 1, j = l & 7;
  const size_t gid = group_id<kBlock, G, kVwg>();
  const size_t ngroups = ((size_t)gridDim.x * kBlock) / G;
  const size_t t_begin = range[0], t_end = range[1];
  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;  // join slot: j = slot & 7
  const uint32_t lane_off = coalesced_lane_offset(l);
  const uint64_t b0 = (uint64_t)(uintptr_t)base;
  const uint64_t safe_line = b0 >> 7;

  auto raw = [&](size_t t) { return raw_task<true>(t, t_end, base, desc, 0, 0); };
  auto load = [&](const VarTask& tk, uint32_t r, uint4 (&v)[8]) {
    const int32_t rel0 = (int32_t)(r * G) - (int32_t)tk.vlead;
    const int32_t rmax = tk.valid ? (int32_t)tk.nlines - 1 : 0;
    const uint64_t ln0 = tk.valid ? tk.line0 : safe_line;
    const uint32_t lo = (uint32_t)ln0, hi = (uint32_t)(ln0 >> 32);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int src = 8 * ((i >> 2) + 2 * (i & 1) + 4 * ((i >> 1) & 1));
      const int32_t rel_g = __builtin_amdgcn_readlane(rel0, src), max_g = __builtin_amdgcn_readlane(rmax, src);
      const uint64_t ln_g = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, src) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)lo, src);
      const int32_t rel = min(max(rel_g + (int32_t)j, 0), max_g);
      const uint64_t off = ((ln_g + (uint64_t)rel) << 7) + (lane_off & 127u) - b0;
      const v4u32 x = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(base + off));
      v[i] = make_uint4(x.x, x.y, x.z, x.w);
    }
  };

  size_t t0 = t_begin + gid;
  if (!__syncthreads_or(t0 < t_end)) return;
  VarTask dec0 = decode_task<G>(raw(t0), t0 < t_end);
  if constexpr (UPD) dec0.state = dec0.valid ? out[dec0.p] : 0u;
  uint32_t r0 = 0;
  size_t t1 = dec0.rounds > 1 ? t0 : t0 + ngroups;
  uint32_t r1 = dec0.rounds > 1 ? 1u : 0u;
  uint4 d1 = raw(t1);

  uint4 A[8], B[8];
  load(dec0, r0, A);
  load_image<kLdsImageBytes, kBlock, kLdsImageBytes, kLdsCommonBytes>(lds4, img_slice, img_group);
  __syncthreads();

  uint32_t s = 0;
  auto compute = [&](uint4 (&v)[8], const VarTask& cur, uint32_t r_c) {
    transpose_blocks(v);
    const int32_t li = (int32_t)(r_c * G + j) - (int32_t)cur.vlead;
    const HalfMask mo = half_mask<UPD>(li, cur);
    HalfMask mp;  // lane ^ 8's line (same position j in the partner group)
    mp.A8 = lane_xor8(mo.A8);
    mp.H8 = lane_xor8(mo.H8);
    if constexpr (UPD) {
      mp.S8 = lane_xor8(mo.S8);
      mp.reg = (uint32_t)lane_xor8((int32_t)mo.reg);
    } else {
      mp.B8 = lane_xor8(mo.B8);
    }
    mp.need = (uint32_t)lane_xor8((int32_t)mo.need);
    // v[0..3]: half l3 of the line of lane l & ~8's group, v[4..7]: of lane l | 8's
    if (l3 ? mp.need : mo.need) apply_half_mask<UPD, 0>(v, l3 ? mp : mo, l3);
    if (l3 ? mo.need : mp.need) apply_half_mask<UPD, 4>(v, l3 ? mo : mp, l3);
    const uint32_t sin = nibble_map_uniform(s, lds, kLdsRoundOff);  // shift_{7*128}; 0 at a first round
    const uint32_t sp = (uint32_t)lane_xor8((int32_t)sin);
    v[0].x ^= l3 ? 0u : sin;
    v[4].x ^= l3 ? 0u : sp;
    {
      uint32_t xa = v[0].x, xb = v[4].x;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        word4x2(xa, v[i].y, xb, v[4 + i].y, k);
        word4x2(xa, v[i].z, xb, v[4 + i].z, k);
        word4x2(xa, v[i].w, xb, v[4 + i].w, k);
        word4x2(xa, i + 1 < 4 ? v[i + 1].x : 0u, xb, i + 1 < 4 ? v[5 + i].x : 0u, k);
      }
      const uint32_t send = l3 ? xa : xb;
      const uint32_t got = (uint32_t)lane_xor8((int32_t)send);
      const uint32_t first = l3 ? got : xa, second = l3 ? xb : got;
      s = nibble_map_uniform(first, lds, kLdsHalfOff) ^ second;  // shift_64
    }
    if (r_c == cur.rounds - 1) {
      uint32_t t = group_xor_reduce<G>(nibble_map_lane(s, lds, k.slot4));
      if (cur.valid && j == G - 1) {
        const uint32_t over = 128 - cur.tailend;
        if (over) {
          t = nibble_map_uniform(t, lds, kLdsUnshiftOff + (over & 15u) * 512);
          t = nibble_map_uniform(t, lds, kLdsUnshiftOff + 8192 + (over >> 4) * 512);
        }
        if constexpr (UPD) {
          if (cur.len < 4) t ^= shift_bits(cur.state, 8u * cur.len);
          out[cur.p] = t;
        } else {
          if (cur.len < 4) {
            constexpr uint32_t k1 = shift_bits(kInit, 8), k2 = shift_bits(kInit, 16), k3 = shift_bits(kInit, 24);
            t ^= cur.len == 1 ? k1 : (cur.len == 2 ? k2 : k3);
          }
          out[cur.p] = ~t;
        }
      }
      s = 0;
    }
  };

  auto step = [&](uint4 (&cur_buf)[8], uint4 (&nxt_buf)[8]) {
    VarTask dec1 = decode_task<G>(d1, t1 < t_end);
    if constexpr (UPD) dec1.state = dec1.valid ? out[dec1.p] : 0u;
    const bool more = r1 + 1 < dec1.rounds;
    const size_t t2 = more ? t1 : t1 + ngroups;
    const uint32_t r2 = more ? r1 + 1 : 0u;
    const uint4 d2 = raw(t2);
    ANNETY_PRIO_HI();
    load(dec1, r1, nxt_buf);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    compute(cur_buf, dec0, r0);
    dec0 = dec1;
    r0 = r1;
    t1 = t2;
    r1 = r2;
    d1 = d2;
  };
  while (__builtin_amdgcn_ballot_w64(dec0.valid) != 0) {
    step(A, B);
    step(B, A);
  }
}

template <int G, bool SORTED, bool UPD = false, int VWG = kVwg, int PROBE = 0>
__global__ __launch_bounds__(kBlock) void crc32_var_kernel(const uint8_t* __restrict__ base, size_t n,
                                                           uint64_t fstride, uint32_t flen,
                                                           const uint4* __restrict__ desc,
                                                           const uint32_t* __restrict__ range,
                                                           const uint4* __restrict__ img_slice,
                                                           const uint4* __restrict__ img_group,
                                                           const uint4* __restrict__ img_unshift,
                                                           uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsVarImageBytes / 16];
  var_class<G, SORTED, UPD, VWG, PROBE, 2>(lds4, base, n, fstride, flen, desc, range, img_slice, img_group,
                                           img_unshift, out);
}

// The sorted path's three length classes in one launch (ranges[0..5] = the classes' [begin, end) in desc,
// longest first): each block runs its share of the G = 32 class, then of the G = 16 class (restaging only
// the group part of the image), then of the G = 4 class. A block that finishes a class early starts the
// next one instead of waiting for the class's slowest lane groups (three launches drained each class:
// a 64 KiB-payload launch loses ~24 us to its tail), and two launch gaps go.
//   NT (bits, ANNETY_CRC_SORTED_NT, default 3): 1 = the G = 32 class with coalesced nontemporal loads
//   (var_class_nt), 2 = the G = 16 class too, 4 = the small class at G = 8 (var_class_nt8); unset classes load
//   per line (small: G = 4). Config 3, one class alone (profiles/r04/sorted_nt/classes.log): G = 32 150.4 us
//   coalesced / 182.6 per line, G = 16 68.6 / 63.8, small 53.2 (G = 8) / 40.9 (G = 4); fused, masks 1 and 3 the
//   same, 7 slower.
template <bool UPD, int NT>
__global__ __launch_bounds__(kBlock) void crc32_var_sorted_kernel(const uint8_t* __restrict__ base, size_t n,
                                                                  const uint4* __restrict__ desc,
                                                                  const uint32_t* __restrict__ ranges,
                                                                  const uint4* __restrict__ img_slice,
                                                                  const uint4* __restrict__ img_g32,
                                                                  const uint4* __restrict__ img_g16,
                                                                  const uint4* __restrict__ img_g4,
                                                                  const uint4* __restrict__ img_g8,
                                                                  const uint4* __restrict__ img_unshift,
                                                                  uint32_t* __restrict__ out, uint32_t classes) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsVarImageBytes / 16];
  // classes: bit c runs class c (the product runs all three; the microbench timing of one class alone leaves
  // digests of the others unwritten, ANNETY_CRC_SORTED_CLASSES); bit 3: the small class per line at G = 8, not 4;
  // bit 4: odd blocks run the classes in reverse order (small, G = 16, G = 32), so that the small class's
  // latency-bound steps overlap other blocks' streaming instead of all blocks' tails
  if ((classes & 16) && (blockIdx.x & 1)) {
    if (classes & 4)
      var_class<4, true, UPD, kVwg, 0, 1>(lds4, base, n, 0, 0, desc, ranges + 4, img_slice, img_g4, img_unshift, out);
    else
      load_image<kLdsVarImageBytes>(lds4, img_slice, img_g4, img_unshift);
    __syncthreads();
    if (classes & 2) {
      if constexpr (NT & 2)
        var_class_nt<16, UPD, 0>(lds4, base, desc, ranges + 2, img_slice, img_g16, img_unshift, out);
      else
        var_class<16, true, UPD, kVwg, 0, 0>(lds4, base, n, 0, 0, desc, ranges + 2, img_slice, img_g16, img_unshift, out);
    }
    __syncthreads();
    if (classes & 1) {
      if constexpr (NT & 1)
        var_class_nt<32, UPD, 0>(lds4, base, desc, ranges, img_slice, img_g32, img_unshift, out);
      else
        var_class<32, true, UPD, kVwg, 0, 0>(lds4, base, n, 0, 0, desc, ranges, img_slice, img_g32, img_unshift, out);
    }
    return;
  }
  if (classes & 1) {
    if constexpr (NT & 1)
      var_class_nt<32, UPD, 1>(lds4, base, desc, ranges, img_slice, img_g32, img_unshift, out);
    else
      var_class<32, true, UPD, kVwg, 0, 1>(lds4, base, n, 0, 0, desc, ranges, img_slice, img_g32, img_unshift, out);
  } else {
    load_image<kLdsVarImageBytes>(lds4, img_slice, img_g32, img_unshift);
  }
  __syncthreads();  // every wave is done with the G = 32 group tables
  if (classes & 2) {
    if constexpr (NT & 2)
      var_class_nt<16, UPD, 0>(lds4, base, desc, ranges + 2, img_slice, img_g16, img_unshift, out);
    else
      var_class<16, true, UPD, kVwg, 0, 0>(lds4, base, n, 0, 0, desc, ranges + 2, img_slice, img_g16, img_unshift, out);
  }
  __syncthreads();
  if (!(classes & 4)) return;
  if constexpr (NT & 4)
    var_class_nt8<UPD>(lds4, base, desc, ranges + 4, img_slice, img_g8, out);
  else if (classes & 8)  // (A/B: the small class per line at G = 8)
    var_class<8, true, UPD, kVwg, 0, 0>(lds4, base, n, 0, 0, desc, ranges + 4, img_slice, img_g8, img_unshift, out);
  else
    var_class<4, true, UPD, kVwg, 0, 0>(lds4, base, n, 0, 0, desc, ranges + 4, img_slice, img_g4, img_unshift, out);
}

// ---- long payloads: segments + CRC combine ----
// A batch of few long payloads cannot fill 256 CUs with at most 32 lanes per payload, and a batch
// whose payload count is not a multiple of the lane-groups leaves a tail. Such payloads are cut into
// segments aligned to their END (segment k of S ends at len - (S-1-k)*seg; segment 0 takes the
// remainder), every segment is a task of the variable-length kernel, and the digests are joined with
// the combine identity crc(A||B) = shift_|B|(crc A) ^ crc B folded over the segments:
//   crc = XOR_k shift_{(S-1-k)*seg}(crc_k),
// where every shift is a multiple of seg, so one table of powers serves the whole batch.
__global__ __launch_bounds__(256) void crc32_split_desc(const uint8_t* __restrict__ base, size_t n, uint64_t len,
                                                        uint64_t stride, uint64_t seg, uint32_t S,
                                                        uint4* __restrict__ desc, uint32_t* __restrict__ range) {
  const size_t total = n * (size_t)S;
  for (size_t t = blockIdx.x * (size_t)256 + threadIdx.x; t < total; t += (size_t)gridDim.x * 256) {
    const size_t i = t / S;
    const uint32_t k = (uint32_t)(t - i * S);
    const uint64_t end = len - (uint64_t)(S - 1 - k) * seg;
    const uint64_t beg = k ? end - seg : 0;
    const uint64_t a = (uint64_t)(uintptr_t)(base + i * stride + beg);
    desc[t] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)(end - beg), (uint32_t)t);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    range[0] = 0;
    range[1] = (uint32_t)total;
  }
}

// One wave per (payload, chunk of 64 segments); lane k applies shift_{(S-1-k)*seg} (32x32 GF(2)
// matrix, powers[(m-1)*32 + bit]) to segment k's digest, the wave XOR-reduces, and a payload spread
// over several chunks is accumulated with atomicXor (out pre-zeroed; XOR is order-independent, so the
// result is deterministic). Every shift is absolute, so the chunks need no further join.
__global__ __launch_bounds__(256) void crc32_split_join(const uint32_t* __restrict__ seg_crc, size_t n, uint32_t S,
                                                        const uint32_t* __restrict__ powers,
                                                        uint32_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t chunks = (S + 63) / 64;
  const size_t units = n * (size_t)chunks;
  for (size_t u = blockIdx.x * (size_t)4 + (threadIdx.x >> 6); u < units; u += (size_t)gridDim.x * 4) {
    const size_t i = u / chunks;
    const uint32_t k = (uint32_t)(u - i * chunks) * 64 + lane;
    uint32_t acc = 0;
    if (k < S) {
      const uint32_t c = seg_crc[i * S + k];
      const uint32_t m = S - 1 - k;
      if (m == 0) {
        acc = c;
      } else {
        const uint32_t* P = powers + (size_t)(m - 1) * 32;
#pragma unroll
        for (int b = 0; b < 32; b++) acc ^= P[b] & (0u - ((c >> b) & 1u));
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc ^= __shfl_xor(acc, o, 64);
    if (lane == 0) {
      if (chunks == 1)
        out[i] = acc;
      else
        atomicXor(out + i, acc);
    }
  }
}

template <int G>
hipError_t launch_var_g(const VarLaunch& a, hipStream_t stream) {
  size_t blocks = a.max_blocks;
  if (!a.range) {  // unsorted direct mode: size the grid to the batch
    const size_t lanes = a.n * (size_t)G;
    blocks = std::min(blocks, (lanes + kBlock - 1) / kBlock);
  }
  if (blocks == 0) return hipSuccess;
  note_kernel(G == 1 ? "crc32_var_kernel<1>" : G == 2 ? "crc32_var_kernel<2>" : G == 4 ? "crc32_var_kernel<4>" :
              G == 8 ? "crc32_var_kernel<8>" : G == 16 ? "crc32_var_kernel<16>" : "crc32_var_kernel<32>");
#define ANNETY_VAR_LAUNCH(SORTED, UPD)                                                                     \
  hipLaunchKernelGGL((crc32_var_kernel<G, SORTED, UPD>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,   \
                     static_cast<const uint8_t*>(a.base), a.n, a.fixed_stride, a.fixed_len,                  \
                     static_cast<const uint4*>(a.desc), a.range, static_cast<const uint4*>(a.img_slice),     \
                     static_cast<const uint4*>(a.img_group), static_cast<const uint4*>(a.img_unshift),       \
                     a.out)
  if (a.desc) {
    if (a.update) ANNETY_VAR_LAUNCH(true, true);
    else ANNETY_VAR_LAUNCH(true, false);
  } else {
    if (a.update) ANNETY_VAR_LAUNCH(false, true);
    else ANNETY_VAR_LAUNCH(false, false);
  }
#undef ANNETY_VAR_LAUNCH
  return hipGetLastError();
}

template <int G, bool FULL, bool RAW>
hipError_t launch_g(const FixedLaunch& a, hipStream_t stream) {
  const size_t lanes = a.n * (size_t)G;
  size_t blocks = (lanes + kBlock - 1) / kBlock;
  if (blocks > a.max_blocks) blocks = a.max_blocks;
  if (blocks == 0) return hipSuccess;
  note_kernel(G == 1 ? "crc32_fixed_kernel<1>" : G == 2 ? "crc32_fixed_kernel<2>" : G == 4 ? "crc32_fixed_kernel<4>" :
              G == 8 ? "crc32_fixed_kernel<8>" : G == 16 ? "crc32_fixed_kernel<16>" : "crc32_fixed_kernel<32>");
  hipLaunchKernelGGL((crc32_fixed_kernel<G, FULL, RAW>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                     static_cast<const uint8_t*>(a.base), a.n, a.stride, a.rounds, a.vlead,
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
  note_kernel(G == 1 ? "crc32_oneround_kernel<1>" : G == 2 ? "crc32_oneround_kernel<2>" :
              G == 4 ? "crc32_oneround_kernel<4>" : G == 8 ? "crc32_oneround_kernel<8>" :
              G == 16 ? "crc32_oneround_kernel<16>" : "crc32_oneround_kernel<32>");
  hipLaunchKernelGGL((crc32_oneround_kernel<G>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                     static_cast<const uint8_t*>(a.base), a.n, a.stride, static_cast<const uint4*>(a.img_slice),
                     static_cast<const uint4*>(a.img_group), a.out);
  return hipGetLastError();
}

// A/B builds only (ANNETY_CRC_FIXED_NT=0): contiguous 1 KiB batches on crc32_oneround_kernel<8> and G = 32
// batches on crc32_fixed_kernel<32>. Read once.
bool onekib_nt_enabled() {
  static const bool on = ANNETY_AB_KNOB("ANNETY_CRC_FIXED_NT", 1) != 0;
  return on;
}

hipError_t launch_one(const FixedLaunch& a, hipStream_t stream) {
  if (a.group == 8 && a.stride == 1024 && a.n % 8 == 0 && onekib_nt_enabled()) {
    size_t blocks = (a.n * 8 + kBlock - 1) / kBlock;
    if (blocks > a.max_blocks) blocks = a.max_blocks;
    if (blocks == 0) return hipSuccess;
    note_kernel("crc32_onekib_nt_kernel");
    hipLaunchKernelGGL((crc32_onekib_nt_kernel<>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                       static_cast<const uint8_t*>(a.base), a.n, static_cast<const uint4*>(a.img_slice),
                       static_cast<const uint4*>(a.img_group), static_cast<const uint4*>(a.img_bytemap), a.out);
    return hipGetLastError();
  }
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
  if (!a.raw && a.full && a.group == 32 && a.n % 2 == 0 && a.stride % 16 == 0 && onekib_nt_enabled()) {
    size_t blocks = (a.n * 32 + kBlock - 1) / kBlock;
    if (blocks > a.max_blocks) blocks = a.max_blocks;
    if (blocks == 0) return hipSuccess;
    note_kernel("crc32_fixed32_nt_kernel");
    hipLaunchKernelGGL((crc32_fixed32_nt_kernel<>), dim3((unsigned)blocks), dim3(kBlock), 0, stream,
                       static_cast<const uint8_t*>(a.base), a.n, a.stride, a.rounds,
                       static_cast<const uint4*>(a.img_slice), static_cast<const uint4*>(a.img_group),
                       static_cast<const uint4*>(a.img_bytemap), a.out);
    return hipGetLastError();
  }
  if (!a.raw && a.full && a.rounds == 1) return launch_one(a, stream);
  if (a.raw) return a.full ? launch_full<true, true>(a, stream) : launch_full<false, true>(a, stream);
  return a.full ? launch_full<true, false>(a, stream) : launch_full<false, false>(a, stream);
}

// the three classes, odd blocks in reverse order (A/B against 7: profiles/r04/sorted_nt/ab_class_order.log)
constexpr uint32_t kSortedClassesDefault = 23;
constexpr int kSortedNtDefault = 3;  // crc32_var_sorted_kernel NT: G = 32 and G = 16 coalesced (A/B against 1: profiles/r04/sorted_nt/ab_nt1_nt3.log)

hipError_t launch_var_sorted(const VarLaunch& a, const void* img_g32, const void* img_g16, const void* img_g4,
                             const void* img_g8, hipStream_t stream) {
  const unsigned blocks = (unsigned)std::max<size_t>(1, a.max_blocks);
  note_kernel("crc32_var_sorted_kernel");
#define ANNETY_SORTED_LAUNCH(UPD, NT)                                                                         \
  hipLaunchKernelGGL((crc32_var_sorted_kernel<UPD, NT>), dim3(blocks), dim3(kBlock), 0, stream,              \
                     static_cast<const uint8_t*>(a.base), a.n, static_cast<const uint4*>(a.desc), a.range,      \
                     static_cast<const uint4*>(a.img_slice), static_cast<const uint4*>(img_g32),               \
                     static_cast<const uint4*>(img_g16), static_cast<const uint4*>(img_g4),                    \
                     static_cast<const uint4*>(img_g8),                                                         \
                     static_cast<const uint4*>(a.img_unshift), a.out, classes)
  constexpr uint32_t classes = kSortedClassesDefault;
  if (a.update) ANNETY_SORTED_LAUNCH(true, kSortedNtDefault);
  else ANNETY_SORTED_LAUNCH(false, kSortedNtDefault);
#undef ANNETY_SORTED_LAUNCH
  return hipGetLastError();
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

hipError_t launch_split_desc(const void* base, size_t n, uint64_t len, uint64_t stride, uint64_t seg, uint32_t S,
                             void* desc, uint32_t* range, hipStream_t stream) {
  const size_t total = n * (size_t)S;
  const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>(2048, (total + 255) / 256));
  note_kernel("crc32_split_desc");
  hipLaunchKernelGGL(crc32_split_desc, dim3(blocks), dim3(256), 0, stream, static_cast<const uint8_t*>(base), n, len,
                     stride, seg, S, static_cast<uint4*>(desc), range);
  return hipGetLastError();
}

hipError_t launch_split_join(const uint32_t* seg_crc, size_t n, uint32_t S, const uint32_t* powers, uint32_t* out,
                             hipStream_t stream) {
  const size_t units = n * (size_t)((S + 63) / 64);
  if (units > n) {
    const hipError_t e = hipMemsetAsync(out, 0, n * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
  }
  const unsigned blocks = (unsigned)std::max<size_t>(1, std::min<size_t>(8192, (units + 3) / 4));
  note_kernel("crc32_split_join");
  hipLaunchKernelGGL(crc32_split_join, dim3(blocks), dim3(256), 0, stream, seg_crc, n, S, powers, out);
  return hipGetLastError();
}

int fixed_kernel_block() { return kBlock; }

}  // namespace annety_crc
