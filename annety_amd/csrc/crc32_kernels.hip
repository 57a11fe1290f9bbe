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
// by rounds of 8 lines (crc32_bucket_place, crc32_arena.hip), so the payloads of a wave finish together. Zero-length payloads never reach this kernel (the bucket pass writes 0).
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
//        task (a kernel of its own); 1 = all of it always; 0 = only the G-specific group part; 3 = the group part
//        and the inverse-shift tables (the later classes of crc32_var_sorted_kernel, whose first class staged
//        the common part).
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
  else if constexpr (STAGE == 3)
    load_image<kLdsVarImageBytes, kBlock, kLdsImageBytes, kLdsCommonBytes>(lds4, img_slice, img_group, img_unshift);
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

// ---------------------------------------------------------------------------------------------
// The length-sorted path (round 5): lane groups of G = 8 on coalesced nontemporal 1 KiB loads,
// with the steady-state round of crc32_onekib_nt_kernel and no per-lane masks or address arithmetic in it.
//
// A payload of nl lines (absolute 128-byte lines L0..L1) is cut into R = (nl - h) / 8 + 1 rounds:
//   round 0 ("head"): the first h = ((nl - 1) mod 8) + 1 lines, end-aligned: lane j reads line j - (8 - h), the
//            lanes before line 0 re-read line 0 and are zeroed, the bytes before the payload start are masked,
//            and the init (or the caller's register) enters as the register shift_{128-lead}(init) of line 0
//            (a payload of <= 8 lines, R = 1, ends in this round);
//   rounds 1 .. R-1 ("body"): the 1 KiB pieces [h + 8 (r - 1), h + 8 r): whole lines, except that the last
//            round's line 7 is the payload's last line (bytes after the payload end masked, removed after the
//            join by the inverse shift of the line's overhang).
// A group's rounds are read from one scalar base per round (the group's round address broadcast from its first
// lane), so a body round costs the loads, the transpose, the round register and the fold, as in config 1.
// The wave's 8 groups take 8 consecutive tasks of the length-sorted list (equal line counts in the same
// bucket), so they start and finish together: every step in which no group is in its head or last round (or
// idle) takes the unmasked branch, wave-uniformly; the rest (about 2 per 8 payloads, 15 % of config 3's steps)
// take the masked one.
// Scheduling: a wave takes SETS of 8 consecutive tasks, one per group, and moves to its next set when all 8 are
// done (equal lengths inside a bucket: the lockstep idles 0.02 % of config 3's group rounds). Blocks own the sets in
// snake order over the sorted list, and a block's waves take its sets longest first, each to the wave that frees up
// first (an LDS counter, claimed 3 steps before the switch): the busiest wave of config 3 holds 67 rounds against a
// mean of 65.3. Static round-robin over the sorted list gave every long set of each row to the same few waves (103
// rounds: 0.63 of the ideal; snake order over waves 74), and a chip-wide counter in HBM cost more than it saved
// (its atomics serialise: DESIGN.md §2.5).
struct W8Task {
  uint64_t a0;  // address of the payload's first line (128-aligned)
  uint32_t lead, te, h, R, p, state;
  // 0: a payload; else a split payload's segment (crc32_kernels.h kSplitSeg): bit 0 its first, bit 1 a later one,
  // bit 2 big segments, bits 16-31 m = the segments after it (p = the payload's index either way)
  uint32_t seg;
  bool valid;
};
__device__ __forceinline__ W8Task decode_w8(uint4 d, bool valid) {
  W8Task k;
  const uint64_t a = ((uint64_t)(d.y & 0xFFFFu) << 32) | d.x;  // (48-bit addresses; a segment's m above them)
  const uint64_t e = a + d.z;  // d.z > 0
  const uint64_t L0 = a >> 7;
  const uint32_t nl = (uint32_t)(((e - 1) >> 7) - L0 + 1);
  k.a0 = L0 << 7;
  k.lead = (uint32_t)(a & 127);
  k.te = (uint32_t)(((e - 1) & 127) + 1);
  k.h = ((nl - 1) & 7u) + 1;
  k.R = ((nl - k.h) >> 3) + 1;
  k.seg = (d.w & kSegFlag) ? (((d.w & kSegFirst) ? 1u : 2u) | ((d.w & kSegBig) ? 4u : 0u) | (d.y & 0xFFFF0000u))
                           : 0u;
  k.p = k.seg ? d.w & kSegIndexMask : d.w;
  k.state = 0;
  k.valid = valid;
  return k;
}
// (w8_unshift, w8_join, lane_xor8: crc32_device.h)
// Update mode: the register a task starts from - the payload's (out[p]); a split payload's first segment takes the
// register the count step moved aside (out[p] then collects the segments' xor), its later segments start from 0.
__device__ __forceinline__ uint32_t w8_state(const W8Task& t, const uint32_t* out, const SortedSplit& split) {
  if (!t.valid) return 0u;
  if (t.seg) return (t.seg & 1u) ? split.state[t.p] : 0u;
  return out[t.p];
}

//   PROBE (A/B builds only, microbench/sorted_probe.py; product = 0): bit 0 = every step takes the unmasked
//   branch, bit 1 = no fold (the data are xored into the register), bit 2 = loads from config 1's window (wave w,
//   step s: 8 KiB at (s W + w) 8 KiB) instead of the tasks' rounds, bit 3 = the same window loaded with config 1's
//   scalar base and immediate offsets, bit 4 = masked rounds without their byte masks - wrong digests, used to
//   measure what the masked rounds, the fold, the access pattern and the per-group addressing cost.
template <bool UPD, int PROBE = 0>
__device__ __forceinline__ void var_class_w8(uint4* lds4, const uint8_t* __restrict__ base,
                                             const uint4* __restrict__ desc, const uint32_t* __restrict__ range,
                                             const uint4* __restrict__ img_slice, const uint4* __restrict__ img_w8,
                                             uint32_t* __restrict__ out, const SortedSplit& split) {
  constexpr int G = 8;
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  const uint32_t l = threadIdx.x & 63, l3 = (l >> 3) & 1, j = l & 7;
  const size_t gid = group_id<kW8Block, G, kVwg>();
  const size_t ngroups = ((size_t)gridDim.x * kW8Block) / G;
  const size_t t_begin = range[0], t_end = range[1];
  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = 0;  // (the w8 join is unreplicated)
  const uint32_t voff = coalesced_lane_offset(l);  // line j, chunk 4 l3 + 2 l5 + l4 of a group's 1 KiB round
  const uint64_t b0 = (uint64_t)(uintptr_t)base;
  auto raw = [&](size_t t) { return raw_task<true>(t, t_end, base, desc, 0, 0); };
  // Load i reads the round of lane group m(i) = (i >> 2) + 2 (i & 1) + 4 ((i >> 1) & 1), so that after
  // transpose_blocks lane l holds half l3 of line j of the even group of its pair (l >> 3 & ~1) in v[0..3] and of
  // the odd one in v[4..7] (crc32_onekib_nt_kernel's layout). Invalid groups decode the last task of the list
  // (raw_task clamps), so every address is inside a payload's lines.
  uint32_t wstep = 0;  // steps so far (PROBE bits 2, 3)
  auto load = [&](const W8Task& tk, uint32_t r, uint4 (&v)[8]) __attribute__((always_inline)) {
    uint64_t ad = tk.a0 + (r == 0 ? 0ull : (uint64_t)tk.h * 128u + (uint64_t)(r - 1) * 1024u);
    if constexpr ((PROBE & 4) != 0)  // config 1's window instead of the tasks' rounds (wrong digests)
      ad = b0 + ((((uint64_t)wstep * (ngroups / 8) + (gid >> 3)) * 8192 + 1024 * (l >> 3)) & ((1ull << 29) - 1));
    if constexpr ((PROBE & 8) != 0) {  // the same window with config 1's scalar base + immediate offsets
      const uint64_t wb = ((((uint64_t)wstep * (ngroups / 8) + (uint32_t)__builtin_amdgcn_readfirstlane((int)(gid >> 3))) *
                           8192) & ((1ull << 29) - 1));
      const uint8_t* p = base + wb + voff;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const v4u32 x = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(p + 1024 * i));
        v[i] = make_uint4(x.x, x.y, x.z, x.w);
      }
      return;
    }
    const uint32_t lo = (uint32_t)ad, hi = (uint32_t)(ad >> 32);
    // the head round is end-aligned: lane j holds line j - (8 - h), and the lanes before line 0 re-read line 0
    // (zeroed in compute), so no load leaves the payload's lines and no line is read twice
    const uint32_t up = r == 0 ? 8 - tk.h : 0u;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int src = 8 * ((i >> 2) + 2 * (i & 1) + 4 * ((i >> 1) & 1));
      const uint64_t g = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, src) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)lo, src);
      const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)up, src);
      v[i] = gload16_nt(g, ((j > c ? j - c : 0u) << 7) | (voff & 127u));
    }
  };

  // Sets: block b owns the sets k NB + b (k even) and k NB + NB - 1 - b (k odd), NB = the grid's blocks (snake
  // order over the sorted list, so every block gets an even share of long and short sets); its 8 waves take them
  // in list order, wave w the w-th first, every later one from a counter in LDS when the wave's set is 3 steps from
  // its end, or a second one ahead while its sets last at most 2 steps: longest first, each to the wave that frees
  // up first (with the shortest interleaved, below). A claim's descriptors load into a register (one per step parity) and land in the wave's ring in LDS
  // at the next step, before its switch reads them: a register copy of a load in flight would wait for it.
  const uint32_t nb = gridDim.x, bb = blockIdx.x, m = l >> 3, wl = threadIdx.x >> 6;
  const uint32_t nsets = (uint32_t)((t_end - t_begin + 7) / 8);
  auto set_of = [&](uint32_t kk) {
    const uint64_t g = (uint64_t)kk * nb + ((kk & 1u) ? nb - 1 - bb : bb);
    return g < nsets ? (uint32_t)g : nsets;  // nsets: no set (every task_of >= t_end)
  };
  auto task_of = [&](uint32_t set) { return t_begin + 8 * (size_t)set + m; };
  uint32_t S0 = set_of(wl);  // the set being loaded
  if (!__syncthreads_or(task_of(S0) < t_end)) return;  // the block has no task
  uint4* const ring = lds4 + kLdsW8RingOff / 16 + wl * 4 * 8;  // [slot][group], 4 slots
  uint32_t* const ring_set = reinterpret_cast<uint32_t*>(lds4) + kLdsW8RingSetOff / 4 + wl * 4;
  uint64_t* const sets_taken = reinterpret_cast<uint64_t*>(lds4) + kLdsW8CounterOff / 8;
  // the block's sets: k NB + (b or NB - 1 - b) < nsets for k < nk
  const uint32_t full = nsets / nb, rem = nsets % nb;
  const uint32_t nk = full + (((full & 1u) ? nb - 1 - bb : bb) < rem ? 1u : 0u);
  // Pipeline: the load side holds the task whose round rL it loads this step (dL); the compute side (dC, rC) is
  // the load side one step later. Claimed sets [head, tail) wait in the ring (slot = index mod 4).
  W8Task dL = decode_w8(raw(task_of(S0)), task_of(S0) < t_end);
  if constexpr (UPD) dL.state = w8_state(dL, out, split);
  uint4 A[8], B[8];
  load(dL, 0, A);
  W8Task dC = dL;
  uint32_t rC = 0, rL = 1, head = 0, tail = 0;
  uint4 inA = make_uint4(0, 0, 0, 0), inB = inA;  // a claim's descriptors in flight, by step parity
  uint32_t setA = 0, setB = 0;
  bool pendA = false, pendB = false;
  load_image<kLdsW8ImageBytes, kW8Block, kLdsCommonBytes>(lds4, img_slice, nullptr, img_w8);
  if (threadIdx.x == 0) *sets_taken = kW8Block / 64;  // front: the waves' first sets; back: none
  __syncthreads();

  // claim rule (wave-uniform): no set queued and S0 within 3 steps of its end, or fewer than 2 queued while S0
  // lasts at most 2 steps
  // The claims alternate between the front of the block's list and its back (the shortest sets, mostly one masked
  // round each), so that the masked rounds' arithmetic overlaps other waves' streaming instead of filling the
  // launch's tail. One 64-bit counter holds both ends' counts, so no set is taken twice.
  bool back = true;
  auto maybe_claim = [&](uint4& in, uint32_t& set, bool& pend) __attribute__((always_inline)) {
    const uint32_t q = tail - head;
    const bool near = __builtin_amdgcn_ballot_w64(rL + 3 < dL.R) == 0;
    const bool shrt = __builtin_amdgcn_ballot_w64(dL.R > 2) == 0;
    if ((near && q == 0) || (shrt && q < 2)) {
      uint64_t old = 0;
      if (l == 0)
        old = __hip_atomic_fetch_add(sets_taken, back ? (1ull << 32) : 1ull, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
      const uint32_t f = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)old),
                     bk = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(old >> 32));
      set = f + bk < nk ? set_of(back ? nk - 1 - bk : f) : nsets;
      back = !back;
      in = raw(task_of(set));
      pend = true;
      tail++;
    }
  };
  maybe_claim(inB, setB, pendB);  // (a first set of <= 4 rounds: its successor is due at once)

  uint32_t s = 0;
  auto fold = [&](uint4 (&v)[8]) __attribute__((always_inline)) {
    // the round register (shift_{7*128} of the lane's register; 0 after a payload's last round) enters the
    // first halves: lanes with l3 = 0 fold the first half of their own line and of lane ^ 8's
    const uint32_t sin = byte_map64(s, lds, kLdsW8RoundOff);
    const uint32_t sp = (uint32_t)__builtin_amdgcn_mov_dpp((int)sin, 0x128, 0xF, 0xF, false);  // lane ^ 8's
    v[0].x ^= l3 ? 0u : sin;
    v[4].x ^= l3 ? 0u : sp;
    s = fold_halves(v, k, lds, l3, kLdsW8HalfOff);
  };
  auto compute = [&](uint4 (&v)[8], W8Task cur, uint32_t r_c) __attribute__((always_inline)) {
    cur.valid = cur.valid && r_c < cur.R;
    const bool body = cur.valid && r_c > 0 && r_c + 1 < cur.R;
    transpose_blocks(v);
    // (a group that finished its task before the rest of its set idles: r_c >= R, treated as invalid)
    if constexpr ((PROBE & 2) != 0) {
      uint32_t x = s;
#pragma unroll
      for (int i = 0; i < 8; i++) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
      s = x;
      if (cur.valid && r_c + 1 == cur.R && j == 7) out[cur.p] = s;
      return;
    }
    if ((PROBE & 1) != 0 || __builtin_amdgcn_ballot_w64(!body) == 0) {  // every group in a body round: no masks
      fold(v);
      if constexpr ((PROBE & 1) != 0) {
        if (cur.valid && r_c + 1 == cur.R && j == 7) out[cur.p] = s;
      }
      return;
    }
    // Masked round. This lane's group (l >> 3): keep bytes [lo, hi) of half q of its line j, for q = l3 (own use)
    // and 1 - l3 (sent to lane ^ 8, whose v holds this group's half 1 - l3 ... = the partner's own half).
    const bool head = cur.valid && r_c == 0, last = cur.valid && r_c + 1 == cur.R;
    // (end-aligned head round: line 0 in lane 8 - h, the lanes before it zeroed; the last line is always lane 7)
    const uint32_t up = 8 - cur.h;
    const int32_t line_lo = head && j == up ? (int32_t)cur.lead : 0;
    const int32_t line_hi = !cur.valid || (head && j < up) ? 0 : (last && j == 7 ? (int32_t)cur.te : 128);
    const int32_t lo_own = min(max(line_lo - 64 * (int32_t)l3, 0), 64), hi_own = min(max(line_hi - 64 * (int32_t)l3, 0), 64);
    const int32_t lo_oth = min(max(line_lo - 64 * (int32_t)(l3 ^ 1), 0), 64),
                  hi_oth = min(max(line_hi - 64 * (int32_t)(l3 ^ 1), 0), 64);
    // lane ^ 8 holds the other group of the pair and computed its bounds for our half as its "other" half
    const int32_t lo_par = lane_xor8(lo_oth), hi_par = lane_xor8(hi_oth);
    // v[0..3]: the even group of the pair (own if l3 = 0), v[4..7]: the odd one
    const int32_t lo_a = l3 ? lo_par : lo_own, hi_a = l3 ? hi_par : hi_own;
    const int32_t lo_b = l3 ? lo_own : lo_par, hi_b = l3 ? hi_own : hi_par;
    if ((PROBE & 16) == 0 && __builtin_amdgcn_ballot_w64(lo_a > 0 || hi_a < 64 || lo_b > 0 || hi_b < 64) != 0) {
      uint4 va[4] = {v[0], v[1], v[2], v[3]}, vb[4] = {v[4], v[5], v[6], v[7]};
      mask_chunks<4>(va, lo_a, hi_a, lds);
      mask_chunks<4>(vb, lo_b, hi_b, lds);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        v[i] = va[i];
        v[4 + i] = vb[i];
      }
    }
    fold(v);
    // head round: line 0's register gains the init as a register at the payload start, shift_{128-lead}(init)
    if (__builtin_amdgcn_ballot_w64(head) != 0) {
      if (head && j == up && (cur.seg & 2u) == 0) {  // (a split payload's later segments start from register 0)
        if constexpr (UPD) {
          uint32_t x = w8_unshift(cur.state, cur.lead, lds);                       // shift_{-lead}
          s ^= byte_map64(byte_map64(x, lds, kLdsW8HalfOff), lds, kLdsW8HalfOff);  // shift_128
        } else {
          s ^= lds[kLdsW8InitOff / 4 + cur.lead];  // shift_{128-lead}(kInit)
        }
      }
    }
    if (__builtin_amdgcn_ballot_w64(last) != 0) {
      const uint32_t t = group_xor_reduce<G>(w8_join(s, lds, j));
      const uint32_t over = 128 - cur.te;  // the last line's bytes past the payload end (zeroed above)
      uint32_t u = 0;
      if (last && j == G - 1) u = over ? w8_unshift(t, over, lds) : t;
      const bool segl = last && j == G - 1 && cur.seg != 0;
      if (__builtin_amdgcn_ballot_w64(segl) != 0) {
        // segments: shift_{m seg}(raw) into the payload's digest (preset to ~0; update mode: 0). When all 8 groups end segments of
        // one payload (a long payload's segments are neighbours in the sorted list), one atomic for the wave: one
        // address took every segment's atomic otherwise (16 payloads of 64 MiB: 963 us per call).
        uint32_t x = u;
        const uint32_t m = cur.seg >> 16;
        if (segl && m) {
          const uint32_t* P = ((cur.seg & 4u) ? split.powers_big : split.powers) + (size_t)(m - 1) * 32;
          x = 0;
#pragma unroll
          for (int b = 0; b < 32; b++) x ^= P[b] & (0u - ((u >> b) & 1u));
        }
        const uint32_t p7 = (uint32_t)__builtin_amdgcn_readlane((int)cur.p, 7);
        const bool same = __builtin_amdgcn_ballot_w64(segl && cur.p == p7) == 0x8080808080808080ull;
        if (same) {
          uint32_t xs = 0;
#pragma unroll
          for (int g = 0; g < 8; g++) xs ^= (uint32_t)__builtin_amdgcn_readlane((int)x, 8 * g + 7);
          if (l == 7) atomicXor(out + p7, xs);
        } else if (segl) {
          atomicXor(out + cur.p, x);
        }
      }
      if (last && j == G - 1 && !cur.seg) out[cur.p] = UPD ? u : ~u;
      s = last ? 0u : s;
    }
  };

  auto step = [&](uint4 (&cur_buf)[8], uint4 (&nxt_buf)[8], uint4& in_new, uint32_t& set_new, bool& pend_new,
                  const uint4& in_old, uint32_t set_old, bool& pend_old) __attribute__((always_inline)) {
    if (pend_old) {  // the previous step's claim (index tail - 1) lands; its load preceded that step's data loads
      const uint32_t slot = (tail - 1) & 3u;
      if (j == 0) ring[slot * 8 + m] = in_old;
      if (l == 0) ring_set[slot] = set_old;
      pend_old = false;
    }
    if (__builtin_amdgcn_ballot_w64(rL < dL.R) == 0) {  // every group is done with S0: the queue's head
      const uint32_t slot = head & 3u;
      head++;
      S0 = ring_set[slot];
      dL = decode_w8(ring[slot * 8 + m], task_of(S0) < t_end);
      if constexpr (UPD) dL.state = w8_state(dL, out, split);
      rL = 0;
    }
    maybe_claim(in_new, set_new, pend_new);
    ANNETY_PRIO_HI();
    load(dL, dL.valid && rL < dL.R ? rL : 0u, nxt_buf);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    compute(cur_buf, dC, rC);
    dC = dL;
    rC = rL;
    rL++;
    wstep++;
  };
  // wave-uniform loop: the loads and the cross-lane steps need every group (a finished group reads a round of
  // the class's last payload and stores nothing)
  while (__builtin_amdgcn_ballot_w64(dC.valid) != 0) {
    step(A, B, inA, setA, pendA, inB, setB, pendB);
    step(B, A, inB, setB, pendB, inA, setA, pendA);
  }
}

// The sorted path in one launch: every non-empty payload (desc[ranges[0], ranges[1]), longest first;
// crc32_bucket_place) in var_class_w8.
//   PROBE: A/B builds only (microbench/sorted_probe.py); the product runs PROBE 0.
template <bool UPD, int PROBE = 0>
__global__ __launch_bounds__(kW8Block) void crc32_var_sorted_kernel(const uint8_t* __restrict__ base, size_t n,
                                                                  const uint4* __restrict__ desc,
                                                                  const uint32_t* __restrict__ ranges,
                                                                  const uint4* __restrict__ img_slice,
                                                                  const uint4* __restrict__ img_w8,
                                                                  uint32_t* __restrict__ out, SortedSplit split,
                                                                  AutoChoice choice) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsW8TotalBytes / 16];
  static_assert(kW8Block % 64 == 0 && kW8Block / 64 <= kW8MaxWaves, "the claim rings hold one ring per wave");
  if (choice.ws) {  // the device's choice (AutoChoice): nothing to do when it is the arena
    ArenaSpan sp;
    if (choose_arena(choice, sp)) return;
  }
  var_class_w8<UPD, PROBE>(lds4, base, desc, ranges, img_slice, img_w8, out, split);
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

hipError_t launch_var_sorted(const VarLaunch& a, const void* img_w8, const SortedSplit& split, hipStream_t stream) {
  const unsigned blocks = (unsigned)std::max<size_t>(1, a.max_blocks);
  note_kernel("crc32_var_sorted_kernel");
#define ANNETY_SORTED_LAUNCH(UPD, PROBE)                                                                      \
  hipLaunchKernelGGL((crc32_var_sorted_kernel<UPD, PROBE>), dim3(blocks), dim3(kW8Block), 0, stream,            \
                     static_cast<const uint8_t*>(a.base), a.n, static_cast<const uint4*>(a.desc), a.range,      \
                     static_cast<const uint4*>(a.img_slice), static_cast<const uint4*>(img_w8), a.out, split, \
                     a.choice)
#ifdef ANNETY_CRC_AB
  static const int probe = ANNETY_AB_KNOB("ANNETY_CRC_W8_PROBE", 0);
  if (!a.update && probe == 1) ANNETY_SORTED_LAUNCH(false, 1);
  else if (!a.update && probe == 16) ANNETY_SORTED_LAUNCH(false, 16);
  else if (!a.update && probe == 2) ANNETY_SORTED_LAUNCH(false, 2);
  else if (!a.update && probe == 6) ANNETY_SORTED_LAUNCH(false, 6);
  else if (a.update) ANNETY_SORTED_LAUNCH(true, 0);
  else ANNETY_SORTED_LAUNCH(false, 0);
#else
  if (a.update) ANNETY_SORTED_LAUNCH(true, 0);
  else ANNETY_SORTED_LAUNCH(false, 0);
#endif
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
