// The arena line pass (crc32_arena_lines_kernel in crc32_arena.hip): the config-1 kernel's
// loop over full 8 KiB superblocks (a wave = 64 consecutive 128-byte lines per task, A/B register double
// buffer, unconditional next-task loads), storing per line the block-suffix CRC S and per block the
// superblock-suffix SB (layout: crc32_kernels.h). Included by crc32_arena.hip only.
#pragma once

#include "crc32_device.h"
#include "crc32_kernels.h"

namespace annety_crc {
namespace {

struct LineOut {
  uint32_t *S, *SB, *S_edge, *SB_edge;
  uint64_t W;  // line-pass waves = 8 * workgroups
  uint64_t byte_lo, byte_hi, line_lo, line_hi, sb0, nsb, fs0, fs1;
  uint64_t zero_line;
  const uint64_t* check;  // ArenaLaunch::check
  uint32_t check_parts;
  uint64_t check_lo, check_hi;
  bool check_any_order;
  AutoChoice choice;  // ArenaLaunch::choice: S = the scratch, the rest from the device's span (line_out_chosen)
  int64_t probe_delta;  // microbench only (PROBE bit 3): each loaded chunk is also stored at its address + this
};

// The line pass's geometry for the span the device chose (AutoChoice; the host's line_out in crc32_arena.hip).
__device__ __forceinline__ void line_out_chosen(LineOut& ar, const ArenaSpan& sp, const ArenaGeom& geo) {
  ar.SB = ar.S + geo.sb_off;
  ar.S_edge = ar.S + geo.edge_off;
  ar.SB_edge = ar.S_edge + 128;
  ar.W = geo.W;
  ar.byte_lo = sp.byte_lo;
  ar.byte_hi = sp.byte_hi;
  ar.line_lo = sp.line_lo;
  ar.line_hi = sp.line_hi;
  ar.sb0 = sp.sb0;
  ar.nsb = sp.nsb;
  ar.fs0 = sp.fs0;
  ar.fs1 = sp.fs1;
  ar.check = nullptr;
}

// (extent_of, choose_arena: crc32_device.h)
// ArenaLaunch::check: this call's extent equals the declared one and the batch is safe (sorted with small gaps,
// or any order when the host found the declared span inside one allocation: any_order).
__device__ __forceinline__ bool extent_matches(const uint64_t* check, uint32_t parts, uint64_t lo, uint64_t hi,
                                               bool any_order) {
  if (!check) return true;
  uint64_t l, h, s, b;
  extent_of(check, parts, l, h, s, b);
  return l == lo && h == hi && (b == 0 || any_order);
}

//   PROBE (microbench only; product = 0): bit 0 drops the S stores, bit 1 the superblock scan, bit 2 only
//   the SB stores - wrong outputs, used to measure what those stages cost; bit 3 adds a copy of every loaded chunk
//   to its address + probe_delta (unaligned 16-byte stores: what a fused copy would cost the pass, microbench/copy_mb).
// `base` = the first full superblock (fs0 * 8192), passed as its own kernel argument: loads through a
// __restrict__ kernel-argument pointer compile to the config-1 kernel's schedule; the same loads through
// integer-built address-space-1 pointers ran this pass 30 % slower (microbench/arena_mb.hip).
// S bursts: nontemporal stores (1, the product) or default-policy stores (0, microbench A/B: they would
// leave S in the caches for the stitch).
#ifndef ANNETY_S_NT
#define ANNETY_S_NT 1
#endif

// NT (product 1; 0 = the per-line loads, for A/B through ANNETY_CRC_LINES_NT=0): a wave's 8 KiB superblock
// arrives as 8 coalesced nontemporal 1 KiB loads (one per block) and transpose_blocks() / fold_halves()
// (crc32_device.h) leave lane l with line l & 7 of block folded_block(l); lane group q = l / 8 then holds block
// bq = folded_block(8 q), and everything per block (the superblock join, SB, the S burst slots) follows bq.
template <int PROBE = 0, bool NT = true>
__device__ __forceinline__ void arena_line_pass(const uint8_t* __restrict__ base, const LineOut& ar, uint32_t bid,
                                                uint32_t nbid, uint4* lds4,
                                                const uint4* __restrict__ img_slice,
                                                const uint4* __restrict__ img_group8,
                                                const uint4* __restrict__ img_sb) {
  constexpr int BLK = kBlock, VWG = kVwg;
  // uniform over the grid: on a mismatch the stitch folds every payload directly
  if (!extent_matches(ar.check, ar.check_parts, ar.check_lo, ar.check_hi, ar.check_any_order)) return;
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  const uint32_t j = threadIdx.x & 7;
  const size_t gid = (((size_t)bid + (size_t)nbid * (threadIdx.x / VWG)) * VWG + threadIdx.x % VWG) / 8;
  const size_t ngroups = (size_t)nbid * (BLK / 8);
  const size_t n = (size_t)(ar.fs1 - ar.fs0) * 8;  // full 1 KiB blocks = lane-group tasks
  // n and ngroups are multiples of 8, so every lane of a wave has the same task count
  const int ntasks = gid < n ? (int)((n - 1 - gid) / ngroups + 1) : 0;
  const uint64_t pstep = ngroups * 1024;
  const uint32_t lane = threadIdx.x & 63;
  // this lane's block in its superblock, and the lane group holding block h
  const uint32_t blk = NT ? folded_block(lane) : lane >> 3;
  auto group_of = [](uint32_t h) { return NT ? (h >> 2) + 2 * (h & 1) + 4 * ((h >> 1) & 1) : h; };
  // the wave's first lane group (wave-uniform: scalar addressing of the coalesced loads)
  const size_t g0 = ((size_t)__builtin_amdgcn_readfirstlane((uint32_t)(gid >> 32)) << 32) |
                    (size_t)(__builtin_amdgcn_readfirstlane((uint32_t)gid) & ~7u);
  const size_t gblk = g0 + blk;  // the lane group whose block this lane's line is in

  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;

  const uint8_t* lp = NT ? base + g0 * 1024 + coalesced_lane_offset(lane) : base + gid * 1024 + (size_t)j * kChunkBytes;
  auto load = [&](const uint8_t* a, uint4 (&v)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if constexpr (NT) {
        const v4u32 x = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(a + 1024 * i));
        v[i] = make_uint4(x.x, x.y, x.z, x.w);
      } else {
        v[i] = reinterpret_cast<const uint4*>(a)[i];
      }
    }
  };
  uint4 A[8], B[8];
  if (ntasks > 0) load(lp, A);
  load_image<NT ? kLdsArenaNtImageBytes : kLdsArenaImageBytes, BLK>(lds4, img_slice, img_group8, img_sb);
  __syncthreads();

  // S of kSTasks = 16 consecutive tasks leaves in four 16-byte stores per lane, each 1 KiB contiguous per
  // wave: interleaved with the read stream, a dword per lane per task cost 30 us of a 211 us pass, 16-byte
  // quads of 4 tasks 20; with the coalesced loads 8-task bursts cost 14-15 us of a 173 us pass, 16-task
  // bursts 11 (170 us), 32-task bursts the same as 16 (microbench/arena_mb.hip, profiles/r03/nt/b16/).
  uint32_t q[kSTasks];
#pragma unroll
  for (uint32_t i = 0; i < kSTasks; i++) q[i] = 0;
  // r = raw CRC of this lane's line (line j of block b, its lane group holding the block's 8 lines in
  // order; block h on lane group gq(h)); returns S for it and (lanes j == 0) SB for its block
  auto arena_scan = [&](uint32_t r, uint32_t& sbv, uint32_t b, auto gq) {
    uint32_t x = nibble_map_lane(r, lds, k.slot4);  // shift_{(7-j)*128}(r): the line seen from the block end
    // suffix scan over the 8 lanes of the group (DPP row_shl:d = the value of lane + d in its row of 16)
    uint32_t y;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x101, 0xF, 0xF, false);
    x ^= j + 1 < 8 ? y : 0u;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x102, 0xF, 0xF, false);
    x ^= j + 2 < 8 ? y : 0u;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x104, 0xF, 0xF, false);
    x ^= j + 4 < 8 ? y : 0u;  // S: lines j..7
    sbv = 0;
    if constexpr ((PROBE & 2) == 0) {
      // the 8 blocks of a wave are one superblock: block b seen from the superblock end on its group's
      // lane 0, then the suffix scan of those 8 values in scalar registers
      uint32_t u = 0;
      if (j == 0) u = sb_join(x, lds, b);
      uint32_t t[8];
      t[7] = (uint32_t)__builtin_amdgcn_readlane((int)u, 8 * gq(7));
#pragma unroll
      for (int h = 6; h >= 0; h--) t[h] = t[h + 1] ^ (uint32_t)__builtin_amdgcn_readlane((int)u, 8 * gq(h));
      sbv = t[0];
#pragma unroll
      for (uint32_t h = 1; h < 8; h++) sbv = b == h ? t[h] : sbv;  // SB: blocks b..7
    }
    return x;
  };
  // partial superblocks at the arena ends (wave-uniform, two waves of the grid): per-line loads, line =
  // lane, block = lane / 8
  const uint64_t gw = (uint64_t)bid * (BLK / 64) + (threadIdx.x >> 6);
  if (gw < 2) {
    const uint64_t sb = gw == 0 ? ar.sb0 : ar.sb0 + ar.nsb - 1;
    if ((sb < ar.fs0 || sb >= ar.fs1) && (gw == 0 || sb != ar.sb0)) {
      const uint64_t line = sb * 64 + lane;
      const bool in = line >= ar.line_lo && line <= ar.line_hi;
      const uint64_t src = in ? line << 7 : ar.zero_line;
      uint4 v[8];
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = gload16(src + 16 * i);
      const int32_t lo8 = line == ar.line_lo ? (int32_t)(ar.byte_lo & 127) * 8 : 0;
      const int32_t hi8 = line == ar.line_hi ? (int32_t)(((ar.byte_hi - 1) & 127) + 1) * 8 : 1024;
      mask_line(v, lo8, hi8);
      uint32_t sbv;
      const uint32_t x = arena_scan(absorb_line(0u, v, k, lds), sbv, lane >> 3, [](uint32_t h) { return h; });
      if constexpr ((PROBE & 1) == 0) ar.S_edge[gw * 64 + lane] = x;
      if (j == 0) ar.SB_edge[gw * 8 + (lane >> 3)] = sbv;
    }
  }

  auto finish = [&](uint4 (&v)[8], int t) __attribute__((always_inline)) {
    if constexpr ((PROBE & 8) != 0) {
      const uint64_t a = (uint64_t)(uintptr_t)base + (g0 + (uint64_t)t * ngroups) * 1024 + coalesced_lane_offset(lane) +
                         (uint64_t)ar.probe_delta;
#pragma unroll
      for (int i = 0; i < 8; i++) gstore16(a + 1024 * i, v[i]);
    }
    uint32_t r;
    if constexpr (NT) {
      transpose_blocks(v);
      r = fold_halves(v, k, lds, (lane >> 3) & 1, kLdsArenaImageBytes);
    } else {
      r = absorb_line(0u, v, k, lds);
    }
    uint32_t sbv;
    const uint32_t x = arena_scan(r, sbv, blk, group_of);
    const uint32_t slot = (uint32_t)t & (kSTasks - 1);
#pragma unroll
    for (uint32_t i = 0; i < kSTasks; i++) q[i] = slot == i ? x : q[i];
    if constexpr ((PROBE & 6) == 0) {
      if (j == 0) ar.SB[(((uint64_t)t * ngroups + g0) / 8) * 8 + blk] = sbv;
    }
    if (slot == kSTasks - 1 || t + 1 == ntasks) {
      const uint64_t t0 = (uint64_t)t & ~(uint64_t)(kSTasks - 1);
      if constexpr ((PROBE & 1) == 0) {
        v4u32* dst = reinterpret_cast<v4u32*>(ar.S + arena_s_word(t0, gblk, j, ar.W));
#pragma unroll
        for (uint32_t b = 0; b < kSTasks / 4; b++) {  // 1 KiB apart
          const v4u32 w = {q[4 * b], q[4 * b + 1], q[4 * b + 2], q[4 * b + 3]};
          if constexpr (ANNETY_S_NT)
            __builtin_nontemporal_store(w, dst + 64 * b);
          else
            dst[64 * b] = w;
        }
      }
    }
  };
  // Loads are unconditional (past the last task a wave re-reads its current superblock, an L2 hit): with the
  // next task's loads behind a branch the waitcnt pass merges the two paths and waits vmcnt(0) before
  // every fold, which serialises the A/B double buffer.
  for (int t = 0; t < ntasks; t += 2) {
    ANNETY_PRIO_HI();
    load(t + 1 < ntasks ? lp + pstep : lp, B);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    finish(A, t);
    ANNETY_PRIO_HI();
    load(t + 2 < ntasks ? lp + 2 * pstep : lp, A);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    if (t + 1 < ntasks) finish(B, t + 1);
    lp += 2 * pstep;
  }
}

}  // namespace
}  // namespace annety_crc
