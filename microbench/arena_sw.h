// MICROBENCH ONLY (not in the product library): the store-wave arena line pass measured in round 3 and
// rejected: 240 us against 186-193 us for the product's burst line pass; with the store
// wave storing nothing 194 us, and the 9-wave block with no hand-off at all 192 us against 177 us for the
// 8-wave pass without S stores (profiles/r03/store_wave/). Included by microbench/arena_mb.hip after the
// product sources.
#pragma once

namespace annety_crc {
namespace {

// ---- store-wave variant: the streaming waves never store ----
// A wave's vector-memory operations retire in issue order, loads and stores alike (the vmcnt counter):
// a store issued between two task loads holds the later loads' retirement until its own acknowledgement,
// which under a saturated read stream takes about a loaded round trip. Bursting S every 8 tasks still cost
// 15-20 us of a 186 us pass. Here the 8 streaming waves of a block hand S and SB to a
// ninth wave through an LDS ring (kSwRing task slots per streaming wave), and only that wave stores:
// S of full superblock i at S[i * 64 + line] and SB at SB[i * 8 + block] (linear: the stitch finds them
// without a division). The (at most two) partial superblocks at the arena ends are stored directly by
// their waves into S_edge/SB_edge as before.
constexpr int kSwBlock = kBlock + 64;
constexpr uint32_t kSwRing = 4;
constexpr uint32_t kSwSlotWords = 72;  // S[64] + SB[8]
constexpr uint32_t kSwRingOff = kLdsArenaImageBytes;
constexpr uint32_t kSwCntOff = kSwRingOff + 8 * kSwRing * kSwSlotWords * 4;  // produced[8], consumed[8]
constexpr uint32_t kLdsArenaSwBytes = kSwCntOff + 64;
static_assert(kLdsArenaSwBytes <= 163840, "line pass + ring must fit one CU's LDS");

__device__ __forceinline__ uint32_t lds_load_relaxed(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_relaxed(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

//   PROBE (microbench only; product = 0): bit 0 = the store wave takes the slots but stores nothing;
//   bit 1 = no hand-off at all (the streaming waves skip the ring, the store wave exits at once).
template <int PROBE = 0>
__device__ __forceinline__ void arena_line_pass_sw(const uint8_t* __restrict__ base, const LineOut& ar, uint32_t bid,
                                                   uint32_t nbid, uint4* lds4, const uint4* __restrict__ img_slice,
                                                   const uint4* __restrict__ img_group8,
                                                   const uint4* __restrict__ img_sb) {
  constexpr int BLK = kBlock, VWG = kVwg;
  uint32_t* ldsw = reinterpret_cast<uint32_t*>(lds4);
  const uint32_t* lds = ldsw;
  uint32_t* ring = ldsw + kSwRingOff / 4;
  uint32_t* produced = ldsw + kSwCntOff / 4;
  uint32_t* consumed = produced + 8;
  const size_t ngroups = (size_t)nbid * (BLK / 8);
  const size_t n = (size_t)(ar.fs1 - ar.fs0) * 8;  // full 1 KiB blocks = lane-group tasks
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // first lane group of streaming wave w (the virtual-workgroup mapping of arena_line_pass)
  auto wave_gid0 = [&](uint32_t w) -> size_t {
    const size_t v = (size_t)bid + (size_t)nbid * ((64 * w) / VWG);
    return (v * VWG + (64 * w) % VWG) / 8;
  };
  auto wave_tasks = [&](size_t gid0) -> uint32_t { return gid0 < n ? (uint32_t)((n - 1 - gid0) / ngroups + 1) : 0u; };

  if (wave == BLK / 64) {  // ---------------- the store wave ----------------
    load_image<kLdsArenaImageBytes, kSwBlock>(lds4, img_slice, img_group8, img_sb);
    if (lane < 16) lds_store_relaxed(produced + lane, 0u);
    __syncthreads();
    uint32_t total[8], cons[8];
    size_t gid0[8];
#pragma unroll
    for (uint32_t w = 0; w < 8; w++) {
      gid0[w] = wave_gid0(w);
      total[w] = (PROBE & 2) ? 0u : wave_tasks(gid0[w]);
      cons[w] = 0;
    }
    const uint32_t q = lane >> 4, part = lane & 15;
    for (;;) {
      // up to four ready tasks (any streaming waves), one per quarter of the wave
      uint32_t sw[4] = {0, 0, 0, 0}, st[4] = {0, 0, 0, 0}, cnt = 0, left = 0;
#pragma unroll
      for (uint32_t w = 0; w < 8; w++) {
        const uint32_t avail = lds_load_relaxed(produced + w);
        while (cnt < 4 && cons[w] < avail) {
          sw[cnt] = w;
          st[cnt] = cons[w]++;
          cnt++;
        }
        left += total[w] - cons[w];
      }
      if (cnt == 0) {
        if (left == 0) break;  // every streaming wave's tasks are stored: the exit every store wave reaches
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      uint32_t w_l = sw[0], t_l = st[0];
#pragma unroll
      for (uint32_t k = 1; k < 4; k++) {
        w_l = q == k ? sw[k] : w_l;
        t_l = q == k ? st[k] : t_l;
      }
      const bool on = q < cnt;
      const uint32_t* slot = ring + (w_l * kSwRing + t_l % kSwRing) * kSwSlotWords;
      const uint4 sv = *reinterpret_cast<const uint4*>(slot + part * 4);
      const uint32_t sbv = slot[64 + (part & 7)];
      // full superblock of (w, t), relative to fs0: a wave's 8 groups are one superblock
      size_t g0 = gid0[0];
#pragma unroll
      for (uint32_t w = 1; w < 8; w++) g0 = w_l == w ? gid0[w] : g0;
      const uint64_t sbi = (g0 + (size_t)t_l * ngroups) / 8;
      if (on && (PROBE & 1) == 0) {
        const v4u32 v = {sv.x, sv.y, sv.z, sv.w};
        __builtin_nontemporal_store(v, reinterpret_cast<v4u32*>(ar.S + sbi * 64 + part * 4));
        if (part < 8) __builtin_nontemporal_store(sbv, ar.SB + sbi * 8 + part);
      }
      // the slots are read (the stores above consumed their data): hand them back
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) {
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
          if (k < cnt) lds_store_relaxed(consumed + sw[k], st[k] + 1);
      }
    }
    return;
  }

  // ---------------- the streaming waves (arena_line_pass without the global stores) ----------------
  const uint32_t j = threadIdx.x & 7;
  const size_t gid = (((size_t)bid + (size_t)nbid * (threadIdx.x / VWG)) * VWG + threadIdx.x % VWG) / 8;
  const int ntasks = gid < n ? (int)((n - 1 - gid) / ngroups + 1) : 0;
  const uint64_t pstep = ngroups * 1024;

  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;

  const uint8_t* lp = base + gid * 1024 + (size_t)j * kChunkBytes;
  uint4 A[8], B[8];
  if (ntasks > 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) A[i] = reinterpret_cast<const uint4*>(lp)[i];
  }
  load_image<kLdsArenaImageBytes, kSwBlock>(lds4, img_slice, img_group8, img_sb);
  __syncthreads();

  uint32_t* my_slot0 = ring + wave * kSwRing * kSwSlotWords;
  auto arena_scan = [&](uint32_t r, uint32_t& sbv) {
    uint32_t x = nibble_map_lane(r, lds, k.slot4);  // shift_{(7-j)*128}(r): the line seen from the block end
    uint32_t y;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x101, 0xF, 0xF, false);
    x ^= j + 1 < 8 ? y : 0u;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x102, 0xF, 0xF, false);
    x ^= j + 2 < 8 ? y : 0u;
    y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x104, 0xF, 0xF, false);
    x ^= j + 4 < 8 ? y : 0u;  // S: lines j..7
    const uint32_t g = lane >> 3;
    uint32_t u = 0;
    if (j == 0) u = sb_join(x, lds, g);
    uint32_t t[8];
    t[7] = (uint32_t)__builtin_amdgcn_readlane((int)u, 56);
#pragma unroll
    for (int h = 6; h >= 0; h--) t[h] = t[h + 1] ^ (uint32_t)__builtin_amdgcn_readlane((int)u, 8 * h);
    sbv = t[0];
#pragma unroll
    for (uint32_t h = 1; h < 8; h++) sbv = g == h ? t[h] : sbv;  // SB: blocks g..7
    return x;
  };
  // partial superblocks at the arena ends (wave-uniform, two waves of the grid): stored directly
  const uint64_t gw = (uint64_t)bid * (BLK / 64) + wave;
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
      const uint32_t x = arena_scan(absorb_line(0u, v, k, lds), sbv);
      ar.S_edge[gw * 64 + lane] = x;
      if (j == 0) ar.SB_edge[gw * 8 + (lane >> 3)] = sbv;
    }
  }

  auto finish = [&](uint32_t s, int t) {
    uint32_t sbv;
    const uint32_t x = arena_scan(s, sbv);
    if constexpr ((PROBE & 2) != 0) {
      my_slot0[lane] = x ^ sbv;  // keep the scan live
      return;
    }
    uint32_t* slot = my_slot0 + ((uint32_t)t % kSwRing) * kSwSlotWords;
    // the store wave has taken task t - kSwRing out of this slot (it keeps up: it does nothing else)
    while ((uint32_t)t >= kSwRing + lds_load_relaxed(consumed + wave)) __builtin_amdgcn_s_sleep(1);
    slot[lane] = x;
    if (j == 0) slot[64 + (lane >> 3)] = sbv;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's words land before the count
    if (lane == 0) lds_store_relaxed(produced + wave, (uint32_t)t + 1);
  };
  for (int t = 0; t < ntasks; t += 2) {
    ANNETY_PRIO_HI();
    {
      const uint4* s = reinterpret_cast<const uint4*>(t + 1 < ntasks ? lp + pstep : lp);
#pragma unroll
      for (int i = 0; i < 8; i++) B[i] = s[i];
    }
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    finish(absorb_line(0u, A, k, lds), t);
    ANNETY_PRIO_HI();
    {
      const uint4* s = reinterpret_cast<const uint4*>(t + 2 < ntasks ? lp + 2 * pstep : lp);
#pragma unroll
      for (int i = 0; i < 8; i++) A[i] = s[i];
    }
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    if (t + 1 < ntasks) finish(absorb_line(0u, B, k, lds), t + 1);
    lp += 2 * pstep;
  }
}


// First launch, store-wave form: 8 streaming waves + 1 store wave.
template <int PROBE = 0>
__global__ __launch_bounds__(kSwBlock) void crc32_arena_lines_sw_kernel(const uint8_t* __restrict__ base, LineOut ar,
                                                                        const uint4* __restrict__ img_slice,
                                                                        const uint4* __restrict__ img_group8,
                                                                        const uint4* __restrict__ img_sb) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsArenaSwBytes / 16];
  arena_line_pass_sw<PROBE>(base, ar, blockIdx.x, gridDim.x, lds4, img_slice, img_group8, img_sb);
}

}  // namespace

template <int PROBE = 0>
hipError_t launch_arena_lines_sw(const ArenaLaunch& a, hipStream_t stream) {
  const ArenaGeom geo = arena_geom(a);
  hipLaunchKernelGGL(crc32_arena_lines_sw_kernel<PROBE>, dim3((unsigned)geo.blocks), dim3(kSwBlock), 0, stream,
                     reinterpret_cast<const uint8_t*>((uintptr_t)(a.fs0 * 8192)), line_out(a, geo),
                     static_cast<const uint4*>(a.img_slice), static_cast<const uint4*>(a.img_group8),
                     static_cast<const uint4*>(a.img_sb));
  return hipGetLastError();
}

}  // namespace annety_crc
