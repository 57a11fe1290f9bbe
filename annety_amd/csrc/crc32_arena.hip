// Arena path for variable-length batches whose payloads lie in one buffer (a NetBuffer, a frame
// stream, a packed batch: BASELINE config 3). Two launches, no sort:
//
//  1. crc32_arena_lines_kernel streams EVERY 128-byte line of the arena, payload-agnostic, in the
//     access shape of the config-1 kernel (a wave reads 64 consecutive lines = one 8 KiB superblock
//     per round). Per line it writes the raw CRC (register 0, no init, no xorout) c1, per aligned
//     1 KiB block c8 = join of 8 lines, per 8 KiB superblock c64 = join of 8 blocks. No byte masks,
//     no per-payload state: the arena runs at the fixed-batch rate whatever the length mix.
//  2. crc32_arena_stitch_kernel gives one lane per payload. The payload's first and last lines are
//     folded from the data with byte masks; the lines between come from c1/c8/c64 by Horner's rule
//         acc = shift_|unit|(acc) ^ crc(unit),   units of 128 B, 1 KiB and 8 KiB,
//     so a 64 KiB payload takes at most ~34 steps of 8 nibble-table lookups. The register before
//     the payload enters as shift_{128-lead}(s) (s = 0xFFFFFFFF, or the caller's register in update
//     mode, include/Crc32c.h:71-82), and the zero bytes after the payload end in its last line are
//     removed by one inverse shift.
//
// Reference semantics: crc32_long include/Crc32c.h:58-69 (digests), crc32_update :71-82 (update
// mode); the math identities are in crc32_math.h. DESIGN.md §2.8.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "crc32_device.h"
#include "crc32_kernels.h"
#include "crc32_math.h"

namespace annety_crc {
namespace {

// 512 lanes per block (one block per CU, LDS-bound), which leaves 256 VGPRs for the four-chain edge
// fold; a config-3 batch (165k payloads) is 1.26 payloads per lane. (1024-lane blocks, which cap the kernel at 128 VGPRs, returned wrong digests
// for whole waves now and then on the MI355X - a register-pressure-dependent fault we did not pin
// down)
constexpr int kStitchBlock = 512;

// Keep bytes [lo8/8, hi8/8) of a 128-byte line, zero the rest (branch-free, per 32-bit word).
__device__ __forceinline__ void mask_line(uint4 (&v)[8], int32_t lo8, int32_t hi8) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
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

// shift_{-m} for m in [0, 128): U_hi[m >> 4] o U_lo[m & 15]
__device__ __forceinline__ uint32_t unshift(uint32_t t, uint32_t m, const uint32_t* lds) {
  t = nibble_map_uniform(t, lds, kLdsStitchUnshiftOff + (m & 15u) * 512);
  return nibble_map_uniform(t, lds, kLdsStitchUnshiftOff + 8192 + (m >> 4) * 512);
}

__device__ __forceinline__ uint32_t gload4(uint64_t addr) {
  return *(const __attribute__((address_space(1))) uint32_t*)addr;
}

//   PROBE (microbench only; product = 0): 1 = descriptors and stores only, 2 = + edge-line loads,
//   3 = + edge folds (no interior steps), 4 = full but single-chain folds (absorb_line twice) - wrong
//   digests for 1-3, used to measure what the stages cost.
template <bool UPD, int BLK = kStitchBlock, int PROBE = 0>
__global__ __launch_bounds__(BLK) void crc32_arena_stitch_kernel(
    const uint8_t* __restrict__ base, uint64_t line_lo, uint64_t line_hi, uint64_t sb0,
    const uint64_t* __restrict__ d_off, const uint32_t* __restrict__ d_len, size_t n,
    const uint32_t* __restrict__ c1, const uint32_t* __restrict__ c8, const uint32_t* __restrict__ c64,
    const uint4* __restrict__ img_slice, const uint4* __restrict__ img_stitch, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsStitchImageBytes / 16];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;
  const uint64_t c1b = (uint64_t)(uintptr_t)c1 - 4 * (sb0 * 64);
  const uint64_t c8b = (uint64_t)(uintptr_t)c8 - 4 * (sb0 * 8);
  const uint64_t c64b = (uint64_t)(uintptr_t)c64 - 4 * sb0;

  struct Pay {
    uint64_t L0, L1;
    uint32_t lead, tailend, len;
  };
  auto describe = [&](size_t p) {
    Pay y;
    y.len = d_len[p];
    const uint64_t a = (uint64_t)(uintptr_t)base + d_off[p];
    const uint64_t e = a + (y.len ? y.len - 1 : 0);
    y.L0 = a >> 7;
    y.L1 = e >> 7;
    y.lead = (uint32_t)(a & 127);
    y.tailend = (uint32_t)(e & 127) + 1;
    return y;
  };
  // Horner steps over interior lines [i, L1) from the arena pass: 8 independent loads per batch, then 8
  // steps acc = shift_unit(acc) ^ crc(unit) with units of 8 KiB / 1 KiB / 128 B (lv = 2 / 1 / 0, 3 = none)
  auto fetch = [&](uint64_t& i, uint64_t L1, uint32_t (&cv)[8], uint32_t& lv) {  // lv: 2 bits per step
    lv = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const bool big = (i & 63) == 0 && i + 64 <= L1;
      const bool mid = !big && (i & 7) == 0 && i + 8 <= L1;
      const bool any = i < L1;
      lv |= (any ? (big ? 2u : (mid ? 1u : 0u)) : 3u) << (2 * q);
      const uint64_t addr = big ? c64b + 4 * (i >> 6) : (mid ? c8b + 4 * (i >> 3) : c1b + 4 * (any ? i : L1 - 1));
      cv[q] = gload4(addr);
      i += any ? (big ? 64 : (mid ? 8 : 1)) : 0;
    }
  };
  auto apply = [&](uint32_t acc, const uint32_t (&cv)[8], uint32_t lv) {
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const uint32_t l = (lv >> (2 * q)) & 3u;
      if (l < 3) acc = nibble_map_uniform(acc, lds, kLdsLevelOff + l * 512) ^ cv[q];
    }
    return acc;
  };
  auto process = [&](size_t p, const Pay& y, uint4 (&v)[8], uint4 (&w)[8]) {
    if (y.len == 0) {  // crc of the empty string is 0; update mode leaves the register alone
      if constexpr (!UPD) out[p] = 0u;
      return;
    }
    const uint32_t s0 = UPD ? out[p] : kInit;
    if constexpr (PROBE == 1) {
      out[p] = (uint32_t)y.L0 ^ y.lead ^ s0;
      return;
    }
    if constexpr (PROBE == 2) {
      uint32_t t = 0;
#pragma unroll
      for (int q = 0; q < 8; q++) t ^= v[q].x ^ w[q].y;
      out[p] = t;
      return;
    }
    const bool interior = y.L1 >= y.L0 + 2;
    const bool arena = y.L0 + 1 >= line_lo && y.L1 - 1 <= line_hi;
    uint64_t i = y.L0 + 1;
    uint32_t cv[8], cv2[8], lv = 0, lv2 = 0;
    if (PROBE != 3 && interior && arena) {  // first 16 steps in flight during the edge folds
      fetch(i, y.L1, cv, lv);
      fetch(i, y.L1, cv2, lv2);
    }
    // edge lines: the first keeps [lead, 128) (or [lead, tailend) when it is also the last), the last
    // keeps [0, tailend); both folded together (a single-line payload folds its line twice, unused)
    mask_line(v, (int32_t)y.lead * 8, (int32_t)(y.L0 == y.L1 ? y.tailend : 128u) * 8);
    mask_line(w, 0, (int32_t)y.tailend * 8);
    uint32_t acc, x;
    if constexpr (PROBE == 4) {
      acc = absorb_line(0u, v, k, lds);
      x = absorb_line(0u, w, k, lds);
    } else {
      absorb_two_lines(v, w, k, lds, acc, x);
    }
    // register before the payload: raw(P, s) = shift_|P|(s) ^ raw(P, 0), |P| = 128 - lead
    acc ^= unshift(nibble_map_uniform(s0, lds, kLdsLevelOff), y.lead, lds);
    if (y.L1 > y.L0) {
      if (PROBE == 3) {
      } else if (interior && arena) {
        acc = apply(acc, cv, lv);
        acc = apply(acc, cv2, lv2);
        while (i < y.L1) {
          fetch(i, y.L1, cv, lv);
          fetch(i, y.L1, cv2, lv2);
          acc = apply(acc, cv, lv);
          acc = apply(acc, cv2, lv2);
        }
      } else {
        // payload reaches outside the arena the caller declared: fold its interior lines directly
        for (; i < y.L1; i++) {
          uint4 u[8];
#pragma unroll
          for (int q = 0; q < 8; q++) u[q] = gload16((i << 7) + 16 * q);
          acc = nibble_map_uniform(acc, lds, kLdsLevelOff) ^ absorb_line(0u, u, k, lds);
        }
      }
      acc = nibble_map_uniform(acc, lds, kLdsLevelOff) ^ x;
    }
    acc = unshift(acc, 128 - y.tailend, lds);  // drop the zero bytes after the payload end
    out[p] = UPD ? acc : ~acc;
  };
  auto load_edges = [&](const Pay& y, uint4 (&v)[8], uint4 (&w)[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = gload16((y.L0 << 7) + 16 * i);
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = gload16((y.L1 << 7) + 16 * i);
  };

  // contiguous payload ranges per block (coalesced descriptor loads), the same count for every block;
  // the first payload's descriptor and edge lines are in flight while the LDS image is staged
  const size_t per = (n + gridDim.x - 1) / gridDim.x;
  const size_t p_end = std::min(n, (size_t)(blockIdx.x + 1) * per);
  size_t p = (size_t)blockIdx.x * per + threadIdx.x;
  Pay y{};
  uint4 v[8], w[8];
  if (p < p_end) {
    y = describe(p);
    load_edges(y, v, w);
  }
  load_image<kLdsStitchImageBytes, BLK, kLdsCommonBytes>(lds4, img_slice, nullptr, img_stitch);
  __syncthreads();
  for (; p < p_end; p += BLK) {
    if (p != (size_t)blockIdx.x * per + threadIdx.x) {
      y = describe(p);
      load_edges(y, v, w);
    }
    process(p, y, v, w);
  }
}

}  // namespace

size_t stitch_blocks(const ArenaLaunch& a) {
  return std::max<size_t>(1, std::min<size_t>(a.max_blocks, (a.n + kStitchBlock - 1) / kStitchBlock));
}

hipError_t launch_arena(const ArenaLaunch& a, hipStream_t stream) {
  if (a.nsb) {
    const hipError_t e = launch_arena_lines(a, stream);  // crc32_kernels.hip
    if (e != hipSuccess) return e;
  }
  const size_t blocks = stitch_blocks(a);
#define ANNETY_STITCH(UPD)                                                                                     \
  hipLaunchKernelGGL((crc32_arena_stitch_kernel<UPD>), dim3((unsigned)blocks), dim3(kStitchBlock), 0, stream,  \
                     static_cast<const uint8_t*>(a.base), a.line_lo, a.line_hi, a.sb0, a.off, a.len, a.n, a.c1,   \
                     a.c8, a.c64, static_cast<const uint4*>(a.img_slice), static_cast<const uint4*>(a.img_stitch), \
                     a.out)
  if (a.update) ANNETY_STITCH(true);
  else ANNETY_STITCH(false);
#undef ANNETY_STITCH
  return hipGetLastError();
}

}  // namespace annety_crc
