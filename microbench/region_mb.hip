// Feasibility of a one-launch config-3 design: can the arena line pass take each
// workgroup's payloads end to end in its own contiguous region (no S/SB stores, no stitch launch)?
// Measures, on a 1 GiB arena with the product's LDS image and fold:
//   MAP 0: the product's task map (superblocks grid-strided, two virtual 256-lane workgroups)
//   MAP 1: one contiguous region per workgroup (wave w takes superblocks r0 + w, r0 + w + 8, ...)
//   MAP 2: two contiguous half regions per workgroup (waves 0-3 and 4-7, like the virtual workgroups)
//   EXTRA 0: fold only; 1: + the S/SB scans and, per task and lane, one masked half-line fold mapped to
//   the superblock end (the work a payload boundary on every line would cost); 2: 1 + a 2-lane digest store
//   per task; 3: 1 on every other task only.
// Outputs are not checksums (timing only). Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Iannety_amd/csrc microbench/region_mb.hip -o microbench/region_mb -L/opt/rocm/lib -lrccl
#include "../annety_amd/csrc/crc32_kernels.hip"
#include "../annety_amd/csrc/crc32_arena.hip"
#include "../annety_amd/csrc/crc32_frames.hip"
#include "../annety_amd/csrc/crc32_host.cpp"
#include "../annety_amd/csrc/crc32_capi.cpp"
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
#define RC(x) do { int r_ = (x); if (r_) { printf("%s -> %d\n", #x, r_); exit(3); } } while (0)
using namespace annety_crc;

namespace {

// One 128-byte line as four 32-byte chains (16 LDS reads per wait instead of 8): timing only, the joins
// use the half-line map for every chain (the arena image has no shift_32 / shift_96 tables).
__device__ __forceinline__ uint32_t absorb_line4(const uint4 (&v)[8], const LaneCtx& k, const uint32_t* lds) {
  uint32_t xa = v[0].x, xb = v[2].x, xc = v[4].x, xd = v[6].x;
#pragma unroll
  for (int i = 0; i < 2; i++) {
    word4x4(xa, v[i].y, xb, v[2 + i].y, xc, v[4 + i].y, xd, v[6 + i].y, k);
    word4x4(xa, v[i].z, xb, v[2 + i].z, xc, v[4 + i].z, xd, v[6 + i].z, k);
    word4x4(xa, v[i].w, xb, v[2 + i].w, xc, v[4 + i].w, xd, v[6 + i].w, k);
    word4x4(xa, i == 0 ? v[1].x : 0u, xb, i == 0 ? v[3].x : 0u, xc, i == 0 ? v[5].x : 0u, xd, i == 0 ? v[7].x : 0u, k);
  }
  return nibble_map_uniform(xa, lds, kLdsHalfOff) ^ nibble_map_uniform(xb, lds, kLdsHalfOff) ^
         nibble_map_uniform(xc, lds, kLdsHalfOff) ^ xd;
}

// LM (load mode): 0 = a lane reads its own 128-byte line as 8 x 16 B (the product); 1 = coalesced, load i
// of a wave covers bytes [1024 i, 1024 i + 1024) of its 8 KiB (16 B per lane); 2 = 1 with nontemporal loads.
// Modes 1 and 2 fold the bytes in the wrong order (timing only).
template <int MAP, int EXTRA, int LM = 0>
__global__ __launch_bounds__(kBlock) void k_region(const uint8_t* __restrict__ base, uint64_t nsb,
                                                   const uint4* __restrict__ img_slice,
                                                   const uint4* __restrict__ img_group8,
                                                   const uint4* __restrict__ img_sb, uint32_t* __restrict__ out,
                                                   uint32_t* __restrict__ dig) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsArenaImageBytes / 16];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6, j = lane & 7, g = lane >> 3;
  uint64_t s, stride, s_end;
  if constexpr (MAP == 0) {
    const uint64_t v = blockIdx.x + (uint64_t)gridDim.x * (w / 4);
    s = 4 * v + (w % 4);
    stride = 8ull * gridDim.x;
    s_end = nsb;
  } else if constexpr (MAP == 1) {
    const uint64_t per = (nsb + gridDim.x - 1) / gridDim.x;
    s = blockIdx.x * per + w;
    stride = 8;
    s_end = min(nsb, (blockIdx.x + 1) * per);
  } else if constexpr (MAP == 3) {  // region, each workgroup starting at a different place in it
    const uint64_t per = (nsb + gridDim.x - 1) / gridDim.x;
    const uint64_t r0 = blockIdx.x * per, r1 = min(nsb, r0 + per);
    const uint64_t rot = ((uint64_t)blockIdx.x * 8 * 37) % per & ~7ull;
    s = r0 + rot + w;  // wraps below
    stride = 8;
    s_end = r1;
    (void)r0;
  } else if constexpr (MAP == 4) {  // regions of per + 1 superblocks: starts not 4 MiB apart
    const uint64_t per = (nsb + gridDim.x - 1) / gridDim.x + 1;
    s = blockIdx.x * per + w;
    stride = 8;
    s_end = min(nsb, (blockIdx.x + 1) * per);
  } else {
    const uint64_t per = (nsb + 2 * gridDim.x - 1) / (2 * gridDim.x);
    const uint64_t r = blockIdx.x + (uint64_t)gridDim.x * (w / 4);
    s = r * per + (w % 4);
    stride = 4;
    s_end = min(nsb, (r + 1) * per);
  }
  int ntasks = s < s_end ? (int)((s_end - 1 - s) / stride + 1) : 0;
  uint64_t wrap_at = ~0ull, wrap_to = 0;
  if constexpr (MAP == 3) {
    const uint64_t per = (nsb + gridDim.x - 1) / gridDim.x;
    const uint64_t r0 = blockIdx.x * per, r1 = min(nsb, r0 + per);
    ntasks = (int)((r1 - r0) / 8);
    wrap_at = (uint64_t)(uintptr_t)(base + r1 * 8192);
    wrap_to = (r1 - r0) * 8192;
  }
  const uint64_t pstep = stride * 8192;
  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;
  const uint8_t* lp = base + s * 8192 + (LM == 0 ? g * 1024 + j * 128 : lane * 16);
  constexpr uint32_t ES = LM == 0 ? 16 : 1024;
  auto ld = [&](const uint8_t* q, uint4 (&v)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint4* a = reinterpret_cast<const uint4*>(q + i * ES);
      if constexpr (LM == 2) {
        const v4u32 x = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(a));
        v[i] = make_uint4(x.x, x.y, x.z, x.w);
      } else {
        v[i] = *a;
      }
    }
  };
  uint4 A[8], B[8];
  if (ntasks > 0) ld(lp, A);
  load_image<kLdsArenaImageBytes, kBlock>(lds4, img_slice, img_group8, img_sb);
  __syncthreads();
  uint32_t acc = 0;
  auto finish = [&](const uint4 (&v)[8], int t) __attribute__((always_inline)) {
    uint32_t r;
    if constexpr (EXTRA == 4)
      r = absorb_line4(v, k, lds);
    else
      r = absorb_line(0u, v, k, lds);
    if constexpr (EXTRA == 0 || EXTRA == 4) {
      acc ^= r;
    } else {
      uint32_t x = nibble_map_lane(r, lds, k.slot4);
      uint32_t y;
      y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x101, 0xF, 0xF, false);
      x ^= j + 1 < 8 ? y : 0u;
      y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x102, 0xF, 0xF, false);
      x ^= j + 2 < 8 ? y : 0u;
      y = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x104, 0xF, 0xF, false);
      x ^= j + 4 < 8 ? y : 0u;
      uint32_t u = 0;
      if (j == 0) u = sb_join(x, lds, g);
      uint32_t tt[8];
      tt[7] = (uint32_t)__builtin_amdgcn_readlane((int)u, 56);
#pragma unroll
      for (int h = 6; h >= 0; h--) tt[h] = tt[h + 1] ^ (uint32_t)__builtin_amdgcn_readlane((int)u, 8 * h);
      uint32_t sbv = tt[0];
#pragma unroll
      for (uint32_t h = 1; h < 8; h++) sbv = g == h ? tt[h] : sbv;
      acc ^= x ^ sbv;
      if (EXTRA != 3 || (t & 1) == 0) {
        // a boundary on this lane's line at byte o: the masked half line [o, half end), two 32-byte chains
        const uint32_t o = (lane * 37u + (uint32_t)t) & 127u;
        uint4 h[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {  // arithmetic select: a ?: on the arrays became a scratch copy
          const uint32_t m = 0u - (uint32_t)(o >= 64);
          h[i] = make_uint4((v[i].x & ~m) | (v[4 + i].x & m), (v[i].y & ~m) | (v[4 + i].y & m),
                            (v[i].z & ~m) | (v[4 + i].z & m), (v[i].w & ~m) | (v[4 + i].w & m));
        }
        const int32_t lo8 = (int32_t)(o & 63) * 8;
        mask_line<4>(h, lo8, 512);
        uint32_t xa = h[0].x, xb = h[2].x;
#pragma unroll
        for (int i = 0; i < 2; i++) {
          word4x2(xa, h[i].y, xb, h[2 + i].y, k);
          word4x2(xa, h[i].z, xb, h[2 + i].z, k);
          word4x2(xa, h[i].w, xb, h[2 + i].w, k);
          word4x2(xa, i == 0 ? h[1].x : 0u, xb, i == 0 ? h[3].x : 0u, k);
        }
        const uint32_t z = nibble_map_uniform(xa, lds, kLdsHalfOff) ^ xb;
        const uint32_t c = sb_join(nibble_map_lane(z, lds, k.slot4) ^ x, lds, g) ^ sbv;
        acc ^= c;
        if constexpr (EXTRA == 2) {
          if (j == 0 && g < 2) dig[((s + (uint64_t)t * stride) * 2 + g) & ((1u << 20) - 1)] = c;
        }
      }
    }
  };
  for (int t = 0; t < ntasks; t += 2) {
    ANNETY_PRIO_HI();
    {
      const uint8_t* nx = lp + pstep;
      if constexpr (MAP == 3) nx = (uint64_t)(uintptr_t)nx >= wrap_at ? nx - wrap_to : nx;
      ld(t + 1 < ntasks ? nx : lp, B);
    }
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    finish(A, t);
    ANNETY_PRIO_HI();
    {
      const uint8_t* nx = lp + 2 * pstep;
      if constexpr (MAP == 3) {
        nx = (uint64_t)(uintptr_t)(lp + pstep) >= wrap_at ? nx - wrap_to : nx;
        nx = (uint64_t)(uintptr_t)nx >= wrap_at ? nx - wrap_to : nx;
      }
      ld(t + 2 < ntasks ? nx : lp, A);
    }
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    if (t + 1 < ntasks) finish(B, t + 1);
    lp += 2 * pstep;
    if constexpr (MAP == 3) {
      lp = (uint64_t)(uintptr_t)lp >= wrap_at ? lp - wrap_to : lp;
    }
  }
  out[(size_t)blockIdx.x * kBlock + threadIdx.x] = acc;
}

}  // namespace

int main() {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const size_t bytes = 1ull << 30;
  char* d;
  uint32_t *scratch, *out, *dig;
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(d, 0x3C, bytes));
  RC(annety_crc_init(0));
  DeviceCtx* c = nullptr;
  RC(current_ctx(&c));
  ArenaLaunch a{};
  arena_fill(*c, d, bytes, a);
  CK(hipMalloc(&scratch, arena_geom(a).words * 4));
  CK(hipMalloc(&out, 256 * kBlock * 4));
  CK(hipMalloc(&dig, 4 << 20));
  a.scratch = scratch;
  const uint64_t nsb = bytes / 8192;
  const auto* b = reinterpret_cast<const uint8_t*>(d);
  const auto* i0 = static_cast<const uint4*>(a.img_slice);
  const auto* i1 = static_cast<const uint4*>(a.img_group8);
  const auto* i2 = static_cast<const uint4*>(a.img_sb);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto t = [&](auto f, const char* name) {
    for (int w = 0; w < 100; w++) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 100; r++) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-44s %.1f us  %.0f GB/s\n", name, ms * 10, bytes / (ms / 100) / 1e6);
  };
#define KL(M, X, L) [&] { hipLaunchKernelGGL((k_region<M, X, L>), dim3(256), dim3(kBlock), 0, 0, b, nsb, i0, i1, i2, out, dig); }
#define K(M, X) [&] { hipLaunchKernelGGL((k_region<M, X>), dim3(256), dim3(kBlock), 0, 0, b, nsb, i0, i1, i2, out, dig); }
  for (int rep = 0; rep < 3; rep++) {
    t(K(0, 0), "map 0 grid-stride, fold only (2 chains)");
    t(K(0, 4), "map 0 grid-stride, fold only (4 chains)");
    t(KL(0, 0, 1), "map 0, fold only, coalesced loads");
    t(KL(0, 0, 2), "map 0, fold only, coalesced nt loads");
    t(KL(0, 0, 1), "map 0, fold only, coalesced loads");
  }
  if (getenv("ONLY_LOADS")) return 0;
  for (int rep = 0; rep < 2; rep++) {
    t([&] { CK(launch_arena_lines_p<0>(a, 0)); }, "product line pass (S + SB stores)");
    t([&] { CK(launch_arena_lines_p<3>(a, 0)); }, "product line pass PROBE 3 (no S, no SB)");
    t(K(0, 0), "map 0 grid-stride, fold only");
    t(K(1, 0), "map 1 region, fold only");
    t(K(2, 0), "map 2 half regions, fold only");
    t(K(3, 0), "map 3 region, rotated start, fold only");
    t(K(4, 0), "map 4 region, 4 MiB + 8 KiB apart, fold only");
    t(K(3, 1), "map 3 + scans + boundary fold every task");
    t(K(0, 1), "map 0 + scans + boundary fold every task");
    t(K(1, 1), "map 1 + scans + boundary fold every task");
    t(K(2, 1), "map 2 + scans + boundary fold every task");
    t(K(1, 2), "map 1 + boundary fold + 2-lane digest store");
    t(K(2, 2), "map 2 + boundary fold + 2-lane digest store");
    t(K(1, 3), "map 1 + boundary fold every other task");
  }
  return 0;
}
