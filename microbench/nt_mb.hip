// Coalesced nontemporal loads for the config-1 kernel: a wave's 8 loads each cover one
// whole 1 KiB payload (16 B per lane), nontemporal, and two permlane swap stages plus one DPP exchange
// turn them into the product's line-per-lane layout. Checks every digest against the product kernel and
// times both. Build (from the repo root):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Iannety_amd/csrc microbench/nt_mb.hip -o microbench/nt_mb -L/opt/rocm/lib -lrccl
#include "../annety_amd/csrc/crc32_kernels.hip"
#include "../annety_amd/csrc/crc32_arena.hip"
#include "../annety_amd/csrc/crc32_frames.hip"
#include "../annety_amd/csrc/crc32_host.cpp"
#include "../annety_amd/csrc/crc32_capi.cpp"
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
#define RC(x) do { int r_ = (x); if (r_) { printf("%s -> %d\n", #x, r_); exit(3); } } while (0)
using namespace annety_crc;

namespace {

// v[r] <-> v[r ^ d] across lane bit 4 (d = 1, permlane16) or lane bit 5 (d = 2, permlane32)
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

// raw CRCs of two 64-byte chains from register 0: v[0..3] and v[4..7]
__device__ __forceinline__ void absorb_halves(const uint4 (&v)[8], const LaneCtx& k, uint32_t& ya, uint32_t& yb) {
  uint32_t xa = v[0].x, xb = v[4].x;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    word4x2(xa, v[i].y, xb, v[4 + i].y, k);
    word4x2(xa, v[i].z, xb, v[4 + i].z, k);
    word4x2(xa, v[i].w, xb, v[4 + i].w, k);
    word4x2(xa, i + 1 < 4 ? v[i + 1].x : 0u, xb, i + 1 < 4 ? v[5 + i].x : 0u, k);
  }
  ya = xa;
  yb = xb;
}

// Four 32-byte chains (v[0..1], v[2..3], v[4..5], v[6..7]), pairs joined with a uniform map at `qoff`
// (probe: the fixed-kernel image has no shift_32 table, so QOFF points at shift_64 - timing only).
__device__ __forceinline__ void absorb_halves4(const uint4 (&v)[8], const LaneCtx& k, const uint32_t* lds,
                                               uint32_t qoff, uint32_t& ya, uint32_t& yb) {
  uint32_t xa = v[0].x, xb = v[2].x, xc = v[4].x, xd = v[6].x;
#pragma unroll
  for (int i = 0; i < 2; i++) {
    word4x4(xa, v[i].y, xb, v[2 + i].y, xc, v[4 + i].y, xd, v[6 + i].y, k);
    word4x4(xa, v[i].z, xb, v[2 + i].z, xc, v[4 + i].z, xd, v[6 + i].z, k);
    word4x4(xa, v[i].w, xb, v[2 + i].w, xc, v[4 + i].w, xd, v[6 + i].w, k);
    word4x4(xa, i == 0 ? v[1].x : 0u, xb, i == 0 ? v[3].x : 0u, xc, i == 0 ? v[5].x : 0u, xd, i == 0 ? v[7].x : 0u, k);
  }
  ya = nibble_map_uniform(xa, lds, qoff) ^ xb;
  yb = nibble_map_uniform(xc, lds, qoff) ^ xd;
}

// 1 KiB payloads (stride a multiple of 16): a wave task = 8 payloads, lane l's load i reads 16 B of payload i:
// line l & 7, chunk 4 l3 + 2 l5 + l4 (lk = bit k of l). After the swaps lane l holds half l3 of line l & 7 of
// payloads 2 l5 + l4 (v[0..3]) and 4 + 2 l5 + l4 (v[4..7]); the halves meet across lane bit 3 (DPP row_ror 8),
// and lane l ends with line l & 7 of payload 4 l3 + 2 l5 + l4.
template <int NT, int SW = 1, int CH = 2, bool FAST = false, int BLK = kBlock, int VWG = kVwg>
__global__ __launch_bounds__(BLK) void k_c1nt(const uint8_t* __restrict__ base, size_t n, size_t stride,
                                              const uint4* __restrict__ img_slice, const uint4* __restrict__ img_group,
                                              uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsImageBytes / 16];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  const uint32_t l = threadIdx.x & 63, j = l & 7, l3 = (l >> 3) & 1, l4 = (l >> 4) & 1, l5 = (l >> 5) & 1;
  const uint32_t pl = 4 * l3 + 2 * l5 + l4;  // payload of this lane's final line
  const size_t gid = group_id<BLK, 8, VWG>();
  // the wave's first payload, wave-uniform (scalar address arithmetic for the loads)
  const size_t p0 = ((size_t)__builtin_amdgcn_readfirstlane((uint32_t)(gid >> 32)) << 32) |
                    (size_t)(__builtin_amdgcn_readfirstlane((uint32_t)gid) & ~7u);
  const size_t ngroups = ((size_t)gridDim.x * BLK) / 8;
  const int ntasks = p0 < n ? (int)((n - 1 - p0) / ngroups + 1) : 0;
  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;
  const uint32_t lane_off = 128 * j + 16 * (4 * l3 + 2 * l5 + l4);
  // first words of a payload (line 0, half 0) carry the init
  const uint32_t sinit = (j == 0 && l3 == 0) ? kInit : 0u;
  auto load = [&](int t, uint4 (&v)[8]) __attribute__((always_inline)) {
    const size_t pt = p0 + (size_t)t * ngroups;
    if constexpr (FAST) {  // n % 8 == 0, stride 1024: one scalar base, immediate offsets
      const uint8_t* wb = base + pt * 1024;
      const uint8_t* a0 = wb + lane_off;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const v4u32 x = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(a0 + 1024 * i));
        v[i] = make_uint4(x.x, x.y, x.z, x.w);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const size_t p = pt + i < n ? pt + i : n - 1;
      // SW == 2 (probe): load i = line i of the wave's 8 payloads, lane l chunk l & 7 of payload l >> 3
      const v4u32* a = SW == 2 ? reinterpret_cast<const v4u32*>(base + (pt + (l >> 3)) * stride + 128 * i + 16 * (l & 7))
                               : reinterpret_cast<const v4u32*>(base + p * stride + lane_off);
      v4u32 x;
      if constexpr (NT) x = __builtin_nontemporal_load(a);
      else x = *a;
      v[i] = make_uint4(x.x, x.y, x.z, x.w);
    }
  };
  uint4 A[8], B[8];
  if (ntasks > 0) load(0, A);
  load_image<kLdsImageBytes, BLK>(lds4, img_slice, img_group);
  __syncthreads();
  auto finish = [&](uint4 (&v)[8], int t) __attribute__((always_inline)) {
    if constexpr (SW == 1) {  // SW = 0 / 2: timing probes without the transpose (wrong digests)
      swap_stage<1>(v);
      swap_stage<2>(v);
    } else if constexpr (SW == 5) {  // probe: stage 2 only
      swap_stage<2>(v);
    } else if constexpr (SW == 6) {  // the stages commute: permlane32 first
      swap_stage<2>(v);
      swap_stage<1>(v);
    } else if constexpr (SW == 3) {  // probe: stage 1 only
      swap_stage<1>(v);
    } else if constexpr (SW == 4) {  // probe: 32 plain VALU ops in place of the swaps
#pragma unroll
      for (int r = 0; r < 8; r += 2) {
        v[r].x ^= v[r + 1].y; v[r].y ^= v[r + 1].z; v[r].z ^= v[r + 1].w; v[r].w ^= v[r + 1].x;
        v[r + 1].x ^= v[r].w; v[r + 1].y ^= v[r].x; v[r + 1].z ^= v[r].y; v[r + 1].w ^= v[r].z;
      }
    }
    v[0].x ^= sinit;
    v[4].x ^= sinit;
    uint32_t ya, yb;
    if constexpr (CH == 4)
      absorb_halves4(v, k, lds, kLdsHalfOff, ya, yb);
    else
      absorb_halves(v, k, ya, yb);
    const uint32_t s = l3 ? ya : yb;
    const uint32_t rcv = (uint32_t)__builtin_amdgcn_mov_dpp((int)s, 0x128, 0xF, 0xF, false);  // row_ror:8 = lane ^ 8
    const uint32_t m = l3 ? rcv : ya, x = l3 ? yb : rcv;
    const uint32_t r = nibble_map_uniform(m, lds, kLdsHalfOff) ^ x;  // raw(line) = shift_64(first half) ^ second
    const uint32_t c = group_xor_reduce<8>(nibble_map_lane(r, lds, k.slot4));
    const size_t p = p0 + (size_t)t * ngroups + pl;
    if (j == 7 && (FAST || p < n)) out[p] = ~c;
  };
  for (int t = 0; t < ntasks; t += 2) {
    ANNETY_PRIO_HI();
    load(t + 1 < ntasks ? t + 1 : t, B);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    finish(A, t);
    ANNETY_PRIO_HI();
    load(t + 2 < ntasks ? t + 2 : t, A);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    if (t + 1 < ntasks) finish(B, t + 1);
  }
}

// The product's line-per-lane shape with a per-load cache policy: bit i of NTM = load i nontemporal.
template <int NTM, int BLK = kBlock, int VWG = kVwg>
__global__ __launch_bounds__(BLK) void k_c1mask(const uint8_t* __restrict__ base, size_t n, size_t stride,
                                                const uint4* __restrict__ img_slice, const uint4* __restrict__ img_group,
                                                uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsImageBytes / 16];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  const uint32_t j = threadIdx.x & 7;
  const size_t gid = group_id<BLK, 8, VWG>();
  const size_t ngroups = ((size_t)gridDim.x * BLK) / 8;
  const int ntasks = gid < n ? (int)((n - 1 - gid) / ngroups + 1) : 0;
  const size_t pstep = ngroups * stride;
  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;
  const uint32_t sinit = j == 0 ? kInit : 0u;
  const uint8_t* lp = base + gid * stride + (size_t)j * kChunkBytes;
  uint32_t* op = out + gid;
  auto ld = [&](const uint8_t* q, uint4 (&v)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const v4u32* a = reinterpret_cast<const v4u32*>(q) + i;
      v4u32 x;
      if ((NTM >> i) & 1) x = __builtin_nontemporal_load(a);
      else x = *a;
      v[i] = make_uint4(x.x, x.y, x.z, x.w);
    }
  };
  uint4 A[8], B[8];
  if (ntasks > 0) ld(lp, A);
  load_image<kLdsImageBytes, BLK>(lds4, img_slice, img_group);
  __syncthreads();
  auto finish = [&](uint32_t s) {
    const uint32_t t = group_xor_reduce<8>(nibble_map_lane(s, lds, k.slot4));
    if (j == 7) *op = ~t;
    op += ngroups;
  };
  for (int t = 0; t < ntasks; t += 2) {
    ANNETY_PRIO_HI();
    ld(t + 1 < ntasks ? lp + pstep : lp, B);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    finish(absorb_line(sinit, A, k, lds));
    ANNETY_PRIO_HI();
    ld(t + 2 < ntasks ? lp + 2 * pstep : lp, A);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    if (t + 1 < ntasks) finish(absorb_line(sinit, B, k, lds));
    lp += 2 * pstep;
  }
}

}  // namespace

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const size_t n = argc > 1 ? strtoull(argv[1], nullptr, 0) : (1u << 20), stride = 1024, bytes = n * stride;
  std::vector<uint8_t> h(bytes);
  uint64_t s = 42;
  for (size_t i = 0; i < bytes; i++) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    h[i] = (uint8_t)(s >> 56);
  }
  uint8_t* d;
  uint32_t *o1, *o2;
  CK(hipMalloc(&d, bytes));
  CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
  CK(hipMalloc(&o1, n * 4));
  CK(hipMalloc(&o2, n * 4));
  RC(annety_crc_init(0));
  DeviceCtx* c = nullptr;
  RC(current_ctx(&c));
  RC(annety_crc32_batch_fixed(d, n, 1024, 1024, o1, nullptr));
  CK(hipDeviceSynchronize());
  // the product's own launch parameters for this shape
  const void* img_slice = c->d_slice;
  const void* img_group = group_image(*c, 8);
  const unsigned blocks = (unsigned)std::min<size_t>(grid_cus(*c), (n * 8 + kBlock - 1) / kBlock);
  auto nt1 = [&] { hipLaunchKernelGGL((k_c1nt<1>), dim3(blocks), dim3(kBlock), 0, 0, d, n, stride, (const uint4*)img_slice, (const uint4*)img_group, o2); };
  auto nt0 = [&] { hipLaunchKernelGGL((k_c1nt<0>), dim3(blocks), dim3(kBlock), 0, 0, d, n, stride, (const uint4*)img_slice, (const uint4*)img_group, o2); };
  auto nts = [&] { hipLaunchKernelGGL((k_c1nt<1, 0>), dim3(blocks), dim3(kBlock), 0, 0, d, n, stride, (const uint4*)img_slice, (const uint4*)img_group, o2); };
#define KM(M) [&] { hipLaunchKernelGGL((k_c1mask<M>), dim3(blocks), dim3(kBlock), 0, 0, d, n, stride, (const uint4*)img_slice, (const uint4*)img_group, o2); }
  auto ntc = [&] { hipLaunchKernelGGL((k_c1nt<1, 2>), dim3(blocks), dim3(kBlock), 0, 0, d, n, stride, (const uint4*)img_slice, (const uint4*)img_group, o2); };
  auto nt3 = [&] { hipLaunchKernelGGL((k_c1nt<1, 3>), dim3(blocks), dim3(kBlock), 0, 0, d, n, stride, (const uint4*)img_slice, (const uint4*)img_group, o2); };
  auto nt4 = [&] { hipLaunchKernelGGL((k_c1nt<1, 4>), dim3(blocks), dim3(kBlock), 0, 0, d, n, stride, (const uint4*)img_slice, (const uint4*)img_group, o2); };
  auto nt5 = [&] { hipLaunchKernelGGL((k_c1nt<1, 5>), dim3(blocks), dim3(kBlock), 0, 0, d, n, stride, (const uint4*)img_slice, (const uint4*)img_group, o2); };
  auto nt6 = [&] { hipLaunchKernelGGL((k_c1nt<1, 6>), dim3(blocks), dim3(kBlock), 0, 0, d, n, stride, (const uint4*)img_slice, (const uint4*)img_group, o2); };
  auto nt1c4 = [&] { hipLaunchKernelGGL((k_c1nt<1, 1, 4>), dim3(blocks), dim3(kBlock), 0, 0, d, n, stride, (const uint4*)img_slice, (const uint4*)img_group, o2); };
  auto nt0c4 = [&] { hipLaunchKernelGGL((k_c1nt<1, 0, 4>), dim3(blocks), dim3(kBlock), 0, 0, d, n, stride, (const uint4*)img_slice, (const uint4*)img_group, o2); };
  auto ntf = [&] { hipLaunchKernelGGL((k_c1nt<1, 1, 2, true>), dim3(blocks), dim3(kBlock), 0, 0, d, n, stride, (const uint4*)img_slice, (const uint4*)img_group, o2); };
  auto prod = [&] { RC(annety_crc32_batch_fixed(d, n, 1024, 1024, o1, nullptr)); };
  CK(hipMemset(o2, 0, n * 4));
  nt1();
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> r1(n), r2(n);
  CK(hipMemcpy(r1.data(), o1, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r2.data(), o2, n * 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < n; i++) bad += r1[i] != r2[i];
  printf("n=%zu blocks=%u mismatches=%zu first: %08x %08x\n", n, blocks, bad, r1[0], r2[0]);
  if (bad) return 2;
  CK(hipMemset(o2, 0, n * 4));
  nt6();
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(r2.data(), o2, n * 4, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < n; i++) bad += r1[i] != r2[i];
  printf("permlane32-first order: mismatches=%zu\n", bad);
  if (bad) return 2;
  if (n % 8 == 0) {
    CK(hipMemset(o2, 0, n * 4));
    ntf();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(r2.data(), o2, n * 4, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; i++) bad += r1[i] != r2[i];
    printf("fast addressing: mismatches=%zu\n", bad);
    if (bad) return 2;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto t = [&](auto f, const char* name) {
    for (int w = 0; w < 100; w++) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 200; r++) f();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipGetLastError());
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-40s %.1f us  %.0f GB/s  %.1f %% of 8 TB/s (algorithmic)\n", name, ms * 5, bytes / (ms / 200) / 1e6,
           (bytes + n * 4) / (ms / 200) / 1e6 / 80);
  };
  for (int rep = 0; rep < 3; rep++) {
    t(prod, "product config-1 kernel");
    t(nt1, "coalesced nt + swaps");
    t(nt0, "coalesced default policy + swaps");
    t(nts, "coalesced nt, no swaps (wrong digests)");
    t(ntf, "coalesced nt + swaps, fast addressing");
  }
  return 0;
}
