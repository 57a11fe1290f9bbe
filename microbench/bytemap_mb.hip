// Half-line join of crc32_onekib_nt_kernel through byte tables (4 lookups of a compact 4 KiB table,
// 2 VALU per address) or through the nibble map (8 lookups, conflict-free): fewer VALU per task against
// 3-4-way LDS bank conflicts. The product kernel uses the byte tables (since this A/B); the microbench
// kernel here is the nibble-map form (NIBBLE = 1) or a byte-table copy (0). Checks every digest against
// the product kernel and times both.
// Build (repo root): hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Iannety_amd/csrc microbench/bytemap_mb.hip -o microbench/bytemap_mb -L/opt/rocm/lib -lrccl
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
constexpr uint32_t kByteMapOff = kLdsImageBytes;  // 4 tables x 256 words

__device__ __forceinline__ uint32_t byte_map(uint32_t x, const uint32_t* lds) {
  const uint32_t* t = lds + kByteMapOff / 4;
  return xor3(t[x & 255], t[256 + ((x >> 8) & 255)], t[512 + ((x >> 16) & 255)]) ^ t[768 + (x >> 24)];
}

template <int NIBBLE, int BLK = kBlock, int VWG = kVwg>
__global__ __launch_bounds__(BLK) void k_bytemap(const uint8_t* __restrict__ base, size_t n,
                                                 const uint4* __restrict__ img_slice,
                                                 const uint4* __restrict__ img_group, const uint32_t* __restrict__ bm,
                                                 uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[(kLdsImageBytes + 4096) / 16];
  uint32_t* ldsw = reinterpret_cast<uint32_t*>(lds4);
  const uint32_t* lds = ldsw;
  const uint32_t l = threadIdx.x & 63, j = l & 7, l3 = (l >> 3) & 1;
  const size_t gid = group_id<BLK, 8, VWG>();
  const size_t p0 = ((size_t)__builtin_amdgcn_readfirstlane((uint32_t)(gid >> 32)) << 32) |
                    (size_t)(__builtin_amdgcn_readfirstlane((uint32_t)gid) & ~7u);
  const size_t ngroups = ((size_t)gridDim.x * BLK) / 8;
  const int ntasks = p0 < n ? (int)((n - 1 - p0) / ngroups + 1) : 0;
  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;
  const uint32_t lane_off = coalesced_lane_offset(l);
  const uint32_t sinit = (j == 0 && l3 == 0) ? kInit : 0u;
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
  load_image<kLdsImageBytes, BLK>(lds4, img_slice, img_group);
  for (uint32_t i = threadIdx.x; i < 1024; i += BLK) ldsw[kByteMapOff / 4 + i] = bm[i];
  __syncthreads();
  auto finish = [&](uint4 (&v)[8]) __attribute__((always_inline)) {
    transpose_blocks(v);
    v[0].x ^= sinit;
    v[4].x ^= sinit;
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
    const uint32_t r = (NIBBLE ? nibble_map_uniform(first, lds, kLdsHalfOff) : byte_map(first, lds)) ^ second;
    const uint32_t c = group_xor_reduce<8>(nibble_map_lane(r, lds, k.slot4));
    if (j == 7) *op = ~c;
    op += ngroups;
  };
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
}  // namespace

int main() {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const size_t n = 1u << 20, bytes = n * 1024;
  std::vector<uint8_t> h(bytes);
  uint64_t s = 42;
  for (size_t i = 0; i < bytes; i++) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    h[i] = (uint8_t)(s >> 56);
  }
  uint8_t* d;
  uint32_t *o1, *o2, *bm;
  CK(hipMalloc(&d, bytes));
  CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
  CK(hipMalloc(&o1, n * 4));
  CK(hipMalloc(&o2, n * 4));
  CK(hipMalloc(&bm, 4096));
  std::vector<uint32_t> hb(1024);
  const Gf2Mat m = shift_matrix(64);
  for (uint32_t k = 0; k < 4; k++)
    for (uint32_t e = 0; e < 256; e++) hb[k * 256 + e] = gf2_apply(m, e << (8 * k));
  CK(hipMemcpy(bm, hb.data(), 4096, hipMemcpyHostToDevice));
  RC(annety_crc_init(0));
  DeviceCtx* c = nullptr;
  RC(current_ctx(&c));
  const void* img_slice = c->d_slice;
  const void* img_group = group_image(*c, 8);
  const unsigned blocks = (unsigned)std::min<size_t>(grid_cus(*c), (n * 8 + kBlock - 1) / kBlock);
  auto prod = [&] { RC(annety_crc32_batch_fixed(d, n, 1024, 1024, o1, nullptr)); };
  auto nbk = [&] { hipLaunchKernelGGL((k_bytemap<1>), dim3(blocks), dim3(kBlock), 0, 0, d, n, (const uint4*)img_slice, (const uint4*)img_group, (const uint32_t*)bm, o2); };
  auto bmk = [&] { hipLaunchKernelGGL((k_bytemap<0>), dim3(blocks), dim3(kBlock), 0, 0, d, n, (const uint4*)img_slice, (const uint4*)img_group, (const uint32_t*)bm, o2); };
  prod();
  nbk();
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> r1(n), r2(n);
  CK(hipMemcpy(r1.data(), o1, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(r2.data(), o2, n * 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < n; i++) bad += r1[i] != r2[i];
  printf("mismatches=%zu\n", bad);
  if (bad) return 2;
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
    printf("%-44s %.1f us  %.1f %% of 8 TB/s (algorithmic)\n", name, ms * 5, (bytes + n * 4) / (ms / 200) / 1e6 / 80);
  };
  for (int rep = 0; rep < 3; rep++) {
    t(prod, "product (byte-table half-join map)");
    t(nbk, "nibble half-join map (round-3 kernel)");
    t(bmk, "byte-table half-join map (microbench copy)");
  }
  return 0;
}
