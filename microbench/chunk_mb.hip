// DRAM granularity probe for the length-sorted path: 1 GiB read by 2048 waves (256 x 512
// lanes), 8 coalesced nontemporal 1 KiB loads per wave step (the product kernels' shape), the bytes split into
// streams that lane groups walk C KiB per step. C = 8: a wave walks one stream 8 KiB per step; C = 1: each of a
// wave's 8 groups walks its own stream 1 KiB per step (var_class_w8's access pattern). Streams sit at permuted
// places of the buffer. "window": the config-1 pattern (wave w, step s reads 8 KiB block s * 2048 + w).
// FAKE adds that many dependent VALU ops per step (the fold's issue time, roughly). Pure reads, no checksum.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 microbench/chunk_mb.hip -o microbench/chunk_mb
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__);                  \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
constexpr int kBlock = 512, kBlocks = 256, kWaves = kBlocks * kBlock / 64;
constexpr size_t kBytes = 1ull << 30;

// C = chunk KiB per group per step (1, 2, 4, 8); WINDOW = config-1 pattern
template <int C, bool WINDOW, int FAKE, int MIS = 0>
__global__ __launch_bounds__(kBlock) void k_chunk(const uint8_t* __restrict__ base, const uint32_t* __restrict__ perm,
                                                  uint32_t* __restrict__ out) {
  const uint32_t l = threadIdx.x & 63;
  const uint32_t w = blockIdx.x + kBlocks * (threadIdx.x >> 6);  // wave id, blocks interleaved
  constexpr int NG = 8 / C;                                        // groups (streams) per wave
  constexpr size_t kStreams = (size_t)kWaves * NG;
  constexpr size_t kStreamBytes = kBytes / kStreams;
  constexpr int kSteps = (int)(kBytes / ((size_t)kWaves * 8192));
  const uint32_t lane_off = 16 * l;  // 64 lanes x 16 B = 1 KiB per load
  uint32_t acc = 0;
  for (int s = 0; s < kSteps; s++) {
    v4u32 v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      size_t a;
      if constexpr (WINDOW) {
        a = ((size_t)s * kWaves + w) * 8192 + 1024 * i;
      } else {
        const int g = i / C, piece = i % C;  // load i: piece `piece` of group g's chunk
        const size_t stream = (size_t)perm[w * NG + g];
        // MIS: every stream starts MIS bytes past its 64 KiB-aligned place (the sorted path's rounds start at any
        // 128-byte line); the buffer has 4 KiB of slack past kBytes for the last stream's tail
        a = stream * kStreamBytes + MIS + (size_t)s * 1024 * C + 1024 * piece;
      }
      v[i] = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(base + a + lane_off));
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
#pragma unroll
    for (int f = 0; f < FAKE; f++) x = __builtin_amdgcn_perm(x, acc, 0x05040706u) + f;
    acc ^= x;
  }
  out[blockIdx.x * kBlock + threadIdx.x] = acc;
}

template <int C, bool WINDOW, int FAKE, int MIS = 0>
int run(const uint8_t* d, const uint32_t* perm, uint32_t* out, const char* name) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 5; i++) k_chunk<C, WINDOW, FAKE, MIS><<<kBlocks, kBlock>>>(d, perm, out);
  CK(hipEventRecord(e0));
  const int reps = 50;
  for (int i = 0; i < reps; i++) k_chunk<C, WINDOW, FAKE, MIS><<<kBlocks, kBlock>>>(d, perm, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  printf("%-10s C=%d fake=%3d mis=%3d  %.4f ms  %.1f GB/s\n", name, C, FAKE, MIS, ms, kBytes / (ms * 1e-3) / 1e9);
  return 0;
}

int main() {
  uint8_t* d = nullptr;
  uint32_t *perm = nullptr, *out = nullptr;
  CK(hipMalloc(&d, kBytes + 4096));  // slack: a misaligned stream's last piece reads up to 1 KiB past kBytes
  CK(hipMemset(d, 1, kBytes + 4096));
  CK(hipMalloc(&out, kBlocks * kBlock * 4));
  const size_t maxs = (size_t)kWaves * 8;
  CK(hipMalloc(&perm, maxs * 4));
  for (int rep = 0; rep < 2; rep++) {
    for (int c : {1, 2, 4, 8}) {
      const size_t ns = (size_t)kWaves * (8 / c);
      std::vector<uint32_t> p(ns);
      for (size_t k = 0; k < ns; k++) p[k] = (uint32_t)k;
      uint64_t x = 88172645463325252ull;
      for (size_t k = ns - 1; k > 0; k--) {  // Fisher-Yates, xorshift
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        std::swap(p[k], p[x % (k + 1)]);
      }
      CK(hipMemcpy(perm, p.data(), ns * 4, hipMemcpyHostToDevice));
      if (c == 1) {
        run<1, false, 0>(d, perm, out, "streams");
        run<1, false, 200>(d, perm, out, "streams");
        run<1, false, 0, 128>(d, perm, out, "streams");
        run<1, false, 0, 384>(d, perm, out, "streams");
        run<1, false, 0, 640>(d, perm, out, "streams");
        run<1, false, 0, 512>(d, perm, out, "streams");
      } else if (c == 2) {
        run<2, false, 0>(d, perm, out, "streams");
        run<2, false, 200>(d, perm, out, "streams");
      } else if (c == 4) {
        run<4, false, 0>(d, perm, out, "streams");
        run<4, false, 200>(d, perm, out, "streams");
      } else {
        run<8, false, 0>(d, perm, out, "streams");
        run<8, false, 200>(d, perm, out, "streams");
      }
    }
    run<8, true, 0>(d, perm, out, "window");
    run<8, true, 200>(d, perm, out, "window");
  }
  return 0;
}
