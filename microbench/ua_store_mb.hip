// Unaligned 16-byte global stores (the fused encode's copy: a payload's bytes move by a byte shift that is one per
// frame): every lane stores the uint4 it loaded from src + 16 t to dst + 16 t + delta, delta = 0..15 bytes. Checks
// the copy byte for byte and times it against delta = 0 (256 MiB per launch).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 microbench/ua_store_mb.hip -o microbench/ua_store_mb
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                      \
  do {                                                             \
    hipError_t e_ = (x);                                           \
    if (e_ != hipSuccess) {                                        \
      printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                    \
    }                                                              \
  } while (0)

typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
constexpr size_t kBytes = 256ull << 20;

__global__ __launch_bounds__(256) void k_copy(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint32_t delta) {
  const size_t n = kBytes / 16;
  for (size_t t = blockIdx.x * (size_t)256 + threadIdx.x; t < n; t += (size_t)gridDim.x * 256) {
    const v4u32 x = __builtin_nontemporal_load(reinterpret_cast<const v4u32*>(src + 16 * t));
    *reinterpret_cast<v4u32*>(dst + 16 * t + delta) = x;
  }
}

int main() {
  uint8_t *src = nullptr, *dst = nullptr;
  CK(hipMalloc(&src, kBytes));
  CK(hipMalloc(&dst, kBytes + 64));
  std::vector<uint8_t> h(kBytes);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < kBytes; i += 8) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    std::memcpy(&h[i], &x, 8);
  }
  CK(hipMemcpy(src, h.data(), kBytes, hipMemcpyHostToDevice));
  std::vector<uint8_t> back(kBytes + 64);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (uint32_t delta : {0u, 1u, 2u, 3u, 4u, 5u, 8u, 12u, 15u}) {
    CK(hipMemset(dst, 0xAB, kBytes + 64));
    k_copy<<<4096, 256>>>(src, dst, delta);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(back.data(), dst, kBytes + 64, hipMemcpyDeviceToHost));
    const bool ok = std::memcmp(back.data() + delta, h.data(), kBytes) == 0 && (delta == 0 || back[0] == 0xAB);
    for (int i = 0; i < 3; i++) k_copy<<<4096, 256>>>(src, dst, delta);
    CK(hipEventRecord(e0));
    const int reps = 20;
    for (int i = 0; i < reps; i++) k_copy<<<4096, 256>>>(src, dst, delta);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("delta %2u  %s  %.4f ms  %.1f GB/s (read + write)\n", delta, ok ? "exact" : "MISMATCH", ms,
           2.0 * kBytes / (ms * 1e-3) / 1e9);
  }
  return 0;
}
