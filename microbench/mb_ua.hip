// Can the variable-length kernel read payload-relative (byte-unaligned) 128-byte lines?
// Streams 1 GiB as lane-per-line 8 x global_load_dwordx4 at base + off (off = 0..16), vs aligned
// loads + one extra block + v_alignbyte funnel (the register-side alternative).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1;} } while (0)

typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ v4u32 gl16(uint64_t a) { return *(const __attribute__((address_space(1))) v4u32*)a; }
__device__ __forceinline__ uint32_t gl4(uint64_t a) { return *(const __attribute__((address_space(1))) uint32_t*)a; }

__global__ __launch_bounds__(512) void k_ua(uint64_t base, size_t lines, uint32_t* out) {
  const size_t t = blockIdx.x * (size_t)512 + threadIdx.x, T = (size_t)gridDim.x * 512;
  uint32_t acc = 0;
  for (size_t l = t; l < lines; l += T) {
    const uint64_t a = base + (l << 7);
    v4u32 v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = gl16(a + 16 * i);
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  }
  out[t] = acc;
}

// aligned loads of the 9 blocks covering [a, a+128), funnel-shifted into the 8 payload-relative blocks
__global__ __launch_bounds__(512) void k_funnel(uint64_t base, size_t lines, uint32_t* out) {
  const size_t t = blockIdx.x * (size_t)512 + threadIdx.x, T = (size_t)gridDim.x * 512;
  uint32_t acc = 0;
  for (size_t l = t; l < lines; l += T) {
    const uint64_t a = base + (l << 7);
    const uint64_t al = a & ~15ull;
    const uint32_t sh = (uint32_t)(a & 15);
    v4u32 v[9];
#pragma unroll
    for (int i = 0; i < 9; i++) v[i] = gl16(al + 16 * i);
    uint32_t w[36];
#pragma unroll
    for (int i = 0; i < 9; i++) { w[4 * i] = v[i].x; w[4 * i + 1] = v[i].y; w[4 * i + 2] = v[i].z; w[4 * i + 3] = v[i].w; }
    const uint32_t dw = sh >> 2, bs = sh & 3;
#pragma unroll
    for (int q = 0; q < 32; q++) {
      // word q of the line = bytes [a + 4q, a + 4q + 4): dword index q + dw (+1), byte shift bs
      const uint32_t lo = dw == 0 ? w[q] : dw == 1 ? w[q + 1] : dw == 2 ? w[q + 2] : w[q + 3];
      const uint32_t hi = dw == 0 ? w[q + 1] : dw == 1 ? w[q + 2] : dw == 2 ? w[q + 3] : w[q + 4];
      acc ^= __builtin_amdgcn_alignbyte(hi, lo, bs);
    }
  }
  out[t] = acc;
}

int main() {
  const size_t bytes = 1ull << 30, lines = bytes / 128 - 1;
  char* d; uint32_t* out;
  CK(hipMalloc(&d, bytes + 4096)); CK(hipMalloc(&out, 256 * 512 * 4));
  CK(hipMemset(d, 1, bytes + 4096));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const uint64_t b = (uint64_t)(uintptr_t)d;
  for (int w = 0; w < 2000; w++) hipLaunchKernelGGL(k_ua, dim3(256), dim3(512), 0, 0, b, lines, out);
  auto run = [&](const char* name, int kind, uint32_t off) -> int {
    for (int w = 0; w < 5; w++) {
      if (kind == 0) hipLaunchKernelGGL(k_ua, dim3(256), dim3(512), 0, 0, b + off, lines, out);
      else hipLaunchKernelGGL(k_funnel, dim3(256), dim3(512), 0, 0, b + off, lines, out);
    }
    CK(hipEventRecord(e0));
    for (int r = 0; r < 50; r++) {
      if (kind == 0) hipLaunchKernelGGL(k_ua, dim3(256), dim3(512), 0, 0, b + off, lines, out);
      else hipLaunchKernelGGL(k_funnel, dim3(256), dim3(512), 0, 0, b + off, lines, out);
    }
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipGetLastError());
    printf("%-10s off=%2u  %.4f ms  %.1f GB/s\n", name, off, ms / 50, lines * 128.0 / (ms / 50) / 1e6);
    return 0;
  };
  for (int rep = 0; rep < 2; rep++)
    for (uint32_t off : {0u, 1u, 3u, 4u, 8u, 16u, 64u}) {
      if (run("unaligned", 0, off)) return 1;
      if (run("funnel", 1, off)) return 1;
    }
  return 0;
}
