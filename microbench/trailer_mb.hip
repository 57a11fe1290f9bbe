// What does the second launch of a split encode pay for its trailers? After a kernel has written a 1.1 GB frame
// stream (and the stream has left the caches), a kernel stores 4 bytes at each of 2M frame ends (every ~530 bytes,
// unaligned): partial-line writes into lines the first kernel wrote long before. Against the same stores into a
// buffer nothing else wrote, and the 8-byte (trailer + next header) form.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void fill(uint4* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
template <int W>
__global__ void trailers(uint8_t* base, const uint64_t* __restrict__ end, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint64_t e = end[i];
    if (W == 4) *(__attribute__((address_space(1))) uint32_t*)(base + e) = (uint32_t)i;
    else *(__attribute__((address_space(1))) uint64_t*)(base + e) = i;
  }
}

int main() {
  const size_t n = 2 << 20;
  std::vector<uint64_t> end(n);
  uint64_t pos = 0, seed = 7;
  for (size_t i = 0; i < n; i++) {
    seed = seed * 6364136223846793005ull + 1442695040888963407ull;
    pos += 4 + 16 + (seed >> 33) % 1009;  // header + payload of 16 B - 1 KiB
    end[i] = pos;
    pos += 4;
  }
  const size_t bytes = (pos + 64) & ~15ull;
  uint8_t *a, *b;
  uint64_t* dend;
  CK(hipMalloc(&a, bytes)); CK(hipMalloc(&b, bytes)); CK(hipMalloc(&dend, n * 8));
  CK(hipMemcpy(dend, end.data(), n * 8, hipMemcpyHostToDevice));
  int dev, cus; CK(hipGetDevice(&dev)); CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  hipEvent_t e0, e1, e2; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
  for (int rep = 0; rep < 3; rep++) {
    for (int w : {4, 8}) {
      float t_fill = 0, t_tr = 0, t_cold = 0;
      for (int it = 0; it < 20; it++) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(fill, dim3(cus * 8), dim3(256), 0, 0, (uint4*)a, bytes / 16);
        CK(hipEventRecord(e1));
        if (w == 4) hipLaunchKernelGGL(trailers<4>, dim3(cus * 8), dim3(256), 0, 0, a, dend, n);
        else hipLaunchKernelGGL(trailers<8>, dim3(cus * 8), dim3(256), 0, 0, a, dend, n);
        CK(hipEventRecord(e2)); CK(hipEventSynchronize(e2));
        float x, y; CK(hipEventElapsedTime(&x, e0, e1)); CK(hipEventElapsedTime(&y, e1, e2));
        if (it >= 5) { t_fill += x; t_tr += y; }
        // the same stores into b, which nothing else wrote (lines not dirty anywhere)
        CK(hipEventRecord(e1));
        if (w == 4) hipLaunchKernelGGL(trailers<4>, dim3(cus * 8), dim3(256), 0, 0, b, dend, n);
        else hipLaunchKernelGGL(trailers<8>, dim3(cus * 8), dim3(256), 0, 0, b, dend, n);
        CK(hipEventRecord(e2)); CK(hipEventSynchronize(e2));
        CK(hipEventElapsedTime(&y, e1, e2));
        if (it >= 5) t_cold += y;
      }
      printf("%d-byte stores at 2M frame ends: after a %.1f ms fill of the stream %.1f us; into an untouched buffer %.1f us\n",
             w, t_fill / 15, t_tr / 15 * 1000, t_cold / 15 * 1000);
    }
  }
  return 0;
}
