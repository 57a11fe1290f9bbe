// A/B of product kernel variants on the headline workload (1M x 1 KiB): virtual-workgroup mapping of
// the single-round kernel (kVwg). Includes the product source directly.
#include "../annety_amd/csrc/crc32_kernels.hip"
#include "../annety_amd/csrc/crc32_frames.hip"
#include "../annety_amd/csrc/crc32_host.cpp"
#include "../annety_amd/csrc/crc32_capi.cpp"
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__global__ void fill_kernel(uint4* p, size_t n16, uint64_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    x ^= x >> 31; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 27; x *= 0x94D049BB133111EBull; x ^= x >> 33;
    uint64_t y = x * 0xD6E8FEB86659FD93ull; y ^= y >> 32;
    p[i] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)y, (uint32_t)(y >> 32));
  }
}

int main() {
  using namespace annety_crc;
  const size_t n = 1u << 20, L = 1024, bytes = n * L;
  uint4* d; uint32_t *out, *ref;
  CK(hipMalloc(&d, bytes)); CK(hipMalloc(&out, n * 4)); CK(hipMalloc(&ref, n * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, d, bytes / 16, 0x1234ull);
  CK(hipDeviceSynchronize());
  if (annety_crc32_batch_fixed(d, n, L, L, ref, nullptr)) return 1;
  DeviceCtx* c = nullptr;
  if (current_ctx(&c)) return 1;
  const void* gimg = group_image(*c, 8);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<uint32_t> h1(n), h2(n);
  auto b2b = [&](auto launch, const char* name) {
    for (int w = 0; w < 20; w++) launch();
    CK(hipEventRecord(e0));
    for (int r = 0; r < 100; r++) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(h1.data(), out, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), ref, n * 4, hipMemcpyDeviceToHost));
    printf("%-34s %.4f ms/launch  %.1f GB/s  %s\n", name, ms / 100, (bytes + 4.0 * n) / (ms / 100) / 1e6, h1 == h2 ? "ok" : "MISMATCH");
  };
  // clocks up
  for (int r = 0; r < 2000; r++) annety_crc32_batch_fixed(d, n, L, L, out, nullptr);
  for (int rep = 0; rep < 3; rep++) {
    b2b([&] { annety_crc32_batch_fixed(d, n, L, L, out, nullptr); }, "product (oneround<8,512>)");
    b2b([&] { hipLaunchKernelGGL((crc32_oneround_kernel<8, 512, 0>), dim3(256), dim3(512), 0, 0, (const uint8_t*)d, n, (size_t)L, (const uint4*)c->d_slice, (const uint4*)gimg, out); }, "oneround<8,512> vwg off");
    b2b([&] { hipLaunchKernelGGL((crc32_oneround_kernel<8, 512, 256>), dim3(256), dim3(512), 0, 0, (const uint8_t*)d, n, (size_t)L, (const uint4*)c->d_slice, (const uint4*)gimg, out); }, "oneround<8,512> vwg 256");
    b2b([&] { hipLaunchKernelGGL((crc32_oneround_kernel<8, 512, 128>), dim3(256), dim3(512), 0, 0, (const uint8_t*)d, n, (size_t)L, (const uint4*)c->d_slice, (const uint4*)gimg, out); }, "oneround<8,512> vwg 128");
    b2b([&] { hipLaunchKernelGGL((crc32_oneround_kernel<8, 512, 64>), dim3(256), dim3(512), 0, 0, (const uint8_t*)d, n, (size_t)L, (const uint4*)c->d_slice, (const uint4*)gimg, out); }, "oneround<8,512> vwg 64");
  }
  return 0;
}
