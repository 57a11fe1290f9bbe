// Config-1 kernel (crc32_oneround_kernel<8>) at 256 / 384 / 512 / 768 / 1024 lanes per workgroup: one workgroup per
// CU either way (the LDS image), so the block size sets the waves per SIMD (1 / 1.5 / 2 / 3 / 4) and the bytes in
// flight per CU. Digests are compared with the product launch (512 lanes).
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

int main() {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const size_t n = 1 << 20, L = 1024, bytes = n * L;
  std::vector<uint8_t> h(bytes);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < bytes; i++) { x = x * 6364136223846793005ull + 1442695040888963407ull; h[i] = (uint8_t)(x >> 56); }
  uint8_t* d; uint32_t *ref, *out;
  CK(hipMalloc(&d, bytes)); CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
  CK(hipMalloc(&ref, n * 4)); CK(hipMalloc(&out, n * 4));
  RC(annety_crc_init(0));
  DeviceCtx* c = nullptr; RC(current_ctx(&c));
  RC(annety_crc32_batch_fixed(d, n, L, L, ref, nullptr));
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> r0(n), r1(n);
  CK(hipMemcpy(r0.data(), ref, n * 4, hipMemcpyDeviceToHost));
  const unsigned grid = (unsigned)grid_cus(*c);
  const uint4* slice = static_cast<const uint4*>(c->d_slice);
  const uint4* grp = static_cast<const uint4*>(group_image(*c, 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto t = [&](auto f, const char* name) {
    CK(hipMemset(out, 0, n * 4));
    f(); CK(hipDeviceSynchronize());
    CK(hipMemcpy(r1.data(), out, n * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < n; i++) bad += r0[i] != r1[i];
    for (int w = 0; w < 200; w++) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 200; r++) f();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipGetLastError());
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-28s %.4f ms  %.1f GB/s  (%zu digests differ)\n", name, ms / 200, (bytes + 4 * n) / (ms / 200) / 1e6, bad);
  };
  t([&] { hipLaunchKernelGGL((crc32_oneround_kernel<8, 512, 256>), dim3(grid), dim3(512), 0, 0, d, n, L, slice, grp, out); }, "512 lanes (product)");
  t([&] { hipLaunchKernelGGL((crc32_oneround_kernel<8, 768, 256>), dim3(grid), dim3(768), 0, 0, d, n, L, slice, grp, out); }, "768 lanes");
  t([&] { hipLaunchKernelGGL((crc32_oneround_kernel<8, 1024, 256>), dim3(grid), dim3(1024), 0, 0, d, n, L, slice, grp, out); }, "1024 lanes");
  t([&] { hipLaunchKernelGGL((crc32_oneround_kernel<8, 256, 0>), dim3(grid), dim3(256), 0, 0, d, n, L, slice, grp, out); }, "256 lanes");
  t([&] { hipLaunchKernelGGL((crc32_oneround_kernel<8, 384, 128>), dim3(grid), dim3(384), 0, 0, d, n, L, slice, grp, out); }, "384 lanes");
  t([&] { hipLaunchKernelGGL((crc32_oneround_kernel<8, 512, 0>), dim3(grid), dim3(512), 0, 0, d, n, L, slice, grp, out); }, "512 lanes, no virtual groups");
  t([&] { hipLaunchKernelGGL((crc32_oneround_kernel<8, 512, 128>), dim3(grid), dim3(512), 0, 0, d, n, L, slice, grp, out); }, "512 lanes, 4 virtual groups");
  t([&] { hipLaunchKernelGGL((crc32_oneround_kernel<8, 512, 256>), dim3(grid), dim3(512), 0, 0, d, n, L, slice, grp, out); }, "512 lanes (product, again)");
  return 0;
}
