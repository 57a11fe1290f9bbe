// What the variable-length kernel's byte masks and unshift cost: the product var kernel vs PROBE
// variants with those stages removed, on aligned fixed-size batches run through the var path
// (direct mode) and through the fixed kernel for reference. Digests of PROBE variants are wrong by
// design; only the product line is checked.
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
    p[i] = make_uint4((uint32_t)x, (uint32_t)(x >> 32), (uint32_t)(x * 3), (uint32_t)(x >> 7));
  }
}

using namespace annety_crc;

template <int G, int PROBE>
void launch_probe(DeviceCtx& c, const void* d, size_t n, uint32_t L, uint32_t* out) {
  const size_t blocks = std::min<size_t>(256, (n * G + kBlock - 1) / kBlock);
  hipLaunchKernelGGL((crc32_var_kernel<G, false, false, kVwg, PROBE>), dim3((unsigned)blocks), dim3(kBlock), 0, 0,
                     (const uint8_t*)d, n, (uint64_t)L, L, (const uint4*)nullptr, (const uint32_t*)nullptr,
                     (const uint4*)c.d_slice, (const uint4*)group_image(c, G), (const uint4*)c.d_unshift, out);
}

int main() {
  const size_t bytes = 1ull << 30;
  uint4* d; uint32_t *out, *ref;
  CK(hipMalloc(&d, bytes + 4096)); CK(hipMalloc(&out, (1u << 20) * 4)); CK(hipMalloc(&ref, (1u << 20) * 4));
  hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, d, (bytes + 4096) / 16, 0x1234ull);
  CK(hipDeviceSynchronize());
  DeviceCtx* c = nullptr;
  if (annety_crc_init(0) || current_ctx(&c)) return 1;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int r = 0; r < 3000; r++) annety_crc32_batch_fixed(d, 1u << 20, 1024, 1024, out, nullptr);  // clocks up
  auto b2b = [&](auto launch, const char* name, size_t n, bool check) {
    for (int w = 0; w < 10; w++) launch();
    CK(hipEventRecord(e0));
    for (int r = 0; r < 50; r++) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    bool ok = true;
    if (check) {
      std::vector<uint32_t> h1(n), h2(n);
      CK(hipMemcpy(h1.data(), out, n * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2.data(), ref, n * 4, hipMemcpyDeviceToHost));
      ok = h1 == h2;
    }
    printf("%-44s %.4f ms  %.1f GB/s %s\n", name, ms / 50, bytes / (ms / 50) / 1e6, check ? (ok ? "ok" : "MISMATCH") : "");
  };
  for (uint32_t L : {4096u, 16384u, 65536u}) {
    const size_t n = bytes / L;
    printf("-- L=%u n=%zu (+3-byte offset for the var lines)\n", L, n);
    const void* d3 = (const char*)d + 3;
    if (annety_crc32_batch_fixed(d, n, L, L, ref, nullptr)) return 1;
    b2b([&] { annety_crc32_batch_fixed(d, n, L, L, out, nullptr); }, "fixed (product)", n, true);
    CK(hipDeviceSynchronize());
    const uint32_t G = L >= 16384 ? 32 : 8;
    std::vector<uint32_t> dummy;
    if (G == 32) {
      b2b([&] { launch_probe<32, 0>(*c, d, n, L, out); }, "var<32> aligned", n, true);
      b2b([&] { launch_probe<32, 0>(*c, d3, n, L, out); }, "var<32> +3", n, false);
      b2b([&] { launch_probe<32, 1>(*c, d3, n, L, out); }, "var<32> +3 no masks", n, false);
      b2b([&] { launch_probe<32, 3>(*c, d3, n, L, out); }, "var<32> +3 no masks no unshift", n, false);
    } else {
      b2b([&] { launch_probe<8, 0>(*c, d, n, L, out); }, "var<8> aligned", n, true);
      b2b([&] { launch_probe<8, 0>(*c, d3, n, L, out); }, "var<8> +3", n, false);
      b2b([&] { launch_probe<8, 1>(*c, d3, n, L, out); }, "var<8> +3 no masks", n, false);
      b2b([&] { launch_probe<8, 3>(*c, d3, n, L, out); }, "var<8> +3 no masks no unshift", n, false);
    }
  }
  return 0;
}
