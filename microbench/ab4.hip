// Config-3 (Zipf 64 B-64 KiB, packed unaligned, ~1 GiB) breakdown of the sorted variable path:
// bucket passes alone, each length class alone, and the classes without byte masks / unshift
// (PROBE variants: wrong digests by design, timing only).
#include "../annety_amd/csrc/crc32_kernels.hip"
#include "../annety_amd/csrc/crc32_arena.hip"
#include "../annety_amd/csrc/crc32_frames.hip"
#include "../annety_amd/csrc/crc32_host.cpp"
#include "../annety_amd/csrc/crc32_capi.cpp"
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

using namespace annety_crc;

// Every stage is synchronised and checked (stage name on stdout, line-buffered) so a failure names
// the stage that caused it.
#define STAGE(name)                                                                        \
  do {                                                                                     \
    hipError_t e_ = hipDeviceSynchronize();                                                \
    if (e_ == hipSuccess) e_ = hipGetLastError();                                          \
    printf("stage %-28s %s\n", name, e_ == hipSuccess ? "ok" : hipGetErrorString(e_));     \
    if (e_ != hipSuccess) exit(2);                                                         \
  } while (0)
#define RC(x) do { int r_ = (x); if (r_) { printf("%s -> %d (%s)\n", #x, r_, annety_crc_strerror(r_)); exit(3); } } while (0)

template <int G, int PROBE>
void launch_cls(DeviceCtx& c, const void* base, size_t n, const void* desc, const uint32_t* range, uint32_t* out) {
  hipLaunchKernelGGL((crc32_var_kernel<G, true, false, kVwg, PROBE>), dim3(c.cus), dim3(kBlock), 0, 0,
                     (const uint8_t*)base, n, (uint64_t)0, 0u, (const uint4*)desc, range, (const uint4*)c.d_slice,
                     (const uint4*)group_image(c, G), (const uint4*)c.d_unshift, out);
}

int main() {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  // SURVEY.md §8d config 3 lengths
  std::mt19937_64 rng(0x5EED);
  std::vector<double> cdf(1024);
  double acc = 0;
  for (int k = 1; k <= 1024; k++) cdf[k - 1] = (acc += std::pow((double)k, -1.1));
  std::vector<uint32_t> lens;
  std::vector<uint64_t> offs;
  uint64_t total = 0;
  std::uniform_real_distribution<double> U(0, acc);
  while (total < (1ull << 30)) {
    const size_t k = std::lower_bound(cdf.begin(), cdf.end(), U(rng)) - cdf.begin() + 1;
    const uint32_t L = std::min<uint32_t>(65536, 64 * (uint32_t)k + (uint32_t)(rng() % 64));
    if (total + L > (1ull << 30)) break;
    offs.push_back(total);
    lens.push_back(L);
    total += L;
  }
  const size_t n = lens.size();
  printf("n=%zu total=%.3f GiB\n", n, total / 1073741824.0);
  char* d; uint64_t* doff; uint32_t *dlen, *out, *ref;
  CK(hipMalloc(&d, total + 256)); CK(hipMalloc(&doff, n * 8)); CK(hipMalloc(&dlen, n * 4));
  CK(hipMalloc(&out, n * 4)); CK(hipMalloc(&ref, n * 4));
  CK(hipMemset(d, 0x5A, total + 256));
  CK(hipMemcpy(doff, offs.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dlen, lens.data(), n * 4, hipMemcpyHostToDevice));
  DeviceCtx* c = nullptr;
  RC(annety_crc_init(0));
  RC(current_ctx(&c));
  STAGE("setup");
  // clocks up: fixed batches inside the arena (total + 256 bytes allocated)
  uint32_t* warm;
  CK(hipMalloc(&warm, (total / 1024) * 4));
  for (int r = 0; r < 3000; r++) RC(annety_crc32_batch_fixed(d, total / 1024, 1024, 1024, warm, nullptr));
  STAGE("warm fixed batches");
  RC(annety_crc32_batch_var(d, doff, dlen, n, ref, nullptr));
  STAGE("reference batch_var");
  const size_t rows_words = (size_t)bucket_grid(n) * kBucketCount;
  uint32_t *rows, *ranges; void *desc, *ws;
  CK(hipMalloc(&rows, rows_words * 4)); CK(hipMalloc(&ranges, 64)); CK(hipMalloc(&desc, 16 * n));
  CK(hipMalloc(&ws, kExtentScratchBytes)); CK(hipMemset(ws, 0, kExtentScratchBytes));
  uint64_t sorts = 0;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto b2b = [&](auto launch, const char* name, bool check) {
    for (int w = 0; w < 5; w++) launch();
    CK(hipEventRecord(e0));
    for (int r = 0; r < 30; r++) launch();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    STAGE(name);
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    bool ok = true;
    if (check) {
      std::vector<uint32_t> h1(n), h2(n);
      CK(hipMemcpy(h1.data(), out, n * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(h2.data(), ref, n * 4, hipMemcpyDeviceToHost));
      ok = h1 == h2;
    }
    printf("%-40s %.4f ms  %.1f GB/s %s\n", name, ms / 30, total / (ms / 30) / 1e6, check ? (ok ? "ok" : "MISMATCH") : "");
  };
  auto bucket = [&] {  // the product's two-launch counting sort (crc32_kernels.h BucketArgs)
    uint32_t* cur = reinterpret_cast<uint32_t*>(static_cast<char*>(ws) + kCursorOff);
    const uint32_t set = (uint32_t)(sorts++ & 1);
    BucketArgs bk{d, rows, cur + set * kBucketCount, cur + (set ^ 1) * kBucketCount, ranges, desc, out};
    uint32_t parts = 0;
    CK(launch_extent(doff, dlen, n, ws, &parts, &bk, nullptr));
    CK(launch_bucket_place(doff, dlen, n, ws, parts, bk, nullptr, 0, nullptr));
  };
  b2b([&] { RC(annety_crc32_batch_var(d, doff, dlen, n, out, nullptr)); }, "product batch_var", true);
  b2b(bucket, "bucket passes only", false);
  bucket();
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> hr(6);
  CK(hipMemcpy(hr.data(), ranges, 24, hipMemcpyDeviceToHost));
  printf("classes: G32 [%u,%u) G8 [%u,%u) G2 [%u,%u)\n", hr[0], hr[1], hr[2], hr[3], hr[4], hr[5]);
  b2b([&] { launch_cls<32, 0>(*c, d, n, desc, ranges, out); }, "class G32", false);
  b2b([&] { launch_cls<8, 0>(*c, d, n, desc, ranges + 2, out); }, "class G8", false);
  b2b([&] { launch_cls<2, 0>(*c, d, n, desc, ranges + 4, out); }, "class G2", false);
  b2b([&] { launch_cls<32, 1>(*c, d, n, desc, ranges, out); }, "class G32 no masks", false);
  b2b([&] { launch_cls<8, 1>(*c, d, n, desc, ranges + 2, out); }, "class G8 no masks", false);
  b2b([&] { launch_cls<2, 1>(*c, d, n, desc, ranges + 4, out); }, "class G2 no masks", false);
  b2b([&] { launch_cls<2, 3>(*c, d, n, desc, ranges + 4, out); }, "class G2 no masks no unshift", false);
  b2b([&] { launch_cls<4, 0>(*c, d, n, desc, ranges + 4, out); }, "G2 class run at G4", false);
  b2b([&] { launch_cls<1, 0>(*c, d, n, desc, ranges + 4, out); }, "G2 class run at G1", false);
  b2b([&] { launch_cls<16, 0>(*c, d, n, desc, ranges + 2, out); }, "G8 class run at G16", false);
  b2b([&] { launch_cls<4, 0>(*c, d, n, desc, ranges + 2, out); }, "G8 class run at G4", false);
  b2b([&] { launch_cls<16, 0>(*c, d, n, desc, ranges, out); }, "G32 class run at G16", false);
  return 0;
}
