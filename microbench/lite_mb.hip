// Lite stitch A/B on the config-3 batch (Zipf lengths as bench.py, packed, ~1 GiB): the product stitch
// (157 KiB LDS image, one block per CU) vs the lite image (30 KiB, no slicing tables) at several block
// shapes / occupancies, after one real line pass; digests compared with the product's.
#include "../annety_amd/csrc/crc32_kernels.hip"
#include "../annety_amd/csrc/crc32_arena.hip"
#include "../annety_amd/csrc/crc32_frames.hip"
#include "../annety_amd/csrc/crc32_host.cpp"
#include "../annety_amd/csrc/crc32_capi.cpp"
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
#define RC(x) do { int r_ = (x); if (r_) { printf("%s -> %d\n", #x, r_); exit(3); } } while (0)
using namespace annety_crc;

int main() {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  std::mt19937_64 rng(0x5EED);
  std::vector<double> cdf(1024);
  double acc = 0;
  for (int k = 1; k <= 1024; k++) cdf[k - 1] = (acc += std::pow((double)k, -1.1));
  std::uniform_real_distribution<double> U(0, acc);
  std::vector<uint32_t> lens;
  std::vector<uint64_t> offs;
  uint64_t total = 0;
  while (true) {
    const size_t k = std::lower_bound(cdf.begin(), cdf.end(), U(rng)) - cdf.begin() + 1;
    const uint32_t L = std::min<uint32_t>(65536, 64 * (uint32_t)k + (uint32_t)(rng() % 64));
    if (total + L > (1ull << 30)) break;
    offs.push_back(total);
    lens.push_back(L);
    total += L;
  }
  const size_t n = lens.size();
  printf("n=%zu total=%.3f GiB\n", n, total / 1073741824.0);
  char* d; uint64_t* doff; uint32_t *dlen, *out;
  CK(hipMalloc(&d, total + 256)); CK(hipMemset(d, 0x5A, total + 256));
  CK(hipMalloc(&doff, n * 8)); CK(hipMalloc(&dlen, n * 4)); CK(hipMalloc(&out, n * 4));
  CK(hipMemcpy(doff, offs.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dlen, lens.data(), n * 4, hipMemcpyHostToDevice));
  RC(annety_crc_init(0));
  DeviceCtx* c = nullptr; RC(current_ctx(&c));
  ArenaLaunch a{};
  arena_fill(*c, d, total, a);
  a.off = doff; a.len = dlen; a.n = n; a.out = out;
  CK(hipMalloc(&a.scratch, arena_geom(a).words * 4));
  CK(launch_arena_lines(a, 0));
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto t = [&](auto f, const char* name) {
    for (int w = 0; w < 50; w++) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 100; r++) f();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipGetLastError());
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-40s %.2f us\n", name, ms / 100 * 1000);
  };
  // lite image: half-line join + segment maps + inverse shifts + quarter join (the stitch layout from
  // kLdsHalfOff) + shift_4
  void* lite; CK(hipMalloc(&lite, kLdsLiteBytes));
  CK(hipMemcpy(lite, (char*)c->d_slice + kLdsHalfOff, 512, hipMemcpyDeviceToDevice));
  CK(hipMemcpy((char*)lite + 512, c->d_stitch, kLdsStitchImageBytes - kLdsCommonBytes, hipMemcpyDeviceToDevice));
  std::vector<uint32_t> w4(128);
  nibble_tables(shift_matrix(4), w4.data());
  CK(hipMemcpy((char*)lite + (kLdsWordOff - kLdsHalfOff), w4.data(), 512, hipMemcpyHostToDevice));
  CK(launch_stitch_p<0>(a, 0));
  std::vector<uint32_t> r0(n), r1(n);
  CK(hipMemcpy(r0.data(), out, n * 4, hipMemcpyDeviceToHost));
  auto same = [&](auto f, const char* name) {
    CK(hipMemset(out, 0, n * 4));
    f(); CK(hipDeviceSynchronize()); CK(hipMemcpy(r1.data(), out, n * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < n; i++) bad += r0[i] != r1[i];
    printf("%-40s %zu of %zu digests differ from the product's\n", name, bad, n);
  };
  const size_t cus = (size_t)c->cus;
#define V(BLK, WPE, BL, NAME) \
  same([&] { CK((launch_stitch_lite<BLK, WPE>(a, lite, BL, 0))); }, NAME); \
  t([&] { CK((launch_stitch_lite<BLK, WPE>(a, lite, BL, 0))); }, NAME);
  t([&] { CK(launch_stitch_p<0>(a, 0)); }, "stitch (product)");
  V(512, 1, cus, "lite 512, grid = CUs")
  V(512, 1, 0, "lite 512, 1 payload/lane")
  V(256, 1, 0, "lite 256, 1 payload/lane")
  V(256, 3, 0, "lite 256, >=3 waves/SIMD")
  V(512, 4, 0, "lite 512, >=4 waves/SIMD")
  V(256, 4, 0, "lite 256, >=4 waves/SIMD")
  V(128, 4, 0, "lite 128, >=4 waves/SIMD")
  t([&] { CK(launch_stitch_p<0>(a, 0)); }, "stitch (product, again)");
  return 0;
}
