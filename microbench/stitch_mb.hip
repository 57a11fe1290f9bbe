// Arena stitch breakdown on the config-3 batch (Zipf lengths as bench.py, packed, ~1 GiB): the full
// stitch vs PROBE variants (descriptors only / + all loads / + window folds), after one real line pass.
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
  t([&] { CK(launch_arena_lines(a, 0)); }, "line pass");
  t([&] { CK(launch_stitch_p<0>(a, 0)); }, "stitch (product)");
  t([&] { CK(launch_stitch_p<1>(a, 0)); }, "  descriptors + store only");
  t([&] { CK(launch_stitch_p<2>(a, 0)); }, "  + all loads");
  t([&] { CK(launch_stitch_p<3>(a, 0)); }, "  + window folds, no map steps");
  t([&] { CK((launch_stitch_p<0, 1>(a, 0))); }, "stitch, next payload prefetched (PIPE 1)");
  t([&] { CK((launch_stitch_p<0, 2>(a, 0))); }, "stitch, two payloads' loads together (PIPE 2)");
  auto same = [&](auto f, const char* name) {
    std::vector<uint32_t> r0(n), r1(n);
    CK(launch_stitch_p<0>(a, 0)); CK(hipMemcpy(r0.data(), out, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemset(out, 0, n * 4));
    f(); CK(hipMemcpy(r1.data(), out, n * 4, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (size_t i = 0; i < n; i++) bad += r0[i] != r1[i];
    printf("%s vs product: %zu of %zu digests differ\n", name, bad, n);
  };
  same([&] { CK((launch_stitch_p<0, 1>(a, 0))); }, "PIPE 1");
  same([&] { CK((launch_stitch_p<0, 2>(a, 0))); }, "PIPE 2");
  t([&] { CK(launch_stitch_p<0>(a, 0)); }, "stitch (product, again)");
  t([&] { CK(launch_arena(a, 0)); }, "line pass + stitch (no alloc)");
  t([&] { RC(annety_crc32_batch_var_arena(d, total, doff, dlen, n, out, nullptr)); }, "product arena call (both + alloc)");
  return 0;
}
