// Would a fused encode copy fit in the arena line pass? The product line pass over a 1 GiB arena against the same
// pass storing every loaded chunk 4 bytes further on in a second buffer (PROBE bit 3: unaligned 16-byte stores,
// the byte shift of a LengthHeaderCodec frame), with and without the S stores, beside a plain copy kernel of the same
// bytes (16-byte loads and unaligned stores, 4 chunks per lane in flight).
#include "../annety_amd/csrc/crc32_kernels.hip"
#include "../annety_amd/csrc/crc32_arena.hip"
#include "../annety_amd/csrc/crc32_frames.hip"
#include "../annety_amd/csrc/crc32_host.cpp"
#include "../annety_amd/csrc/crc32_capi.cpp"
#include <cstdio>
#include <string>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
#define RC(x) do { int r_ = (x); if (r_) { printf("%s -> %d\n", #x, r_); exit(3); } } while (0)
using namespace annety_crc;

template <int PROBE>
void lines(const ArenaLaunch& a, int64_t delta) {
  const ArenaGeom geo = launch_geom(a);
  LineOut ar = line_out(a, geo);
  ar.probe_delta = delta;
  hipLaunchKernelGGL((crc32_arena_lines_kernel<PROBE, true>), dim3((unsigned)geo.blocks), dim3(kBlock), 0, 0,
                     reinterpret_cast<const uint8_t*>((uintptr_t)(a.fs0 * 8192)), ar,
                     static_cast<const uint4*>(a.img_slice), static_cast<const uint4*>(a.img_group8),
                     static_cast<const uint4*>(a.img_sb));
  CK(hipGetLastError());
}

template <int SHIFT, bool NTS>
__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ src, uint8_t* __restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256 * 4;
  for (size_t i = blockIdx.x * (size_t)1024 + threadIdx.x; i < n; i += stride) {
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = gload16_nt((uint64_t)(uintptr_t)(i + 256 * k < n ? src + i + 256 * k : src), 0);
#pragma unroll
    for (int k = 0; k < 4; k++)
      if (i + 256 * k < n) {
        if constexpr (NTS) gstore16_nt((uint64_t)(uintptr_t)dst + 16 * (i + 256 * k) + SHIFT, v[k]);
        else gstore16((uint64_t)(uintptr_t)dst + 16 * (i + 256 * k) + SHIFT, v[k]);
      }
  }
}

int main() {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const size_t bytes = 1ull << 30;
  char *d, *dst;
  uint32_t* scratch;
  CK(hipMalloc(&d, bytes)); CK(hipMemset(d, 0x3C, bytes));
  CK(hipMalloc(&dst, bytes + 4096)); CK(hipMemset(dst, 0, bytes + 4096));
  RC(annety_crc_init(0));
  DeviceCtx* c = nullptr; RC(current_ctx(&c));
  ArenaLaunch a{};
  arena_fill(*c, d, bytes, a);
  CK(hipMalloc(&scratch, arena_geom(a).words * 4));
  a.scratch = scratch;
  const int64_t delta = (int64_t)((uintptr_t)dst - (uintptr_t)d) + 4;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto t = [&](auto f, const char* name) {
    for (int w = 0; w < 100; w++) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 100; r++) f();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipGetLastError());
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-48s %.4f ms  %.1f GB/s of reads\n", name, ms / 100, bytes / (ms / 100) / 1e6);
  };
  int dev; CK(hipGetDevice(&dev)); int cus; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  for (int rep = 0; rep < 2; rep++) {
    t([&] { lines<0>(a, 0); }, "arena lines (product)");
    t([&] { lines<8>(a, delta); }, "  + copy of every chunk (+4 B, unaligned)");
    t([&] { lines<9>(a, delta); }, "  + copy, no S stores");
    auto cp = [&](auto kern, const char* what) {
      for (int per : {8, 16}) {
        char name[96]; snprintf(name, sizeof name, "plain copy %s, %d blocks per CU", what, per);
        t([&] { hipLaunchKernelGGL(kern, dim3(cus * per), dim3(256), 0, 0, reinterpret_cast<const uint4*>(d),
                                   reinterpret_cast<uint8_t*>(dst), bytes / 16); }, name);
      }
    };
    cp(copy_kernel<4, false>, "+4 B");
    cp(copy_kernel<4, true>, "+4 B, nt stores");
    cp(copy_kernel<0, false>, "aligned");
    cp(copy_kernel<0, true>, "aligned, nt stores");
    t([&] { CK(hipMemcpyAsync(dst, d, bytes, hipMemcpyDeviceToDevice, 0)); }, "hipMemcpyAsync D2D");
  }
  // the copy is right
  std::string h(bytes, 0), g(bytes, 0);
  for (int i = 0; i < 3; i++) {
    CK(hipMemset(dst, 0, bytes + 4096));
    uint8_t pat[4] = {1, 2, 3, 4};
    (void)pat;
    lines<8>(a, delta);
    CK(hipDeviceSynchronize());
  }
  CK(hipMemcpy(h.data(), d, bytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(g.data(), dst + 4, bytes, hipMemcpyDeviceToHost));
  printf("copy %s\n", h == g ? "exact" : "WRONG");
  return 0;
}
