// Does more data in flight per wave stream faster in the config-1 access shape? Pure read (xor of the
// words, no CRC): 256 workgroups x 512 lanes (one per CU, held there by a 144 KiB LDS allocation like the
// product's image), a lane reads one 128-byte line as 8 x 16 B per task, a wave 64 consecutive lines (8 KiB),
// tasks grid-strided; NBUF line buffers per lane (NBUF - 1 tasks' loads in flight during a fold).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 microbench/inflight_mb.hip -o inflight_mb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "HIP %s line %d\n", hipGetErrorString(e_), __LINE__);        \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

template <int NBUF>
__global__ __launch_bounds__(512) void k_inflight(const uint4* __restrict__ d, size_t ntask, uint32_t* out) {
  __shared__ uint32_t hold[144 * 1024 / 4];  // occupancy as the product: one workgroup per CU
  if (threadIdx.x == 0x7fffffff) hold[0] = 1;  // keep the allocation
  const size_t wave = (size_t)blockIdx.x * 8 + (threadIdx.x >> 6);
  const size_t nwave = (size_t)gridDim.x * 8;
  const uint32_t lane = threadIdx.x & 63;
  uint4 buf[NBUF][8];
  uint32_t acc = 0;
  // task t of this wave = wave + t * nwave; lane's line = task * 64 + lane (16 B units: * 8)
  auto load = [&](size_t t, uint4 (&v)[8]) {
    const size_t tt = t < ntask ? t : wave;  // past the end: re-read the first task (an L2 hit)
    const uint4* p = d + (tt * 64 + lane) * 8;
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = p[i];
  };
  size_t t = wave;
#pragma unroll
  for (int b = 0; b < NBUF - 1; b++) load(t + b * nwave, buf[b]);
  for (; t < ntask; t += NBUF * nwave) {
#pragma unroll
    for (int b = 0; b < NBUF; b++) {
      load(t + (b + NBUF - 1) * nwave, buf[(b + NBUF - 1) % NBUF]);
      __builtin_amdgcn_sched_barrier(0);
      if (t + b * nwave < ntask) {
#pragma unroll
        for (int i = 0; i < 8; i++) acc ^= buf[b][i].x ^ buf[b][i].y ^ buf[b][i].z ^ buf[b][i].w;
      }
    }
  }
  out[(size_t)blockIdx.x * 512 + threadIdx.x] = acc;
}

template <int NBUF>
float run(const uint4* d, size_t ntask, uint32_t* out, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 3; i++) hipLaunchKernelGGL(k_inflight<NBUF>, dim3(256), dim3(512), 0, 0, d, ntask, out);
  CK(hipEventRecord(e0));
  for (int i = 0; i < reps; i++) hipLaunchKernelGGL(k_inflight<NBUF>, dim3(256), dim3(512), 0, 0, d, ntask, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main() {
  const size_t bytes = 1ull << 30, ntask = bytes / 8192;
  uint4* d;
  uint32_t* out;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&out, 256 * 512 * 4));
  CK(hipMemset(d, 0x5A, bytes));
  for (int i = 0; i < 400; i++) hipLaunchKernelGGL(k_inflight<2>, dim3(256), dim3(512), 0, 0, d, ntask, out);  // clocks
  for (int rep = 0; rep < 3; rep++) {
    const float m2 = run<2>(d, ntask, out, 50), m3 = run<3>(d, ntask, out, 50), m4 = run<4>(d, ntask, out, 50),
                m6 = run<6>(d, ntask, out, 50);
    printf("NBUF 2: %.4f ms %.0f GB/s | 3: %.4f ms %.0f | 4: %.4f ms %.0f | 6: %.4f ms %.0f\n", m2, bytes / m2 / 1e6, m3,
           bytes / m3 / 1e6, m4, bytes / m4 / 1e6, m6, bytes / m6 / 1e6);
    fflush(stdout);
  }
  return 0;
}
