// Arena line pass breakdown at config-3 size (1 GiB arena): the product kernel vs PROBE variants that
// drop the S store / superblock scan, next to the config-1 kernel on the same bytes.
#include "../annety_amd/csrc/crc32_kernels.hip"
#include "../annety_amd/csrc/crc32_arena.hip"
#include "../annety_amd/csrc/crc32_frames.hip"
#include "../annety_amd/csrc/crc32_host.cpp"
#include "../annety_amd/csrc/crc32_capi.cpp"
#include "arena_sw.h"
#include <cstdio>
#include <string>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)
#define RC(x) do { int r_ = (x); if (r_) { printf("%s -> %d\n", #x, r_); exit(3); } } while (0)
using namespace annety_crc;

template <int PROBE, bool NT = true>
void lines(DeviceCtx&, const ArenaLaunch& a) {
  CK((launch_arena_lines_p<PROBE, NT>(a, 0)));
}

// `arena_mb place`: the product line pass with the arena and the S/SB scratch at different offsets in
// their allocations (does the placement of the two streams in HBM move the pass time?)
int place() {
  const size_t bytes = 1ull << 30, slack = 64ull << 20;
  char* d0; uint32_t* s0;
  CK(hipMalloc(&d0, bytes + slack)); CK(hipMemset(d0, 0x3C, bytes + slack));
  RC(annety_crc_init(0));
  DeviceCtx* c = nullptr; RC(current_ctx(&c));
  ArenaLaunch a{};
  arena_fill(*c, d0, bytes, a);
  const size_t words = arena_geom(a).words;
  CK(hipMalloc(&s0, words * 4 + slack));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const size_t doffs[] = {0, 8192, 1 << 20, 32ull << 20};
  const size_t soffs[] = {0, 1024, 4096, 65536, 1 << 20, 16ull << 20};
  for (size_t dof : doffs)
    for (size_t sof : soffs) {
      ArenaLaunch b{};
      arena_fill(*c, d0 + dof, bytes, b);
      b.scratch = s0 + sof / 4;
      for (int w = 0; w < 100; w++) CK(launch_arena_lines(b, 0));
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      for (int r = 0; r < 100; r++) CK(launch_arena_lines(b, 0));
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipGetLastError());
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      printf("arena +%-10zu scratch +%-10zu %.4f ms\n", dof, sof, ms / 100);
    }
  return 0;
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  if (argc > 1 && std::string(argv[1]) == "place") return place();
  const size_t bytes = 1ull << 30;
  char* d; uint32_t *scratch, *out;
  CK(hipMalloc(&d, bytes)); CK(hipMemset(d, 0x3C, bytes));
  RC(annety_crc_init(0));
  DeviceCtx* c = nullptr; RC(current_ctx(&c));
  ArenaLaunch a{};
  arena_fill(*c, d, bytes, a);
  CK(hipMalloc(&scratch, arena_geom(a).words * 4)); CK(hipMalloc(&out, (bytes / 1024) * 4));
  a.scratch = scratch;
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto t = [&](auto f, const char* name) {
    for (int w = 0; w < 200; w++) f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < 100; r++) f();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipGetLastError());
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%-36s %.4f ms  %.1f GB/s\n", name, ms / 100, bytes / (ms / 100) / 1e6);
  };
  t([&] { RC(annety_crc32_batch_fixed(d, bytes / 1024, 1024, 1024, out, nullptr)); }, "config-1 kernel (oneround<8>)");
  for (int rep = 0; rep < 2; rep++) {
    t([&] { lines<0>(*c, a); }, "arena lines (product, coalesced nt loads)");
    t([&] { lines<1>(*c, a); }, "  no S store");
    t([&] { lines<2>(*c, a); }, "  no superblock scan");
    t([&] { lines<3>(*c, a); }, "  no S store, no superblock scan");
    t([&] { lines<4>(*c, a); }, "  no SB store");
    t([&] { lines<5>(*c, a); }, "  no S store, no SB store");
    t([&] { lines<0, false>(*c, a); }, "arena lines, per-line loads");
    t([&] { lines<1, false>(*c, a); }, "  no S store");
    t([&] { lines<3, false>(*c, a); }, "  no S store, no superblock scan");
  }
  if (getenv("NO_SW")) return 0;
  t([&] { CK(launch_arena_lines_sw<0>(a, 0)); }, "store wave (8 + 1 waves, LDS ring)");
  t([&] { CK(launch_arena_lines_sw<1>(a, 0)); }, "  ring, store wave stores nothing");
  t([&] { CK(launch_arena_lines_sw<2>(a, 0)); }, "  no ring (9 waves, no hand-off)");
  t([&] { lines<0>(*c, a); }, "arena lines (product) again");
  // S traffic alone: the same 32 MiB of stores as a separate pass
  t([&] { CK(hipMemsetAsync(a.scratch, 0, a.nsb * 64 * 4, 0)); }, "memset of S (32 MiB)");
  return 0;
}
