// ISA-only build (never run): the product stitch kernel instantiated at 512 lanes (the product), at 768 lanes
// (3 waves per SIMD: a 168-VGPR cap) and at 1024 lanes (the variant that returned wrong digests in round 2,
// DESIGN.md §7.2), for microbench/isa_check.py.
// hipcc --offload-arch=gfx950 -O3 --save-temps -c microbench/isa_stitch.hip
#include "../annety_amd/csrc/crc32_arena.hip"

namespace annety_crc {
void* isa_stitch_kernels[] = {
    reinterpret_cast<void*>(&crc32_arena_stitch_kernel<false, 512, 0, 1>),
    reinterpret_cast<void*>(&crc32_arena_stitch_kernel<false, 768, 0, 0>),
    reinterpret_cast<void*>(&crc32_arena_stitch_kernel<false, 768, 0, 1>),
    reinterpret_cast<void*>(&crc32_arena_stitch_kernel<false, 1024, 0, 1>),
    reinterpret_cast<void*>(&crc32_arena_stitch_kernel<false, 1024, 0, 0>),
    reinterpret_cast<void*>(&crc32_arena_stitch_kernel<true, 1024, 0, 1>),
};
}  // namespace annety_crc
namespace annety_crc {
void* isa_stitch_lite_kernels[] = {
    reinterpret_cast<void*>(&crc32_arena_stitch_lite_kernel<false, 256, 4>),
    reinterpret_cast<void*>(&crc32_arena_stitch_lite_kernel<false, 512, 4>),
    reinterpret_cast<void*>(&crc32_arena_stitch_lite_kernel<false, 256, 3>),
};
}  // namespace annety_crc
