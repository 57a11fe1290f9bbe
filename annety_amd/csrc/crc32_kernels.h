// Internal launcher interface between the C-ABI shim (crc32_capi.cpp) and the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace annety_crc {

struct ShiftCols {
  uint32_t c[32];  // columns of a GF(2) 32x32 matrix (passed by value in the kernarg segment)
};

struct FixedLaunch {
  const void* base;        // device pointer to payload 0 (16-byte aligned)
  size_t n;                // payload count
  size_t stride;           // bytes between payload starts (multiple of 16)
  uint32_t len_blocks;     // payload length / 16
  uint32_t group;          // lanes per payload: 1, 2, 4, 8, 16 or 32
  uint32_t rounds;         // ceil(ceil(len/128) / group)
  uint32_t vlead;          // virtual leading zero blocks = rounds*group*8 - len_blocks
  bool full;               // vlead == 0
  bool raw;                // crc32_update semantics (out holds the input register, in place)
  const void* img_slice;   // 128 KiB slicing-table image (device)
  const void* img_group;   // 16.5 KiB join + round image for `group` (device)
  ShiftCols raw_shift_cols;  // raw only: shift_len columns
  uint32_t* out;           // digests (device)
  size_t max_blocks;       // persistent grid size (one workgroup per CU)
};

hipError_t launch_fixed(const FixedLaunch& a, hipStream_t stream);

struct VarLaunch {
  const void* base;          // device base pointer
  size_t n;                  // payload count
  const uint64_t* off;       // device offsets (or null: off = i * fixed_stride)
  const uint32_t* len;       // device lengths (or null: len = fixed_len)
  uint64_t fixed_stride;
  uint32_t fixed_len;
  const uint32_t* order;     // optional device permutation of payload indices
  uint32_t group;            // lanes per payload
  const void* img_slice;
  const void* img_group;
  const uint32_t* unshift;   // 128 x 8 x 16 nibble tables of shift_{-over}
  const uint32_t* short_init;  // shift_len(0xFFFFFFFF) for len = 0..3
  uint32_t* out;
  size_t max_blocks;
};

hipError_t launch_var(const VarLaunch& a, hipStream_t stream);
int fixed_kernel_block();

}  // namespace annety_crc
