// Frame-level kernels for annety's LengthHeaderCodec wire format:
//   [length: T bytes, big-endian, T = 1/2/4/8][payload: length - 4 bytes][crc32(payload): 4 bytes BE]
// (include/codec/LengthHeaderCodec.h:33-46 layout, decode :71-137, encode :146-201; the big-endian
// integers are NetBuffer::append_int*/peek_int*, include/NetBuffer.h:38-105).
// The CRC itself comes from the batch kernels (crc32_kernels.hip); these kernels only read/write the
// 4-byte trailers, the headers and the payload copies.
#include <hip/hip_runtime.h>

#include "crc32_kernels.h"

namespace annety_crc {
namespace {

__device__ __forceinline__ uint32_t load_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | (uint32_t)p[3];
}

// ok[i] = digest[i] == big-endian trailer after payload i (LengthHeaderCodec::decode :111,123)
__global__ __launch_bounds__(256) void lhc_compare_kernel(const uint8_t* __restrict__ stream,
                                                          const uint64_t* __restrict__ off,
                                                          const uint32_t* __restrict__ len, size_t n,
                                                          const uint32_t* __restrict__ digest,
                                                          uint8_t* __restrict__ ok) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    ok[i] = load_be32(stream + off[i] + len[i]) == digest[i] ? 1 : 0;
}

// One wave per frame: header, payload copy, trailer (LengthHeaderCodec::encode :179-197, ProtobufCodec::
// encode :235-247). Payloads the reference would not write (empty: rt 0; length outside [enc_min,
// enc_max]: rt -1) are skipped, and
// the host plan (annety_lhc_encode_plan) gives them zero bytes in the output.
// The copy stores aligned dwords; each one is assembled from the two source dwords it straddles with
// v_alignbyte, so unaligned payloads still move 4 bytes per lane per instruction.
__global__ __launch_bounds__(256) void lhc_encode_kernel(const uint8_t* __restrict__ src,
                                                         const uint64_t* __restrict__ src_off,
                                                         const uint32_t* __restrict__ len, size_t n, int T,
                                                         int64_t enc_min, int64_t enc_max, uint8_t* __restrict__ dst,
                                                         const uint64_t* __restrict__ dst_off,
                                                         const uint32_t* __restrict__ digest) {
  const size_t waves = (size_t)gridDim.x * 4;
  const uint32_t lane = threadIdx.x & 63;
  for (size_t i = blockIdx.x * (size_t)4 + (threadIdx.x >> 6); i < n; i += waves) {
    const uint32_t L = len[i];
    if (L == 0 || (int64_t)L < enc_min || (enc_max > 0 && (int64_t)L > enc_max)) continue;
    const uint8_t* s = src + src_off[i];
    uint8_t* d = dst + dst_off[i];
    const uint64_t hdr = (uint64_t)L + 4;  // append_intT(length + 4): low T bytes, big-endian
    if (lane < (uint32_t)T) d[lane] = (uint8_t)(hdr >> (8 * (T - 1 - lane)));
    uint8_t* pd = d + T;
    const uint32_t to_align = (uint32_t)(-(uintptr_t)pd & 3);  // bytes until pd is dword aligned
    const uint32_t head = to_align < L ? to_align : L;
    if (lane < head) pd[lane] = s[lane];
    const uint32_t words = (L - head) >> 2;
    const uint8_t* sb = s + head;
    const uint32_t sh = (uint32_t)((uintptr_t)sb & 3);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>((uintptr_t)sb & ~(uintptr_t)3);
    uint32_t* dw = reinterpret_cast<uint32_t*>(pd + head);
    if (sh == 0) {
      for (uint32_t w = lane; w < words; w += 64) dw[w] = sw[w];
    } else {
      // the high dword holds source bytes of this word whenever sh != 0, so it is inside the payload
      for (uint32_t w = lane; w < words; w += 64)
        dw[w] = __builtin_amdgcn_alignbyte(sw[w + 1], sw[w], sh);
    }
    for (uint32_t b = head + 4 * words + lane; b < L; b += 64) pd[b] = s[b];
    if (lane < 4) pd[L + lane] = (uint8_t)(digest[i] >> (8 * (3 - lane)));
  }
}

}  // namespace

hipError_t launch_lhc_compare(const void* stream_base, const uint64_t* off, const uint32_t* len, size_t n,
                              const uint32_t* digest, uint8_t* ok, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const unsigned blocks = (unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  note_kernel("lhc_compare_kernel");
  hipLaunchKernelGGL(lhc_compare_kernel, dim3(blocks), dim3(256), 0, stream,
                     static_cast<const uint8_t*>(stream_base), off, len, n, digest, ok);
  return hipGetLastError();
}

hipError_t launch_lhc_encode(const void* src, const uint64_t* src_off, const uint32_t* len, size_t n, int T,
                             int64_t enc_min, int64_t enc_max, void* dst, const uint64_t* dst_off,
                             const uint32_t* digest, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const unsigned blocks = (unsigned)((n + 3) / 4 < 8192 ? (n + 3) / 4 : 8192);
  note_kernel("lhc_encode_kernel");
  hipLaunchKernelGGL(lhc_encode_kernel, dim3(blocks), dim3(256), 0, stream, static_cast<const uint8_t*>(src),
                     src_off, len, n, T, enc_min, enc_max, static_cast<uint8_t*>(dst), dst_off, digest);
  return hipGetLastError();
}

}  // namespace annety_crc
