// Frame-level kernels for annety's LengthHeaderCodec wire format:
//   [length: T bytes, big-endian, T = 1/2/4/8][payload: length - 4 bytes][crc32(payload): 4 bytes BE]
// (include/codec/LengthHeaderCodec.h:33-46 layout, decode :71-137, encode :146-201; the big-endian
// integers are NetBuffer::append_int*/peek_int*, include/NetBuffer.h:38-105).
// Verify takes the CRCs from the batch kernels (crc32_kernels.hip) and compares the 4-byte trailers; encode
// (lhc_encode_fused_kernel) reads each payload once and writes its whole frame, CRC included.
#include <hip/hip_runtime.h>

#include "crc32_device.h"
#include "crc32_kernels.h"
#include "crc32_math.h"

#include <algorithm>

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

// ---------------------------------------------------------------------------------------------
// Fused LengthHeaderCodec encode (round 5; LengthHeaderCodec::encode :146-201 over a batch): each payload is read
// once. One lane group of 8 per frame, frames i = group, group + groups, ... Rounds of 8 end-aligned 128-byte
// lines (lane j holds line 8 r + j - vlead of the payload, the lanes before line 0 re-read it), per-line loads
// plus the first dword of the next line. From the same registers:
//   * the CRC, as the sorted path's one-round payloads (bytes outside the payload masked, the init as the register shift_{128-lead}(init)
//     of line 0, rounds chained through shift_{7*128}, the join and the inverse shift of the last line's
//     overhang);
//   * the copy: every destination-aligned dword whose four bytes are payload bytes is stored by the lane holding
//     its first byte, as v_alignbyte of two line words (the byte shift c = (src - dst) mod 4 is one per frame);
//   * at the frame's end the group's lanes store the T header bytes, the 4 trailer bytes and the <= 3 payload
//     bytes before the first and after the last aligned dword (loaded as bytes with the lines).
// Frames the reference would not write (empty, or length outside [enc_min, enc_max]) get no bytes (the host plan
// gave them none). Algorithmic traffic: the payload read once, the frame written once.
struct EncTask {
  uint64_t A, Dp;  // payload source address, payload destination address (frame start + T)
  uint64_t L0;     // first source line (absolute)
  uint32_t L, nl, R, vlead, lead, te;
  bool live, valid;  // live: an index of the batch; valid: a frame to write
};
__device__ __forceinline__ EncTask decode_enc(const uint8_t* src, uint8_t* dst, uint64_t soff, uint32_t L,
                                              uint64_t foff, int T, int64_t enc_min, int64_t enc_max, bool live,
                                              uint64_t zero_line) {
  EncTask k;
  k.live = live;
  k.valid = live && L > 0 && (int64_t)L >= enc_min && !(enc_max > 0 && (int64_t)L > enc_max);
  k.L = L;
  // a task without a frame reads the library's zero line (its payload may sit at the very end of the source)
  k.A = k.valid ? (uint64_t)(uintptr_t)(src + soff) : zero_line;
  const uint64_t e = k.A + (k.valid ? L : 1u);
  k.Dp = (uint64_t)(uintptr_t)(dst + foff) + (uint32_t)T;
  k.L0 = k.A >> 7;
  k.nl = (uint32_t)(((e - 1) >> 7) - k.L0 + 1);
  k.R = (k.nl + 7) >> 3;
  k.vlead = 8 * k.R - k.nl;
  k.lead = (uint32_t)(k.A & 127);
  k.te = (uint32_t)(((e - 1) & 127) + 1);
  return k;
}

__global__ __launch_bounds__(kBlock) void lhc_encode_fused_kernel(const uint8_t* __restrict__ src,
                                                                  const uint64_t* __restrict__ src_off,
                                                                  const uint32_t* __restrict__ len, size_t n, int T,
                                                                  int64_t enc_min, int64_t enc_max,
                                                                  uint8_t* __restrict__ dst,
                                                                  const uint64_t* __restrict__ dst_off,
                                                                  uint64_t zero_line,
                                                                  const uint4* __restrict__ img_slice,
                                                                  const uint4* __restrict__ img_g8,
                                                                  const uint4* __restrict__ img_unshift) {
  constexpr int G = 8;
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsVarImageBytes / 16];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  const uint32_t j = threadIdx.x & 7, l = threadIdx.x & 63;
  const size_t gid = group_id<kBlock, G, kVwg>();
  const size_t ngroups = ((size_t)gridDim.x * kBlock) / G;
  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;
  const uint32_t slot128 = ((threadIdx.x & 24) | 6) << 2;  // shift_128 (join slot j = 6 of this replica row)
  auto fetch = [&](size_t t, uint64_t& so, uint32_t& ln, uint64_t& fo) __attribute__((always_inline)) {
    const size_t tc = t < n ? t : n - 1;  // unconditional: past the end re-read the last frame's fields
    so = src_off[tc];
    ln = len[tc];
    fo = dst_off[tc];
  };
  auto dec = [&](size_t t, uint64_t so, uint32_t ln, uint64_t fo) __attribute__((always_inline)) {
    return decode_enc(src, dst, so, ln, fo, T, enc_min, enc_max, t < n, zero_line);
  };
  // lane j: its line of round r, the next line's first dword, and edge byte slot j (0-2: payload bytes 0-2,
  // 3-5: the last three)
  auto load = [&](const EncTask& tk, uint32_t r, uint4 (&v)[8], uint32_t& nxt, uint32_t& eb)
      __attribute__((always_inline)) {
    const int32_t li = (int32_t)(8 * r + j) - (int32_t)tk.vlead;
    const int32_t lc = min(max(li, 0), (int32_t)tk.nl - 1);
    const uint64_t a = (tk.L0 + (uint64_t)lc) << 7;
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = gload16(a + 16 * i);
    nxt = gload4(lc + 1 < (int32_t)tk.nl ? a + 128 : a);
    const int32_t b = j < 3 ? (int32_t)j : (int32_t)tk.L - 6 + (int32_t)j;
    const int32_t bc = tk.valid ? min(max(b, 0), (int32_t)tk.L - 1) : 0;
    eb = gload1(tk.A + (uint64_t)bc);
  };

  size_t tL = gid;
  if (!__syncthreads_or(tL < n)) return;
  uint64_t so, fo;
  uint32_t ln;
  fetch(tL, so, ln, fo);
  EncTask dL = dec(tL, so, ln, fo);
  uint64_t sn, fn;
  uint32_t lnn;
  fetch(tL + ngroups, sn, lnn, fn);
  uint4 A[8], B[8];
  uint32_t nA = 0, nB = 0, eA = 0, eB = 0;
  load(dL, 0, A, nA, eA);
  EncTask dC = dL;
  uint32_t rC = 0, rL = 1;
  load_image<kLdsVarImageBytes>(lds4, img_slice, img_g8, img_unshift);
  __syncthreads();

  uint32_t s = 0;
  auto compute = [&](uint4 (&v)[8], uint32_t nxtw, uint32_t ebyte, const EncTask& tk, uint32_t r)
      __attribute__((always_inline)) {
    const int32_t li = (int32_t)(8 * r + j) - (int32_t)tk.vlead;
    const int32_t lo = li == 0 ? (int32_t)tk.lead : 0;
    const int32_t hi = li < 0 ? 0 : (li == (int32_t)tk.nl - 1 ? (int32_t)tk.te : 128);
    // the copy first (the unmasked line): dword q = source bytes [4q + c, 4q + c + 4) of this line
    if (tk.valid && li >= 0) {
      const uint32_t c = (uint32_t)(tk.A - tk.Dp) & 3u;
      const int32_t hi2 = li + 1 < (int32_t)tk.nl ? 128 + (li + 2 == (int32_t)tk.nl ? (int32_t)tk.te : 128) : hi;
      const uint64_t lb = (tk.L0 + (uint64_t)li) << 7;
      const uint64_t d = tk.Dp - tk.A + lb;  // + o: the destination of line byte o
      const uint32_t* w = reinterpret_cast<const uint32_t*>(v);
#pragma unroll
      for (int q = 0; q < 32; q++) {
        const int32_t o = 4 * q + (int32_t)c;
        const uint32_t hiw = q < 31 ? w[q + 1] : nxtw;
        const uint32_t x = __builtin_amdgcn_alignbyte(hiw, w[q], c);
        if (o >= lo && o + 4 <= hi2) gstore4(d + (uint64_t)o, x);
      }
    }
    mask_line<8>(v, lo * 8, hi * 8);
    const uint32_t sin = r > 0 ? nibble_map_uniform(s, lds, kLdsRoundOff) : 0u;  // shift_{7*128}
    s = absorb_line(sin, v, k, lds);
    if (li == 0) {  // the init as the register at the payload start
      uint32_t x = nibble_map_uniform(kInit, lds, kLdsUnshiftOff + (tk.lead & 15u) * 512);
      x = nibble_map_uniform(x, lds, kLdsUnshiftOff + 8192 + (tk.lead >> 4) * 512);
      s ^= nibble_map_lane(x, lds, slot128);
    }
    if (__builtin_amdgcn_ballot_w64(r + 1 == tk.R) != 0) {  // some group finishes its frame
      uint32_t t = group_xor_reduce<G>(nibble_map_lane(s, lds, k.slot4));
      const uint32_t over = 128 - tk.te;
      if (over) {
        t = nibble_map_uniform(t, lds, kLdsUnshiftOff + (over & 15u) * 512);
        t = nibble_map_uniform(t, lds, kLdsUnshiftOff + 8192 + (over >> 4) * 512);
      }
      const uint32_t crc = ~(uint32_t)__builtin_amdgcn_ds_bpermute(4 * (int)(l | 7u), (int)t);  // lane 7's
      if (r + 1 == tk.R) {
        if (tk.valid) {
          const uint64_t p = tk.Dp;
          const uint64_t hdr = (uint64_t)tk.L + 4;  // append_intT(length + 4), big-endian
          if ((int)j < T) gstore1(p - (uint64_t)T + j, (uint32_t)(hdr >> (8 * (T - 1 - (int)j))));
          if (j < 4) gstore1(p + tk.L + j, crc >> (8 * (3 - j)));
          const uint32_t hb = min((4u - (uint32_t)(tk.Dp & 3)) & 3u, tk.L);
          const uint32_t tb = min((uint32_t)((tk.Dp + tk.L) & 3), tk.L - hb);
          const int32_t b = j < 3 ? (int32_t)j : (int32_t)tk.L - 6 + (int32_t)j;
          const bool edge = j < 3 ? b < (int32_t)hb : (j < 6 && b >= (int32_t)(tk.L - tb) && b >= (int32_t)hb);
          if (edge) gstore1(p + (uint64_t)b, ebyte);
        }
        s = 0;
      }
    }
  };
  auto step = [&](uint4 (&cur)[8], uint32_t cn, uint32_t ce, uint4 (&nxt)[8], uint32_t& nn, uint32_t& ne)
      __attribute__((always_inline)) {
    if (__builtin_amdgcn_ballot_w64(rL >= dL.R) != 0) {
      if (rL >= dL.R) {
        tL += ngroups;
        dL = dec(tL, sn, lnn, fn);
        rL = 0;
      }
    }
    fetch(tL + ngroups, sn, lnn, fn);  // unconditional: the same addresses until dL ends
    load(dL, rL, nxt, nn, ne);
    __builtin_amdgcn_sched_barrier(0);
    compute(cur, cn, ce, dC, rC);
    dC = dL;
    rC = rL;
    rL++;
  };
  while (__builtin_amdgcn_ballot_w64(dC.live) != 0) {
    step(A, nA, eA, B, nB, eB);
    step(B, nB, eB, A, nA, eA);
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

hipError_t launch_lhc_encode_fused(const void* src, const uint64_t* src_off, const uint32_t* len, size_t n, int T,
                                   int64_t enc_min, int64_t enc_max, void* dst, const uint64_t* dst_off,
                                   const void* zero_line, const void* img_slice, const void* img_g8,
                                   const void* img_unshift, size_t max_blocks, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const size_t want = (n * 8 + kBlock - 1) / kBlock;
  const unsigned blocks = (unsigned)std::max<size_t>(1, std::min(max_blocks, want));
  note_kernel("lhc_encode_fused_kernel");
  hipLaunchKernelGGL(lhc_encode_fused_kernel, dim3(blocks), dim3(kBlock), 0, stream, static_cast<const uint8_t*>(src),
                     src_off, len, n, T, enc_min, enc_max, static_cast<uint8_t*>(dst), dst_off,
                     (uint64_t)(uintptr_t)zero_line, static_cast<const uint4*>(img_slice),
                     static_cast<const uint4*>(img_g8), static_cast<const uint4*>(img_unshift));
  return hipGetLastError();
}

}  // namespace annety_crc
