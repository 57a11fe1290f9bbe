// Line-stream path for variable-length batches in any layout (annety_crc32_batch_var and its update form):
// every payload's absolute 128-byte lines, concatenated in payload order, form one stream of "positions",
// and the chip walks that stream in equal chunks, one chunk per wave. No sort, no length classes, no
// virtual lines: a wave step is 64 real lines whatever the length mix. Three launches:
//
//  1. crc32_stream_scan_kernel: one pass over the descriptors with a decoupled look-back scan (tiles of
//     2048 payloads, a ticket per tile): for the k-th non-empty payload, desc[k] = {address, length, index}
//     and posv[k] = its first position; totals = {K, positions}. Empty payloads get their digest (0) here.
//  2. crc32_stream_kernel: wave w takes positions [w * C, (w + 1) * C) (C = a multiple of 64 chosen on the
//     device from the total). Per step, lane l owns position q0 + l: it finds its payload from a window of
//     64 descriptors (a start flag per position, mbcnt of the flags), loads its line, masks the bytes
//     outside the payload (and complements the first four payload bytes: the init), folds it from register
//     0, and the wave runs a segmented inclusive scan of the lines' registers,
//         R_l = shift_{d*128}(R_{l-d}) ^ R_l   for d = 1, 2, ..., 32 while l - d is in l's payload,
//     whose maps are the same for every lane (broadcast LDS reads, no bank conflicts). A payload's last
//     line then holds its register; one inverse shift drops the zeros behind its last byte. The register
//     of a payload still open at the end of a step enters the next step's first line (the carry).
//  3. crc32_stream_fixup_kernel: payloads that cross a chunk boundary are joined from the chunks' pieces,
//     crc = XOR_c shift_{lines after piece c}(piece c), one wave per payload.
//
// Roofline: HBM-bound like the fixed kernels (a step reads 64 lines = 8 KiB per wave; the lines shared by
// two payloads are read twice, 2 % on BASELINE config 3). DESIGN.md §2.5.
// Reference semantics: crc32_long include/Crc32c.h:58-69, crc32_update :71-82 (UPD); math: crc32_math.h.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "crc32_device.h"
#include "crc32_kernels.h"
#include "crc32_math.h"

namespace annety_crc {
namespace {

constexpr int kScanBlock = 512;
constexpr int kScanPer = kStreamTile / kScanBlock;  // payloads per thread (contiguous)
static_assert(kScanPer * kScanBlock == (int)kStreamTile, "tile = block * per-thread");
constexpr int kFixBlock = 1024;
constexpr uint32_t kNoPayload = 0xFFFFFFFFu;
// A look-back that waits this long for a predecessor tile gives up (the digests are then wrong and
// totals[2] says so) instead of hanging the GPU: a bound, never reached by a correct launch.
constexpr uint32_t kSpinMax = 1u << 22;

__device__ __forceinline__ uint64_t ld_acquire(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_release(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// 128-byte lines of a payload at absolute address a, length len > 0.
__device__ __forceinline__ uint32_t line_count(uint64_t a, uint32_t len) {
  return (uint32_t)(((a + len - 1) >> 7) - (a >> 7) + 1);
}

// ---------------------------------------------------------------------------------------------------
// 1. Scan. Status set (crc32_kernels.h StreamLaunch::status): word 0 = ticket counter, tile t's record at
// 8 + 8t: [0] flag (0 none, 1 aggregate, 2 inclusive), [1] aggregate lines, [2] aggregate count,
// [3] inclusive lines, [4] inclusive count. The set is zero when the call starts (zeroed by the previous
// call on the slot, which used the other set, or at allocation).
template <bool UPD>
__global__ __launch_bounds__(kScanBlock) void crc32_stream_scan_kernel(StreamScanArgs a) {
  __shared__ uint64_t wl[kScanBlock / 64];
  __shared__ uint32_t wc[kScanBlock / 64];
  __shared__ uint64_t s_tile, s_pl, s_pc;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t == 0) s_tile = __hip_atomic_fetch_add(a.status, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the previous call's set, for the next call
  for (size_t i = (size_t)blockIdx.x * kScanBlock + t; i < a.other_words; i += (size_t)gridDim.x * kScanBlock)
    a.other[i] = 0;
  __syncthreads();
  const uint64_t tile = s_tile;
  const size_t p0 = tile * kStreamTile + (size_t)t * kScanPer;
  uint64_t addr[kScanPer];
  uint32_t len[kScanPer], nl[kScanPer];
  uint64_t sl = 0;
  uint32_t sc = 0;
#pragma unroll
  for (int i = 0; i < kScanPer; i++) {
    const size_t p = p0 + i;
    len[i] = p < a.n ? a.len[p] : 0u;
    addr[i] = p < a.n ? (uint64_t)(uintptr_t)a.base + a.off[p] : 0ull;
    nl[i] = len[i] ? line_count(addr[i], len[i]) : 0u;
    sl += nl[i];
    sc += len[i] ? 1u : 0u;
  }
  // block scan of (lines, count), thread-major
  uint64_t il = sl;
  uint32_t ic = sc;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t yl = (uint64_t)__shfl_up((unsigned long long)il, d);
    const uint32_t yc = (uint32_t)__shfl_up((int)ic, d);
    if (lane >= (uint32_t)d) {
      il += yl;
      ic += yc;
    }
  }
  if (lane == 63) {
    wl[wv] = il;
    wc[wv] = ic;
  }
  __syncthreads();
  uint64_t bl = 0, tl = 0;
  uint32_t bc = 0, tc = 0;
#pragma unroll
  for (uint32_t k = 0; k < kScanBlock / 64; k++) {
    if (k < wv) {
      bl += wl[k];
      bc += wc[k];
    }
    tl += wl[k];
    tc += wc[k];
  }
  if (t == 0) {
    uint64_t* rec = a.status + 8 + 8 * tile;
    uint64_t pl = 0, pc = 0;
    if (tile > 0) {
      st_relaxed(rec + 1, tl);
      st_relaxed(rec + 2, tc);
      st_release(rec, 1);
      uint32_t spins = 0;
      for (int64_t j = (int64_t)tile - 1; j >= 0;) {
        const uint64_t* r = a.status + 8 + 8 * (uint64_t)j;
        const uint64_t f = ld_acquire(r);
        if (f == 0) {
          if (++spins > kSpinMax) {
            st_relaxed(a.totals + 2, 1);  // never expected: the launch reports wrong results, not a hang
            break;
          }
          __builtin_amdgcn_s_sleep(2);
          continue;
        }
        if (f == 2) {
          pl += ld_relaxed(r + 3);
          pc += ld_relaxed(r + 4);
          break;
        }
        pl += ld_relaxed(r + 1);
        pc += ld_relaxed(r + 2);
        j--;
      }
    }
    st_relaxed(rec + 3, pl + tl);
    st_relaxed(rec + 4, pc + tc);
    st_release(rec, 2);
    if (tile == a.ntiles - 1) {
      a.totals[0] = pc + tc;
      a.totals[1] = pl + tl;
    }
    s_pl = pl;
    s_pc = pc;
  }
  __syncthreads();
  uint64_t pos = s_pl + bl + il - sl;
  uint64_t k = s_pc + bc + ic - sc;
#pragma unroll
  for (int i = 0; i < kScanPer; i++) {
    const size_t p = p0 + i;
    if (len[i]) {
      a.desc[k] = make_uint4((uint32_t)addr[i], (uint32_t)(addr[i] >> 32), len[i], (uint32_t)p);
      a.posv[k] = pos;
      k++;
      pos += nl[i];
    } else if (!UPD && p < a.n) {
      a.out[p] = 0u;  // crc of the empty string (update mode: the register is unchanged)
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// 2. The line stream. Per-lane state of one step.
struct LaneLine {
  uint64_t src;   // the line's address (the zero line for lanes past the stream)
  uint32_t li;    // line index inside the payload
  uint32_t nl;    // the payload's lines
  uint32_t len, lead, tailend, p, k;  // payload length, A % 128, bytes of the last line, index, desc index
  uint32_t state; // update mode: the register before the payload (lanes with li <= 1)
  bool valid;
};

// The payload mask of a line (var_class's masks, crc32_kernels.hip): bytes before the payload's first byte
// and after its last are zeroed; the init 0xFFFFFFFF is the complement of payload bytes [0, 4) (len >= 4;
// they may spill into line 1), and in update mode the caller's register is injected there instead.
template <bool UPD>
__device__ __forceinline__ void mask_payload_line(uint4 (&v)[8], const LaneLine& x) {
  const bool first = x.li == 0, last = x.li + 1 == x.nl;
  const bool spill = x.li == 1 && x.lead > 124 && x.len >= 4;
  if (first || spill) {
    const int32_t A8 = first ? (int32_t)x.lead * 8 : 0;
    if constexpr (UPD) {
      const int32_t S8 = ((int32_t)x.lead - (first ? 0 : 128)) * 8;
      const uint32_t reg = x.len < 4 ? 0u : x.state;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        uint32_t* w = reinterpret_cast<uint32_t*>(&v[i]);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int32_t p8 = (i * 16 + q * 4) * 8;
          const uint32_t keepA = (uint32_t)(0xFFFFFFFFull << clamp032(A8 - p8));
          const int32_t s = S8 - p8;
          const uint32_t sw = s >= 32 || s <= -32 ? 0u : (s >= 0 ? reg << s : reg >> -s);
          w[q] = (keepA & w[q]) ^ sw;
        }
      }
    } else {
      const int32_t B8 = x.len < 4 ? A8 : ((int32_t)x.lead + 4 - (first ? 0 : 128)) * 8;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        uint32_t* w = reinterpret_cast<uint32_t*>(&v[i]);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int32_t p8 = (i * 16 + q * 4) * 8;
          const uint32_t keepA = (uint32_t)(0xFFFFFFFFull << clamp032(A8 - p8));
          const uint32_t keepB = (uint32_t)(0xFFFFFFFFull << clamp032(B8 - p8));
          w[q] = keepA & (w[q] ^ ~keepB);
        }
      }
    }
  }
  if (last) {
    const int32_t H8 = (int32_t)x.tailend * 8;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint32_t* w = reinterpret_cast<uint32_t*>(&v[i]);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int32_t p8 = (i * 16 + q * 4) * 8;
        w[q] &= (uint32_t)(0xFFFFFFFFull >> clamp032(p8 + 32 - H8));
      }
    }
  }
}

// The digest from the register after a payload's last line: drop the zeros behind its last byte
// (shift_{-over}, two lane-varying maps from the U sets at `uoff`), then crc32_long's final xor, or the
// update register. Payloads shorter than 4 bytes carry their init (or register) as a constant term.
template <bool UPD>
__device__ __forceinline__ uint32_t finish_payload(uint32_t r, uint32_t tailend, uint32_t len, uint32_t state,
                                                   const uint32_t* lds, uint32_t uoff) {
  const uint32_t over = 128 - tailend;
  uint32_t t = nibble_map_set<16>(r, lds, uoff, over & 15u);
  t = nibble_map_set<8>(t, lds, uoff + (kStreamUHiOff - kStreamULoOff), over >> 4);
  if constexpr (UPD) {
    if (len < 4) t ^= shift_bits(state, 8u * len);  // <= 24 bit steps
    return t;
  } else {
    if (len < 4) {
      constexpr uint32_t k1 = shift_bits(kInit, 8), k2 = shift_bits(kInit, 16), k3 = shift_bits(kInit, 24);
      t ^= len == 1 ? k1 : (len == 2 ? k2 : k3);
    }
    return ~t;
  }
}

template <bool UPD>
__global__ __launch_bounds__(kBlock) void crc32_stream_kernel(const uint4* __restrict__ desc,
                                                              const uint64_t* __restrict__ posv,
                                                              const uint64_t* __restrict__ totals,
                                                              uint32_t* __restrict__ out, uint4* __restrict__ pieces,
                                                              const uint8_t* __restrict__ zero_line,
                                                              const uint4* __restrict__ img_slice,
                                                              const uint4* __restrict__ img_stream) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsStreamImageBytes / 16];
  __shared__ uint32_t flag_lds[kBlock];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  const uint32_t l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  volatile uint32_t* fl = flag_lds + wv * 64;
  const uint64_t W = (uint64_t)gridDim.x * (kBlock / 64), w = (uint64_t)blockIdx.x * (kBlock / 64) + wv;
  const uint64_t K = totals[0], N = totals[1];
  const uint64_t steps = (N + 63) >> 6, spw = (steps + W - 1) / W;
  const uint64_t s_begin = std::min(w * spw, steps), s_end = std::min(s_begin + spw, steps);
  const bool active = s_begin < s_end;  // wave-uniform
  const uint64_t zl = (uint64_t)(uintptr_t)zero_line;

  LaneCtx kc;
  kc.L0 = (threadIdx.x & 31) << 3;
  kc.L1 = kc.L0 | (1u << 16);
  kc.slot4 = (threadIdx.x & 31) << 2;

  // window of 64 descriptors from kb: lane l holds payload kb + l (past K: position "infinity")
  uint4 wd = make_uint4(0, 0, 0, 0);
  uint64_t wP = ~0ull;
  auto load_window = [&](uint64_t kb) __attribute__((always_inline)) {
    const uint64_t k = kb + l;
    const uint64_t kc2 = k < K ? k : (K ? K - 1 : 0);
    const uint4 d = desc[kc2];
    const uint64_t P = posv[kc2];
    wd = d;
    wP = k < K ? P : ~0ull;
  };
  // the payload of every lane's position q0 + l, from the window at kb (posv[kb] <= q0 < posv[kb + 1]);
  // returns the window base of the next step
  auto assign = [&](uint64_t q0, uint64_t kb, bool beyond, LaneLine& x) __attribute__((always_inline)) -> uint64_t {
    fl[l] = 0u;
    if (l > 0 && wP < q0 + 64) fl[(uint32_t)(wP - q0)] = 1u;  // payload starts inside the step (offsets 1..63)
    const uint32_t f = fl[l];
    const uint64_t M = __ballot(f != 0u);
    const uint32_t own = __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u)) + f;
    // window lane -> start relative to q0 (lane 0: at or before q0; lanes past the step: clamped)
    const int32_t rel_mine = l == 0 ? -(int32_t)(q0 - wP) : (int32_t)(wP < q0 + 64 ? wP - q0 : 64);
    const uint32_t a_lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(own << 2), (int)wd.x);
    const uint32_t a_hi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(own << 2), (int)wd.y);
    const uint32_t len = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(own << 2), (int)wd.z);
    const uint32_t p = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(own << 2), (int)wd.w);
    const int32_t rel = __builtin_amdgcn_ds_bpermute((int)(own << 2), rel_mine);
    const uint64_t A = ((uint64_t)a_hi << 32) | a_lo;
    const uint64_t E = A + len;
    x.li = (uint32_t)((int32_t)l - rel);
    x.nl = len ? (uint32_t)(((E - 1) >> 7) - (A >> 7) + 1) : 1u;
    x.len = len;
    x.lead = (uint32_t)(A & 127);
    x.tailend = (uint32_t)(((E - 1) & 127) + 1);
    x.p = p;
    x.k = (uint32_t)(kb + own);
    x.valid = !beyond && q0 + l < N;
    x.src = x.valid ? ((A >> 7) + x.li) << 7 : zl;
    x.state = 0u;
    if constexpr (UPD) {
      if (x.valid && x.li <= 1) x.state = out[p];
    }
    const uint32_t own63 = (uint32_t)__builtin_amdgcn_readlane((int)own, 63);
    const uint32_t open63 = (uint32_t)__builtin_amdgcn_readlane((int)(x.li + 1 < x.nl ? 1u : 0u), 63);
    return kb + own63 + (open63 ? 0u : 1u);
  };
  auto load_line = [&](const LaneLine& x, uint4 (&v)[8]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = gload16(x.src + 16 * i);
  };

  LaneLine cur{}, nxt{};
  uint4 A[8], B[8];
  uint64_t kw = 0;
  uint32_t kh = kNoPayload;  // the chunk's head payload: started before the chunk (its register starts at 0 here)
  const uint64_t Q0 = s_begin * 64;
  if (active) {
    // the payload holding Q0: 64-ary search of posv (posv[0] = 0 <= Q0)
    uint64_t lo = 0, hi = K;
    while (hi - lo > 1) {
      const uint64_t st = (hi - lo + 63) / 64;
      const uint64_t idx = lo + l * st;
      const uint64_t v = posv[idx < hi ? idx : hi - 1];
      const uint64_t m = __ballot(idx < hi && v <= Q0);
      const uint64_t j = (uint64_t)__popcll(m) - 1;
      lo += j * st;
      hi = std::min(lo + st, hi);
    }
    load_window(lo);
    const uint64_t P0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(wP >> 32), 0) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)wP, 0);
    kh = P0 < Q0 ? (uint32_t)lo : kNoPayload;
    kw = assign(Q0, lo, false, cur);
    load_line(cur, A);
    load_window(kw);
  }
  load_image<kLdsStreamImageBytes, kBlock, kLdsStreamImageBytes>(lds4, img_slice, img_stream);
  __syncthreads();
  if (!active) return;

  uint32_t C = 0;         // register of the payload open at the end of the previous step
  uint32_t head_val = 0;  // register of the head payload after its last line (if it ends in the chunk)
  uint64_t s = s_begin;
  auto compute = [&](uint4 (&v)[8], const LaneLine& x) __attribute__((always_inline)) {
    if (x.valid) mask_payload_line<UPD>(v, x);
    uint32_t r = absorb_line(0u, v, kc, lds);
    const uint32_t cm = nibble_map_uniform(C, lds, kLdsStreamOff + kStreamScanOff);  // shift_128(carry)
    r = x.valid ? r ^ (l == 0 && x.li > 0 ? cm : 0u) : 0u;
    // segmented inclusive scan over the step's positions (lanes), uniform maps shift_{d*128}
    const int32_t seg0 = x.li <= l ? (int32_t)(l - x.li) : 0;
#pragma unroll
    for (int i = 0; i < 6; i++) {
      const int d = 1 << i;
      const uint32_t y = (uint32_t)__shfl_up((int)r, d);
      const uint32_t m = nibble_map_uniform(y, lds, kLdsStreamOff + kStreamScanOff + 512 * i);
      r = (int32_t)l - d >= seg0 ? r ^ m : r;
    }
    const bool last = x.valid && x.li + 1 == x.nl;
    const bool head = x.k == kh;
    const uint64_t hm = __ballot(last && head);
    if (hm) head_val = (uint32_t)__builtin_amdgcn_readlane((int)r, (int)__builtin_ctzll(hm));
    if (last && !head) out[x.p] = finish_payload<UPD>(r, x.tailend, x.len, x.state, lds, kLdsStreamOff + kStreamULoOff);
    C = (uint32_t)__builtin_amdgcn_readlane((int)r, 63);
  };
  auto step = [&](uint4 (&cb)[8], uint4 (&nb)[8]) __attribute__((always_inline)) {
    const bool beyond = s + 1 >= s_end;
    const uint64_t kn = assign((s + 1) * 64, kw, beyond, nxt);
    load_line(nxt, nb);
    kw = kn;
    load_window(kw);
    __builtin_amdgcn_sched_barrier(0);
    compute(cb, cur);
    cur = nxt;
    s++;
  };
  while (true) {
    step(A, B);
    if (s >= s_end) break;
    step(B, A);
    if (s >= s_end) break;
  }
  // this chunk's pieces for the fixup: the head payload's register at its end (if it ends here), the
  // register of the payload open at the chunk end (C), and the head payload's index
  if (l == 0) pieces[w] = make_uint4(head_val, C, kh, 0u);
}

// ---------------------------------------------------------------------------------------------------
// 3. Payloads crossing chunk boundaries. Chunk c = positions [c * CL, (c + 1) * CL); a payload from chunk c0
// to chunk c1 > c0 has pieces: chunk c0's open register (pieces[c0].y), the whole-chunk registers of the
// chunks between (pieces[c].y, the head payload open at their end), and chunk c1's head register
// (pieces[c1].x). The owner of the payload is the boundary c0 + 1 (pieces[c0 + 1].z names it and
// pieces[c0].z does not). One wave per boundary; lanes take pieces, shift each by the lines of the payload
// after it (power maps P(i) = shift_{2^i * 128}), and xor.
template <bool UPD>
__global__ __launch_bounds__(kFixBlock) void crc32_stream_fixup_kernel(const uint4* __restrict__ desc,
                                                                       const uint64_t* __restrict__ posv,
                                                                       const uint64_t* __restrict__ totals,
                                                                       uint32_t* __restrict__ out,
                                                                       const uint4* __restrict__ pieces, uint32_t W,
                                                                       const uint4* __restrict__ img_fix) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kStreamFixupBytes / 16];
  for (uint32_t i = threadIdx.x; i < kStreamFixupBytes / 16; i += kFixBlock) lds4[i] = img_fix[i];
  __syncthreads();
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  const uint32_t l = threadIdx.x & 63;
  const uint64_t N = totals[1];
  const uint64_t steps = (N + 63) >> 6, spw = (steps + W - 1) / W;
  if (spw == 0) return;
  const uint64_t nchunks = (steps + spw - 1) / spw, CL = spw * 64;
  const uint64_t waves = (uint64_t)gridDim.x * (kFixBlock / 64);
  for (uint64_t b = 1 + (uint64_t)blockIdx.x * (kFixBlock / 64) + (threadIdx.x >> 6); b < nchunks; b += waves) {
    const uint32_t k = pieces[b].z;
    if (k == kNoPayload || pieces[b - 1].z == k) continue;  // none, or owned by an earlier boundary
    const uint4 d = desc[k];
    const uint64_t A = ((uint64_t)d.y << 32) | d.x;
    const uint32_t len = d.z, p = d.w;
    const uint64_t end = posv[k] + line_count(A, len);
    const uint64_t c1 = (end - 1) / CL, m = c1 - (b - 1) + 1;
    uint32_t acc = 0;
    for (uint64_t i0 = 0; i0 < m; i0 += 64) {
      const uint64_t i = i0 + l;
      const bool in = i < m;
      const uint64_t c = b - 1 + (in ? i : 0);
      const uint4 pc = pieces[c];
      uint32_t v = in ? (i > 0 && c == c1 ? pc.x : pc.y) : 0u;
      const uint64_t dist = in && c != c1 ? end - (c + 1) * CL : 0;
      uint64_t any = dist;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) any |= (uint64_t)__shfl_xor((unsigned long long)any, o);
      for (int bit = 0; bit < 32 && (any >> bit); bit++) {
        const uint32_t mv = nibble_map_uniform(v, lds, kStreamPowOff + 512 * bit);
        v = (dist >> bit) & 1 ? mv : v;
      }
      acc ^= v;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, o);
    const uint32_t tailend = (uint32_t)(((A + len - 1) & 127) + 1);
    const uint32_t state = UPD ? out[p] : 0u;
    const uint32_t r = finish_payload<UPD>(acc, tailend, len, state, lds, kStreamULoOff);
    if (l == 0) out[p] = r;
  }
}

}  // namespace

hipError_t launch_stream(const StreamLaunch& a, hipStream_t stream) {
  StreamScanArgs s{};
  s.base = static_cast<const uint8_t*>(a.base);
  s.off = a.off;
  s.len = a.len;
  s.n = a.n;
  s.out = a.out;
  s.desc = static_cast<uint4*>(a.desc);
  s.posv = a.posv;
  s.totals = a.totals;
  s.status = a.status;
  s.other = a.status_other;
  s.other_words = a.other_words;
  s.ntiles = a.ntiles;
  note_kernel("crc32_stream_scan_kernel");
  if (a.update)
    hipLaunchKernelGGL(crc32_stream_scan_kernel<true>, dim3(a.ntiles), dim3(kScanBlock), 0, stream, s);
  else
    hipLaunchKernelGGL(crc32_stream_scan_kernel<false>, dim3(a.ntiles), dim3(kScanBlock), 0, stream, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const unsigned blocks = (unsigned)std::max<size_t>(1, a.max_blocks);
  const uint4* desc = static_cast<const uint4*>(a.desc);
  const uint8_t* zl = static_cast<const uint8_t*>(a.zero_line);
  const uint4* img_slice = static_cast<const uint4*>(a.img_slice);
  const uint4* img_stream = static_cast<const uint4*>(a.img_stream);
  note_kernel("crc32_stream_kernel");
  if (a.update)
    hipLaunchKernelGGL(crc32_stream_kernel<true>, dim3(blocks), dim3(kBlock), 0, stream, desc, a.posv, a.totals, a.out,
                       a.pieces, zl, img_slice, img_stream);
  else
    hipLaunchKernelGGL(crc32_stream_kernel<false>, dim3(blocks), dim3(kBlock), 0, stream, desc, a.posv, a.totals, a.out,
                       a.pieces, zl, img_slice, img_stream);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const uint32_t W = blocks * (kBlock / 64);
  const unsigned fblocks = (unsigned)std::max<uint32_t>(1, std::min<uint32_t>((W + 15) / 16, 256));
  note_kernel("crc32_stream_fixup_kernel");
  if (a.update)
    hipLaunchKernelGGL(crc32_stream_fixup_kernel<true>, dim3(fblocks), dim3(kFixBlock), 0, stream, desc, a.posv, a.totals,
                       a.out, a.pieces, W, img_stream);
  else
    hipLaunchKernelGGL(crc32_stream_fixup_kernel<false>, dim3(fblocks), dim3(kFixBlock), 0, stream, desc, a.posv,
                       a.totals, a.out, a.pieces, W, img_stream);
  return hipGetLastError();
}

}  // namespace annety_crc
