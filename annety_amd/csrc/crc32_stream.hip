// Line-stream path for variable-length batches in any layout (annety_crc32_batch_var and its update form):
// every payload's absolute 128-byte lines, concatenated in payload order, form one stream of "positions",
// and the chip walks that stream in equal chunks, one chunk per wave. No sort, no length classes, no
// virtual lines: a wave step is 64 real lines whatever the length mix. Two launches:
//
//  1. crc32_stream_scan_kernel: one pass over the descriptors with a decoupled look-back scan (tiles of
//     2048 payloads, a ticket per tile, 64 predecessors inspected at once): for the k-th non-empty payload,
//     desc[k] = {address, length, index} and posv[k] = its first position; totals = {K, positions}. Empty
//     payloads get their digest (0) here.
//  2. crc32_stream_kernel: wave w takes positions [w * C, (w + 1) * C) (C = a multiple of 64 chosen on the
//     device from the total).
//     Edge phase: one lane per payload whose first or last line lies in the chunk folds those two lines
//     with the bytes outside the payload zeroed, plus the init as a register term.
//     Stream phase: per step, lane l owns position q0 + l; it finds its payload from a window of 64
//     descriptors (a start flag per position, mbcnt of the flags), folds its line whole from register 0
//     (edge lines take the edge phase's value), and the wave runs a segmented inclusive scan,
//         R_l = shift_{d*128}(R_{l-d}) ^ R_l   for d = 1, 2, ..., 32 while l - d is in l's payload,
//     whose maps are the same for every lane (broadcast LDS reads, no bank conflicts). A payload's last
//     line then holds its register; one inverse shift drops the zeros behind its last byte. The register
//     of a payload still open at the end of a step enters the next step's first line (the carry). The
//     scan of step s-1 and the payload lookup of step s+2 run inside the 16 LDS rounds of step s's fold.
//     Cross-chunk payloads: each chunk leaves its pieces (the head payload's register at its end, the
//     register of the payload open at the chunk end); the last chunk to finish a payload's pieces (a
//     counter per payload) joins them, crc = XOR_c shift_{lines after piece c}(piece c).
//
// Roofline: HBM-bound like the fixed kernels (a step reads 64 lines = 8 KiB per wave; the lines shared by
// two payloads are read twice, 2 % on BASELINE config 3). DESIGN.md §2.5.
// Reference semantics: crc32_long include/Crc32c.h:58-69, crc32_update :71-82 (UPD); math: crc32_math.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "crc32_device.h"
#include "crc32_kernels.h"
#include "crc32_math.h"

namespace annety_crc {
namespace {

constexpr int kScanBlock = 512;
constexpr int kScanPer = kStreamTile / kScanBlock;  // payloads per thread (contiguous)
static_assert(kScanPer * kScanBlock == (int)kStreamTile, "tile = block * per-thread");
constexpr uint32_t kNoPayload = 0xFFFFFFFFu;
#ifndef ANNETY_STREAM_BLOCK
#define ANNETY_STREAM_BLOCK 512
#endif
constexpr int kStreamBlock = ANNETY_STREAM_BLOCK;  // lanes per stream workgroup (one per CU: the LDS image)
// A look-back that waits this long for a predecessor tile gives up (the digests are then wrong and
// totals[2] says so) instead of hanging the GPU: a bound, never reached by a correct launch.
constexpr uint32_t kSpinMax = 1u << 20;

__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Cross-wave records (the scan's tile records, the stream launch's pieces) are written and read only with
// relaxed agent-scope atomics, which go through to the coherence point of all XCDs, and a writer orders its
// value stores before the flag or counter that publishes them by waiting for their completion. Release and
// acquire fences would write back or invalidate the whole L2 of the XCD instead (buffer_wbl2 / buffer_inv),
// at the end of every wave: 0.46 ms per config-3 step against 0.24 without them.
__device__ __forceinline__ void stores_done() { __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// 128-byte lines of a payload at absolute address a, length len > 0.
__device__ __forceinline__ uint32_t line_count(uint64_t a, uint32_t len) {
  return (uint32_t)(((a + len - 1) >> 7) - (a >> 7) + 1);
}

// ---------------------------------------------------------------------------------------------------
// 1. Scan. Status set (crc32_kernels.h StreamLaunch::status): word 0 = ticket counter, tile t's record at
// 8 + 8t: [0] flag (0 none, 1 aggregate, 2 inclusive), [1] aggregate lines, [2] aggregate count,
// [3] inclusive lines, [4] inclusive count. The set is zero when the call starts (zeroed by the previous
// call on the slot, which used the other set, or at allocation). The scan also zeroes the stream launch's
// per-payload join counters (one per chunk).
template <bool UPD>
__global__ __launch_bounds__(kScanBlock) void crc32_stream_scan_kernel(StreamScanArgs a) {
  __shared__ uint64_t wl[kScanBlock / 64];
  __shared__ uint32_t wc[kScanBlock / 64];
  __shared__ uint64_t s_tile, s_pl, s_pc;
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t == 0) s_tile = __hip_atomic_fetch_add(a.status, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the previous call's set, for the next call; this call's join counters
  for (size_t i = (size_t)blockIdx.x * kScanBlock + t; i < a.other_words; i += (size_t)gridDim.x * kScanBlock)
    a.other[i] = 0;
  for (size_t i = (size_t)blockIdx.x * kScanBlock + t; i < a.ncounters; i += (size_t)gridDim.x * kScanBlock)
    a.counters[i] = 0;
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
  if (wv == 0) {
    // look-back: lane j inspects tile (top - j); the nearest inclusive record (or the start) ends the walk,
    // the aggregates before it add up. A window with a tile that has published nothing yet is read again.
    uint64_t* rec = a.status + 8 + 8 * tile;
    uint64_t pl = 0, pc = 0;
    if (tile > 0) {
      if (lane == 0) {
        st_relaxed(rec + 1, tl);
        st_relaxed(rec + 2, tc);
        stores_done();
        st_relaxed(rec, 1);
      }
      int64_t top = (int64_t)tile - 1;
      uint32_t spins = 0;
      while (top >= 0) {
        const int64_t j = top - (int64_t)lane;
        const uint64_t* r = a.status + 8 + 8 * (uint64_t)(j >= 0 ? j : 0);
        const uint64_t f = j >= 0 ? ld_relaxed(r) : 2u;
        const uint64_t stop = __ballot(f == 2u);  // inclusive, or before tile 0
        const uint32_t end = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;
        const uint64_t none = __ballot(f == 0u) & (end < 64 ? ((2ull << end) - 1) : ~0ull);
        if (none) {
          if (++spins > kSpinMax) {
            if (lane == 0) st_relaxed(a.totals + 2, 1);  // never expected: wrong results, not a hang
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        __asm__ volatile("" ::: "memory");  // the values are read after the flags (relaxed atomics, in order)
        uint64_t vl = 0, vc = 0;
        if (j >= 0 && lane < end) {
          vl = ld_relaxed(r + 1);
          vc = ld_relaxed(r + 2);
        } else if (j >= 0 && lane == end) {
          vl = ld_relaxed(r + 3);
          vc = ld_relaxed(r + 4);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
          vl += (uint64_t)__shfl_xor((unsigned long long)vl, o);
          vc += (uint64_t)__shfl_xor((unsigned long long)vc, o);
        }
        pl += vl;
        pc += vc;
        if (end < 64) break;
        top -= 64;
      }
    }
    if (lane == 0) {
      st_relaxed(rec + 3, pl + tl);
      st_relaxed(rec + 4, pc + tc);
      stores_done();
      st_relaxed(rec, 2);
      if (tile == a.ntiles - 1) {
        a.totals[0] = pc + tc;
        a.totals[1] = pl + tl;
      }
      s_pl = pl;
      s_pc = pc;
    }
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
// 2. The line stream.
//
// Edge lines (a payload's first and last line) are the only ones with bytes outside their payload. Each
// wave first computes them for the payloads whose first or last line lies in its chunk, one lane per
// payload and both lines folded together (the edge phase): the first line with the bytes before the
// payload zeroed (and, for one-line payloads, those after it) plus the init term I[lead] = the register
// crc32_long starts from, seen from the end of that line (update mode: shift_{128-lead} of the caller's
// register); the last line with the bytes after the payload zeroed. The stream phase then folds every
// other line whole, with no per-lane masks, and takes the edge lines' values from the edge phase (their
// lanes read the zero line).
struct LaneLine {
  uint64_t src;   // the line's address (the zero line for edge lines and lanes past the stream)
  uint32_t lt;    // line index inside the payload (bits 0-24) | (bytes of the payload's last line - 1) << 25
  uint32_t nf;    // the payload's lines (bits 0-24) | valid << 30 | edge line << 31
  uint32_t p, k;  // payload index, desc index
  uint32_t edge;  // edge lines: the edge phase's value
  __device__ __forceinline__ uint32_t li() const { return lt & 0x1FFFFFFu; }
  __device__ __forceinline__ uint32_t tailend() const { return (lt >> 25) + 1; }
  __device__ __forceinline__ uint32_t nl() const { return nf & 0x1FFFFFFu; }
  __device__ __forceinline__ bool valid() const { return (nf >> 30) & 1u; }
  __device__ __forceinline__ bool is_edge() const { return nf >> 31; }
};

constexpr uint32_t kPowLds = kLdsStreamOff + kStreamPowOff;
constexpr uint32_t kULoLds = kLdsStreamOff + kStreamULoOff;
constexpr uint32_t kUHiLds = kLdsStreamOff + kStreamUHiOff;

// shift_{d * 128} for a lane-varying d < 2^32 lines: the power matrices M(i) (global, uniform: scalar loads),
// applied for the bits any lane needs and selected per lane. Only the cross-chunk join uses it.
__device__ __forceinline__ uint32_t shift_lines(uint32_t v, uint64_t d, const uint32_t* __restrict__ mats) {
  uint64_t any = d;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) any |= (uint64_t)__shfl_xor((unsigned long long)any, o);
  for (int bit = 0; bit < 32 && (any >> bit); bit++) {
    const uint32_t* M = mats + 32 * bit;
    uint32_t r = 0;
#pragma unroll
    for (int b = 0; b < 32; b++) r ^= ((v >> b) & 1u) ? M[b] : 0u;
    v = (d >> bit) & 1 ? r : v;
  }
  return v;
}

template <bool UPD, int PROBE = 0, int BLK = kStreamBlock>
__global__ __launch_bounds__(BLK) void crc32_stream_kernel(StreamArgs g) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsStreamImageBytes / 16];
  __shared__ uint32_t flag_lds[BLK];
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  const uint32_t l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // (plain LDS accesses ordered by compiler barriers: a volatile pointer here compiles to flat stores that wait
  // for every outstanding global load, i.e. for the next step's lines)
  uint32_t* fl = flag_lds + wv * 64;
  const uint64_t W = (uint64_t)gridDim.x * (BLK / 64), w = (uint64_t)blockIdx.x * (BLK / 64) + wv;
  const uint64_t K = g.totals[0], N = g.totals[1];
  const uint64_t steps = (N + 63) >> 6, spw = (steps + W - 1) / W;
  const uint64_t s_begin = std::min(w * spw, steps), s_end = std::min(s_begin + spw, steps);
  const bool active = s_begin < s_end;  // wave-uniform
  const uint64_t zl = (uint64_t)(uintptr_t)g.zero_line;
  const uint64_t CL = spw * 64;  // positions per chunk
  const uint64_t Q0 = s_begin * 64, Q1 = std::min(s_end * 64, N);
  const uint4* __restrict__ desc = g.desc;
  const uint64_t* __restrict__ posv = g.posv;
  uint32_t* __restrict__ edges = g.edges;
  uint32_t* __restrict__ out = g.out;

  LaneCtx kc;
  kc.L0 = (threadIdx.x & 31) << 3;
  kc.L1 = kc.L0 | (1u << 16);
  kc.slot4 = (threadIdx.x & 31) << 2;

  // the payload holding Q0: 64-ary search of posv (posv[0] = 0 <= Q0), before the image is staged
  uint64_t kw0 = 0;
  if (active) {
    uint64_t hi = K;
    while (hi - kw0 > 1) {
      const uint64_t st = (hi - kw0 + 63) / 64;
      const uint64_t idx = kw0 + l * st;
      const uint64_t v = posv[idx < hi ? idx : hi - 1];
      const uint64_t m = __ballot(idx < hi && v <= Q0);
      kw0 += ((uint64_t)__popcll(m) - 1) * st;
      hi = std::min(kw0 + st, hi);
    }
  }
  load_image<kLdsStreamImageBytes, BLK, kLdsStreamImageBytes>(lds4, g.img_slice, g.img_stream);
  __syncthreads();
  if (!active) return;

  // ---- edge phase: payloads kw0, kw0 + 1, ... while they start before Q1, 64 at a time ----
  for (uint64_t kb = kw0; !(PROBE & 1); kb += 64) {
    const uint64_t k = kb + l;
    const uint64_t kk = k < K ? k : K - 1;
    const uint4 d = desc[kk];
    const uint64_t P = posv[kk];
    const uint64_t A = ((uint64_t)d.y << 32) | d.x, E = A + d.z;
    const uint32_t nl = line_count(A, d.z);
    const bool in = k < K && P < Q1;
    const bool doF = in && P >= Q0, doL = in && nl >= 2 && P + nl <= Q1;
    uint4 vf[8], vl[8];
    const uint64_t fsrc = doF ? (A >> 7) << 7 : zl, lsrc = doL ? ((E - 1) >> 7) << 7 : zl;
#pragma unroll
    for (int i = 0; i < 8; i++) vf[i] = gload16(fsrc + 16 * i);
#pragma unroll
    for (int i = 0; i < 8; i++) vl[i] = gload16(lsrc + 16 * i);
    const uint32_t lead = (uint32_t)(A & 127), tailend = (uint32_t)(((E - 1) & 127) + 1);
    uint32_t state = 0;
    if constexpr (UPD) state = out[doF ? d.w : 0];
    mask_line<8>(vf, (int32_t)lead * 8, nl == 1 ? (int32_t)tailend * 8 : 1024);
    mask_line<8>(vl, 0, (int32_t)tailend * 8);
    // (one line after the other: two at once would hold 16 more registers across the whole kernel)
    uint32_t rf = absorb_line(0u, vf, kc, lds);
    const uint32_t rl = absorb_line(0u, vl, kc, lds);
    if constexpr (UPD) {
      // shift_{128-lead}(state) = shift_128(shift_{-lead}(state))
      uint32_t t = nibble_map_set<16>(state, lds, kULoLds, lead & 15u);
      t = nibble_map_set<8>(t, lds, kUHiLds, lead >> 4);
      rf ^= nibble_map_uniform(t, lds, kPowLds);
    } else {
      rf ^= lds[(kLdsStreamOff + kStreamInitOff) / 4 + lead];
    }
    if (doF) edges[2 * k] = rf;
    if (doL) edges[2 * k + 1] = rl;
    if (__ballot(!in) != 0) break;  // a payload at or past the chunk end: the later ones are too
  }
  // the stream phase reads these values back (other lanes of this wave): stores complete first
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");

  // ---- stream phase ----
  // Window of 64 descriptors from kb (lane l holds payload kb + l; past K: position "infinity"), loaded at
  // the start of the iteration whose end uses it.
  uint4 wd = make_uint4(0, 0, 0, 0);
  uint64_t wP = ~0ull;
  auto load_window = [&](uint64_t kb) __attribute__((always_inline)) {
    const uint64_t k = kb + l;
    const uint64_t kk = k < K ? k : K - 1;
    wd = desc[kk];
    const uint64_t P = posv[kk];
    wP = k < K ? P : ~0ull;
  };
  // The payload of every lane's position q0 + l, from the window at kb (posv[kb] <= q0 < posv[kb + 1]), in
  // three parts that run in the gaps of a fold; the last returns the window base of the next step.
  uint32_t as_f = 0, as_own = 0;
  auto assign1 = [&](uint64_t q0) __attribute__((always_inline)) {
    fl[l] = 0u;
    __asm__ volatile("" ::: "memory");
    // payloads that start inside the step (offsets 1..63; the bounds keep a flush step inside the flags)
    if (wP > q0 && wP < q0 + 64) fl[(uint32_t)(wP - q0)] = 1u;
  };
  auto assign2 = [&]() __attribute__((always_inline)) {
    __asm__ volatile("" ::: "memory");  // the other lanes' flags (LDS operations of one wave run in order)
    as_f = fl[l];
    const uint64_t M = __ballot(as_f != 0u);
    as_own = __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u)) + as_f;
  };
  auto assign3 = [&](uint64_t q0, uint64_t kb, bool beyond, LaneLine& x) __attribute__((always_inline)) -> uint64_t {
    const int src = (int)(as_own << 2);
    // window lane -> start relative to q0 (lane 0: at or before q0; lanes past the step: clamped)
    const int32_t rel_mine = l == 0 ? -(int32_t)(q0 - wP) : (int32_t)(wP < q0 + 64 ? wP - q0 : 64);
    const uint32_t a_lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)wd.x);
    const uint32_t a_hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)wd.y);
    const uint32_t len = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)wd.z);
    const uint32_t p = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)wd.w);
    const int32_t rel = __builtin_amdgcn_ds_bpermute(src, rel_mine);
    const uint64_t A = ((uint64_t)a_hi << 32) | a_lo;
    const uint64_t E = A + len;
    const uint32_t li = (uint32_t)((int32_t)l - rel) & 0x1FFFFFFu;
    const uint32_t nl = len ? (uint32_t)(((E - 1) >> 7) - (A >> 7) + 1) : 1u;
    const bool valid = !beyond && q0 + l < N;
    const bool is_edge = valid && (li == 0 || li + 1 == nl);
    x.lt = li | ((uint32_t)((E - 1) & 127) << 25);
    x.nf = nl | (valid ? 1u << 30 : 0u) | (is_edge ? 1u << 31 : 0u);
    x.p = p;
    x.k = (uint32_t)(kb + as_own);
    x.src = valid && !is_edge ? ((A >> 7) + li) << 7 : zl;
    // unconditional (lanes that need none read entry 0)
    x.edge = edges[is_edge ? 2 * (uint64_t)x.k + (li == 0 ? 0 : 1) : 0];
    const uint32_t own63 = (uint32_t)__builtin_amdgcn_readlane((int)as_own, 63);
    const uint32_t open63 = (uint32_t)__builtin_amdgcn_readlane((int)(li + 1 < nl ? 1u : 0u), 63);
    return kb + own63 + (open63 ? 0u : 1u);
  };
  // Coalesced loads (crc32_device.h coalesced_lane_offset): load i reads the 8 lines of positions 8i..8i+7,
  // each line by 8 lanes, 16 bytes each; lane l reads piece c(l) of the line of position 8i + (l & 7), whose
  // address it takes from that position's lane. A block of consecutive lines of one payload is one 1 KiB
  // read; the loads are nontemporal (the config-1 kernel's access shape). Per-line loads (each lane its own
  // line: 64 lines per instruction) left the line-stream kernel issue-bound on the vector memory pipeline.
  const uint32_t piece = coalesced_lane_offset(l) & 127u;
  auto load_lines = [&](const LaneLine& x, uint4 (&v)[8]) __attribute__((always_inline)) {
    uint64_t a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int from = (int)((8 * i + (l & 7)) << 2);
      const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)(uint32_t)x.src);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(from, (int)(uint32_t)(x.src >> 32));
      a[i] = (((uint64_t)hi << 32) | lo) + piece;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const v4u32 d = __builtin_nontemporal_load(reinterpret_cast<const __attribute__((address_space(1))) v4u32*>(a[i]));
      v[i] = make_uint4(d.x, d.y, d.z, d.w);
    }
  };
  // after transpose_blocks(): lane l holds line l & 7 of block folded_block(l), i.e. position
  // 8 * folded_block(l) + (l & 7); position m's lane:
  const uint32_t m3 = l >> 3;
  const int pos_lane = (int)(((l & 7) | ((m3 >> 2) << 3) | ((m3 & 1) << 4) | (((m3 >> 1) & 1) << 5)) << 2);
  const uint32_t l3 = (l >> 3) & 1;

  const uint32_t kh = posv[kw0] < Q0 ? (uint32_t)kw0 : kNoPayload;  // the chunk's head payload (register 0 here)
  uint32_t C = 0;           // register of the payload open at the end of the latest scanned step
  uint32_t head_val = 0;    // register of the head payload after its last line (if it ends in the chunk)
  uint32_t open_k = kNoPayload;  // the payload open at the end of the latest scanned step

  // Pipeline. Iteration s: issue the window of step s + 2 and the lines of step s + 1; transpose and fold
  // step s in 16 LDS rounds and, in the gaps, scan and finish step s - 1 and look up step s + 2. Step s_end is
  // a flush (its lanes are past the chunk, its lines the zero line) whose iteration scans step s_end - 1.
  LaneLine prev{}, cur{}, nxt{}, nn{};
  prev.nf = 1u;
  uint32_t r_prev = 0;
  uint4 A[8], B[8];
  load_window(kw0);
  assign1(Q0);
  assign2();
  uint64_t kw = assign3(Q0, kw0, false, cur);
  load_window(kw);
  load_lines(cur, A);
  assign1(Q0 + 64);
  assign2();
  kw = assign3(Q0 + 64, kw, s_begin + 1 >= s_end, nxt);
  uint64_t s = s_begin;
  // The fold as two 64-byte chains in 16 LDS rounds; the scan as a Kogge-Stone over the wave (a shuffle and a
  // map per level). Measured against a four-chain fold with a two-phase scan (DPP inside 16-lane rows, then
  // the rows' carries through lane-position maps), same box: 279 against 287 us per config-3 call
  // (microbench/stream_probe.py, profiles/r04/README.md).
  auto iter = [&](uint4 (&cb)[8], uint4 (&nb)[8]) __attribute__((always_inline)) {
    const uint64_t kb2 = kw;
    load_window(kb2);
    load_lines(nxt, nb);
    __builtin_amdgcn_sched_barrier(0);
    transpose_blocks(cb);
    uint32_t xa = cb[0].x, xb = cb[4].x;
    uint32_t R = 0, y = 0, m = 0, cm = 0, t = 0;
    const int32_t seg0 = prev.li() <= l ? (int32_t)(l - prev.li()) : 0;
    const bool last = prev.valid() && prev.li() + 1 == prev.nl();
    const bool head = prev.k == kh;
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const int i = q >> 2, wq = q & 3;
      const uint32_t wa = wq == 0 ? cb[i].y : wq == 1 ? cb[i].z : wq == 2 ? cb[i].w : (i + 1 < 4 ? cb[i + 1].x : 0u);
      const uint32_t wb = wq == 0 ? cb[4 + i].y : wq == 1 ? cb[4 + i].z : wq == 2 ? cb[4 + i].w : (i + 1 < 4 ? cb[5 + i].x : 0u);
      if constexpr (PROBE & 4) {
        xa = (xa * 0x9E3779B1u) ^ wa;
        xb = (xb * 0x9E3779B1u) ^ wb;
      } else {
        word4x2(xa, wa, xb, wb, kc);
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((PROBE & 2) != 0) {
        if (q == 14) assign1((s + 2) * 64);
        if (q == 15) {
          assign2();
          if (prev.valid() && prev.li() + 1 == prev.nl() && prev.k != kh) out[prev.p] = r_prev;
        }
        C = r_prev;
        __builtin_amdgcn_sched_barrier(0);
        continue;
      }
      // the scan of step s - 1: one LDS round per level half (shuffle, then map)
      // (odd q: level (q-3)/2 applies its map, then level (q-1)/2 shuffles; even q: level (q-2)/2 maps)
      if (q == 0) cm = nibble_map_uniform(C, lds, kPowLds);  // shift_128(carry)
      if (q == 1) {
        R = prev.is_edge() ? prev.edge : r_prev;
        R = prev.valid() ? R ^ (l == 0 && prev.li() > 0 ? cm : 0u) : 0u;
      }
      if (q >= 3 && q <= 13 && (q & 1)) R = (int32_t)l - (1 << ((q - 3) >> 1)) >= seg0 ? R ^ m : R;
      if (q >= 1 && q <= 11 && (q & 1)) y = (uint32_t)__shfl_up((int)R, 1 << ((q - 1) >> 1));
      if (q >= 2 && q <= 12 && !(q & 1)) m = nibble_map_uniform(y, lds, kPowLds + 512 * ((q - 2) >> 1));
      if (q == 13) {
        const uint64_t hm = __ballot(last && head);
        if (hm) head_val = (uint32_t)__builtin_amdgcn_readlane((int)R, (int)__builtin_ctzll(hm));
        C = (uint32_t)__builtin_amdgcn_readlane((int)R, 63);
        const bool open = prev.valid() && prev.li() + 1 < prev.nl();
        open_k = (uint32_t)__builtin_amdgcn_readlane((int)(open ? prev.k : kNoPayload), 63);
        t = nibble_map_set<16>(R, lds, kULoLds, (128 - prev.tailend()) & 15u);
      }
      if (q == 14) {
        t = nibble_map_set<8>(t, lds, kUHiLds, (128 - prev.tailend()) >> 4);
        assign1((s + 2) * 64);
      }
      if (q == 15) {
        if (last && !head) out[prev.p] = UPD ? t : ~t;
        assign2();
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    const uint32_t send = l3 ? xa : xb;
    const uint32_t got = (uint32_t)__builtin_amdgcn_mov_dpp((int)send, 0x128, 0xF, 0xF, false);
    const uint32_t first = l3 ? got : xa, second = l3 ? xb : got;
    const uint32_t r_line = nibble_map_uniform(first, lds, kLdsHalfOff) ^ second;
    const uint32_t r_cur = (uint32_t)__builtin_amdgcn_ds_bpermute(pos_lane, (int)r_line);
    kw = assign3((s + 2) * 64, kb2, s + 2 >= s_end, nn);
    r_prev = r_cur;
    prev = cur;
    cur = nxt;
    nxt = nn;
    s++;
  };
  while (true) {
    iter(A, B);
    if (s > s_end) break;
    iter(B, A);
    if (s > s_end) break;
  }

  // ---- payloads crossing chunk boundaries ----
  // This chunk's pieces: the head payload's register at its end (if it ends here) and the register of the
  // payload open at the chunk end. A payload from chunk c0 to c1 > c0 has c1 - c0 + 1 pieces; every chunk
  // that holds one bumps the payload's counter (at its start chunk c0), and the last to arrive joins them.
  const uint32_t kt = open_k;
  if (l == 0) {
    uint64_t* pw = reinterpret_cast<uint64_t*>(g.pieces + w);
    st_relaxed(pw, ((uint64_t)C << 32) | head_val);
    st_relaxed(pw + 1, ((uint64_t)kt << 32) | kh);
  }
  stores_done();
  for (int part = 0; part < 2; part++) {
    const uint32_t k = part == 0 ? kh : (kt != kh ? kt : kNoPayload);
    if (k == kNoPayload) continue;
    const uint4 d = desc[k];
    const uint64_t A0 = ((uint64_t)d.y << 32) | d.x;
    const uint64_t P = posv[k], end = P + line_count(A0, d.z);
    const uint64_t c0 = P / CL, c1 = (end - 1) / CL, need = c1 - c0 + 1;
    uint32_t old = 0;
    if (l == 0) old = __hip_atomic_fetch_add(g.counters + c0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    old = (uint32_t)__builtin_amdgcn_readfirstlane((int)old);
    if (old + 1 != need) continue;
    __asm__ volatile("" ::: "memory");
    uint32_t acc = 0;
    for (uint64_t i0 = 0; i0 < need; i0 += 64) {
      const uint64_t i = i0 + l;
      const bool in = i < need;
      const uint64_t c = c0 + (in ? i : 0);
      const uint64_t pc = ld_relaxed(reinterpret_cast<const uint64_t*>(g.pieces + c));  // {head_val, C}
      const uint32_t v = in ? (i > 0 && c == c1 ? (uint32_t)pc : (uint32_t)(pc >> 32)) : 0u;
      acc ^= shift_lines(v, in && c != c1 ? end - (c + 1) * CL : 0, g.mats);
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc ^= (uint32_t)__shfl_xor((int)acc, o);
    const uint32_t over = 128 - (uint32_t)(((A0 + d.z - 1) & 127) + 1);
    uint32_t r = nibble_map_set<16>(acc, lds, kULoLds, over & 15u);
    r = nibble_map_set<8>(r, lds, kUHiLds, over >> 4);
    if (l == 0) out[d.w] = UPD ? r : ~r;
  }
}

}  // namespace

hipError_t launch_stream(const StreamLaunch& a, hipStream_t stream) {
  const unsigned blocks = (unsigned)std::max<size_t>(1, a.max_blocks);
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
  s.counters = a.counters;
  s.ncounters = (size_t)blocks * (kStreamBlock / 64);
  note_kernel("crc32_stream_scan_kernel");
  if (a.update)
    hipLaunchKernelGGL(crc32_stream_scan_kernel<true>, dim3(a.ntiles), dim3(kScanBlock), 0, stream, s);
  else
    hipLaunchKernelGGL(crc32_stream_scan_kernel<false>, dim3(a.ntiles), dim3(kScanBlock), 0, stream, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  StreamArgs g{};
  g.desc = static_cast<const uint4*>(a.desc);
  g.posv = a.posv;
  g.totals = a.totals;
  g.edges = a.edges;
  g.out = a.out;
  g.pieces = a.pieces;
  g.counters = a.counters;
  g.zero_line = static_cast<const uint8_t*>(a.zero_line);
  g.img_slice = static_cast<const uint4*>(a.img_slice);
  g.img_stream = static_cast<const uint4*>(a.img_stream);
  g.mats = reinterpret_cast<const uint32_t*>(static_cast<const char*>(a.img_stream) + kStreamMatOff);
  note_kernel("crc32_stream_kernel");
  static const int probe = [] {
    const char* e = std::getenv("ANNETY_CRC_STREAM_PROBE");
    return e && *e ? std::atoi(e) : 0;
  }();
  if (a.update) {
    hipLaunchKernelGGL(crc32_stream_kernel<true>, dim3(blocks), dim3(kStreamBlock), 0, stream, g);
  } else {
    switch (probe) {
      case 1: hipLaunchKernelGGL((crc32_stream_kernel<false, 1>), dim3(blocks), dim3(kStreamBlock), 0, stream, g); break;
      case 2: hipLaunchKernelGGL((crc32_stream_kernel<false, 2>), dim3(blocks), dim3(kStreamBlock), 0, stream, g); break;
      case 3: hipLaunchKernelGGL((crc32_stream_kernel<false, 3>), dim3(blocks), dim3(kStreamBlock), 0, stream, g); break;
      case 4: hipLaunchKernelGGL((crc32_stream_kernel<false, 4>), dim3(blocks), dim3(kStreamBlock), 0, stream, g); break;
      case 7: hipLaunchKernelGGL((crc32_stream_kernel<false, 7>), dim3(blocks), dim3(kStreamBlock), 0, stream, g); break;
      default: hipLaunchKernelGGL((crc32_stream_kernel<false>), dim3(blocks), dim3(kStreamBlock), 0, stream, g);
    }
  }
  return hipGetLastError();
}

}  // namespace annety_crc
