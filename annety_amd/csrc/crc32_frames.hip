// Frame-level kernels for annety's LengthHeaderCodec wire format:
//   [length: T bytes, big-endian, T = 1/2/4/8][payload: length - 4 bytes][crc32(payload): 4 bytes BE]
// (include/codec/LengthHeaderCodec.h:33-46 layout, decode :71-137, encode :146-201; the big-endian
// integers are NetBuffer::append_int*/peek_int*, include/NetBuffer.h:38-105).
// Verify takes the CRCs from the batch kernels (crc32_kernels.hip; the arena stitch compares the trailers itself)
// and compares the 4-byte trailers; encode (lhc_encode_fused_kernel) reads each payload once and writes its whole
// frame, CRC included.
#include <hip/hip_runtime.h>

#include "crc32_device.h"
#include "crc32_kernels.h"
#include "crc32_math.h"

#include <algorithm>

namespace annety_crc {
namespace {

// Nontemporal 16-byte load from a per-lane 64-bit address (the 4-lane encode: a block's two groups, two bases).
__device__ __forceinline__ uint4 gload16_nt_at(uint64_t a) {
  const v4u32 x = __builtin_nontemporal_load((const __attribute__((address_space(1))) v4u32*)a);
  return make_uint4(x.x, x.y, x.z, x.w);
}

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
// once, with the coalesced 1 KiB loads of the sorted path (crc32_kernels.hip var_class_w8), and each frame written
// once, with coalesced 16-byte stores at the frame's byte shift. One lane group of G = 8 (or 4, round 6: chosen per
// call from sampled lengths, lhc_encode_fused_kernel) per frame (frames i = group, group + groups, ...), the payload
// [A, E) cut into VIRTUAL lines of 128 bytes from a0 = A rounded down to 16: every load is an aligned 16-byte chunk
// (the chunks past the payload's last one re-read it, so no load leaves the payload's chunks), and only the lead =
// A - a0 < 16 bytes before the payload and the bytes after E need masks. Rounds as var_class_w8 (a head round of
// the first h lines, start-aligned, then rounds of G lines).
//   * the copy, before the transpose: a chunk wholly inside the payload is stored as it is at its source address +
//     (destination - A), unaligned; the <= 2 partial chunks of a frame (loaded once more, by lanes 0 and 1 of the
//     group, with the round) store their payload bytes as 8/4/2/1-byte pieces;
//   * the CRC: var_class_w8's round (transpose, fold, masked head and last rounds), the init as the register
//     shift_{128-lead}(init) of line 0, the join and the inverse shift of the last line's overhang;
//   * the group's last lane stores the T header bytes and the 4 trailer bytes (big-endian) when the frame ends.
// Frames the reference would not write (empty, or length outside [enc_min, enc_max]) get no bytes (the host plan
// gave them none); they read the library's zero line. Algorithmic traffic: the payload read once, the frame
// written once.
struct EncW {
  uint64_t A, Dp;  // payload [A, E = A + L), payload destination (frame start + T)
  uint32_t L, te, h, R;
  bool live, valid;  // live: an index of the batch; valid: a frame to write
  __device__ __forceinline__ uint64_t E() const { return A + L; }
  __device__ __forceinline__ uint64_t a0() const { return A & ~15ull; }  // virtual line 0
  __device__ __forceinline__ uint32_t lead() const { return (uint32_t)A & 15u; }
};
template <int G>
__device__ __forceinline__ EncW decode_encw(const uint8_t* src, uint8_t* dst, uint64_t soff, uint32_t L,
                                            uint64_t foff, int T, int64_t enc_min, int64_t enc_max, bool live,
                                            uint64_t zero_line) {
  EncW k;
  k.live = live;
  k.valid = live && L > 0 && (int64_t)L >= enc_min && !(enc_max > 0 && (int64_t)L > enc_max);
  k.L = k.valid ? L : 16u;  // (16 bytes of the zero line)
  k.A = k.valid ? (uint64_t)(uintptr_t)(src + soff) : zero_line;
  k.Dp = (uint64_t)(uintptr_t)(dst + foff) + (uint32_t)T;
  const uint64_t span = (uint64_t)k.lead() + k.L;
  const uint32_t nl = (uint32_t)((span + 127) >> 7);
  k.te = (uint32_t)(span - 128ull * (nl - 1));
  k.h = ((nl - 1) & (G - 1)) + 1;
  k.R = (nl - k.h) / G + 1;
  return k;
}
// round r's first byte (rounds of G lines after the head round's h)
template <int G>
__device__ __forceinline__ uint64_t encw_round(const EncW& k, uint32_t r) {
  return k.a0() + (r == 0 ? 0ull : (uint64_t)k.h * 128u + (uint64_t)(r - 1) * (128u * G));
}

// The long path's claim (crc32_kernels.h EncLong), by a frame's lane group (its 8 lanes alike; want false: no
// claim). Lane 0 takes an entry and the frame's S segment descriptors from the counter (a compare-and-swap, so a
// claim past either cap takes nothing); the group writes the descriptors in crc32_var_sorted_kernel's segment
// format (crc32_arena.hip crc32_bucket_place: end-aligned, the first takes the remainder, m = segments after it)
// and the entry, and presets the digest the segments xor into. Returns whether the frame was taken.
template <int G>
__device__ __forceinline__ bool enc_hand_over(const EncLong& lg, uint64_t A, uint64_t Dp, uint32_t L, uint32_t t,
                                              bool want, uint32_t l) {
  const uint32_t seg = (uint64_t)L > (uint64_t)kSplitSeg * (kSplitMaxSegs - 1) ? kSplitSegBig : kSplitSeg;
  const uint32_t S = (uint32_t)(((uint64_t)L + seg - 1) / seg);
  uint32_t e = ~0u, b = 0;
  if (want && (l & (G - 1)) == 0) {
    unsigned long long old = __hip_atomic_load(lg.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (true) {
      const uint32_t segs = (uint32_t)old, ents = (uint32_t)(old >> 32);
      if (ents >= kEncLongCap || (uint64_t)segs + S > kEncLongSegCap) break;
      const unsigned long long prev = atomicCAS(lg.ctr, old, old + ((1ull << 32) | S));
      if (prev == old) {
        e = ents;
        b = segs;
        break;
      }
      old = prev;
    }
  }
  e = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * (l & ~(uint32_t)(G - 1))), (int)e);
  b = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(4 * (l & ~(uint32_t)(G - 1))), (int)b);
  if (!want || e == ~0u) return false;
  const uint32_t l0 = L - (S - 1) * seg;
  const uint32_t big = seg == kSplitSegBig ? kSegBig : 0u;
  uint4* desc = static_cast<uint4*>(lg.desc);
  for (uint32_t k = l & (G - 1); k < S; k += G) {
    const uint64_t ak = k == 0 ? A : A + l0 + (uint64_t)(k - 1) * seg;
    desc[b + k] = make_uint4((uint32_t)ak, (uint32_t)(ak >> 32) | ((S - 1 - k) << 16), k == 0 ? l0 : seg,
                             kSegFlag | (k == 0 ? kSegFirst : 0u) | big | e);
    lg.seg_dst[b + k] = Dp + (ak - A);
  }
  if ((l & (G - 1)) == 0) {
    lg.entry[e] = t;
    lg.digest[e] = ~0u;
  }
  return true;
}

// The frames the fused kernel handed over (digests from crc32_var_sorted_kernel): the copy runs over the segment
// descriptors, a block per segment (its descriptor and destination loaded an iteration ahead, its first 4 x 256
// chunks before any store). The destination is cut into aligned 16-byte chunks of the FRAME: a segment owns
// the chunks that start inside it (the first segment also the one holding the payload's first byte), so a chunk
// that straddles two segments is whole, loaded from two aligned source chunks and stored once after a byte funnel,
// and only the payload's first and last chunks are partial (their bytes stored one by one). Thread e < frames
// stores frame e's header and trailer (as the fused kernel does). Block 0 zeroes the next call's counter.
constexpr int kEncLongBlock = 256;
constexpr int kEncLongPer = 4;  // chunks per thread and segment in flight (a 16 KiB segment: 1024 chunks)
struct EncSeg {
  uint64_t lo;      // the segment's first owned chunk
  uint64_t nc;      // owned chunks
  uint64_t Df, Ef;  // the payload's destination bounds where the segment holds them (else 0 / ~0)
  uint64_t delta;   // destination - source
  uint64_t safe;    // the aligned source chunk holding the segment's first byte (the address of loads not used)
};
struct EncChunk {
  uint64_t dc;  // destination chunk address
  uint4 x0, x1;
  uint32_t o;   // source byte offset in x0:x1
  bool whole, on;
};
__device__ __forceinline__ void enc_chunk_load(EncChunk& ch, const EncSeg& g, uint64_t q, bool on) {
  ch.dc = g.lo + 16 * q;
  ch.on = on && q < g.nc;
  ch.whole = ch.on && ch.dc >= g.Df && ch.dc + 16 <= g.Ef;
  const uint64_t sp = ch.dc - g.delta, sa = sp & ~15ull;
  ch.o = (uint32_t)sp & 15u;
  // unconditional loads (a select of the second load made the compiler wait for the first): a chunk that is not
  // whole loads the segment's first source chunk; the second load is the next source chunk when o > 0 (it holds a
  // payload byte then), else the first again. Nontemporal: every byte is read once, by one or two neighbouring lanes.
  const uint64_t l0 = ch.whole ? sa : g.safe;
  ch.x0 = gload16_nt(l0, 0);
  ch.x1 = gload16_nt(l0, ch.whole && ch.o ? 16u : 0u);
}
__device__ __forceinline__ void enc_chunk_store(const EncChunk& ch) {
  if (ch.whole) {
    const uint32_t w[8] = {ch.x0.x, ch.x0.y, ch.x0.z, ch.x0.w, ch.x1.x, ch.x1.y, ch.x1.z, ch.x1.w};
    const uint32_t qd = ch.o >> 2, sh = ch.o & 3u;
    uint32_t y[5];
#pragma unroll
    for (int k = 0; k < 5; k++) y[k] = qd == 0 ? w[k] : (qd == 1 ? w[k + 1] : (qd == 2 ? w[k + 2] : w[k + 3]));
    gstore16_nt(ch.dc, make_uint4(__builtin_amdgcn_alignbyte(y[1], y[0], sh), __builtin_amdgcn_alignbyte(y[2], y[1], sh),
                                  __builtin_amdgcn_alignbyte(y[3], y[2], sh), __builtin_amdgcn_alignbyte(y[4], y[3], sh)));
  }
}
// The payload's first or last chunk when it is partial: the <= 2 aligned source chunks holding its payload bytes
// (both hold one, so no load leaves the payload's chunks), then the bytes one by one.
__device__ __forceinline__ void enc_chunk_partial(uint64_t dc, const EncSeg& g) {
  const uint64_t b0 = dc > g.Df ? dc : g.Df, b1 = dc + 16 < g.Ef ? dc + 16 : g.Ef;
  const uint64_t g0 = (b0 - g.delta) & ~15ull, g1 = (b1 - 1 - g.delta) & ~15ull;
  const uint4 y0 = gload16(g0), y1 = g1 != g0 ? gload16(g1) : y0;
  for (uint64_t x = b0; x < b1; x++) {
    const uint32_t i = (uint32_t)(x - g.delta - g0), q = (i >> 2) & 3u;
    const uint4 y = i < 16 ? y0 : y1;
    const uint32_t wd = q == 0 ? y.x : (q == 1 ? y.y : (q == 2 ? y.z : y.w));
    gstore1(x, wd >> (8 * (i & 3u)));
  }
}
__global__ __launch_bounds__(kEncLongBlock, 4) void lhc_encode_long_kernel(const uint32_t* __restrict__ len, int T,
                                                                     uint8_t* __restrict__ dst,
                                                                     const uint64_t* __restrict__ dst_off,
                                                                     EncLong lg) {
  const unsigned long long cv = *lg.ctr;
  const uint32_t ents = min((uint32_t)(cv >> 32), kEncLongCap), segs = min((uint32_t)cv, kEncLongSegCap);
  if (blockIdx.x == 0 && threadIdx.x == 0) *lg.ctr_next = 0ull;
  const uint32_t c = threadIdx.x, nb = gridDim.x;
  const uint4* desc = static_cast<const uint4*>(lg.desc);
  // the block's next segment's descriptor and destination are loaded one iteration ahead
  uint4 dn = make_uint4(0, 0, 0, 0);
  uint64_t Dn = 0;
  if (blockIdx.x < segs) {
    dn = desc[blockIdx.x];
    Dn = lg.seg_dst[blockIdx.x];
  }
  for (uint32_t k = blockIdx.x; k < segs; k += nb) {
    const uint4 d = dn;
    const uint64_t D0 = Dn;
    const uint32_t kn = k + nb < segs ? k + nb : k;
    dn = desc[kn];
    Dn = lg.seg_dst[kn];
    EncSeg g;
    const uint64_t a = ((uint64_t)(d.y & 0xFFFFu) << 32) | d.x, E0 = D0 + d.z;
    const bool first = (d.w & kSegFirst) != 0, last = (d.y >> 16) == 0;
    g.lo = first ? D0 & ~15ull : (D0 + 15) & ~15ull;
    g.nc = ((((E0 - 1) & ~15ull) - g.lo) >> 4) + 1;
    g.Df = first ? D0 : 0ull;
    g.Ef = last ? E0 : ~0ull;
    g.delta = D0 - a;
    g.safe = a & ~15ull;
    EncChunk ch[kEncLongPer];
#pragma unroll
    for (int v = 0; v < kEncLongPer; v++) enc_chunk_load(ch[v], g, c + v * kEncLongBlock, true);
#pragma unroll
    for (int v = 0; v < kEncLongPer; v++) enc_chunk_store(ch[v]);
    // the rest of the segment's whole chunks (the 1 MiB segments')
    for (uint64_t q = c + kEncLongPer * kEncLongBlock; q < g.nc; q += kEncLongBlock) {
      EncChunk x;
      enc_chunk_load(x, g, q, true);
      enc_chunk_store(x);
    }
    // the payload's partial first chunk (thread 0) and last chunk (thread 1; thread 0 when it is the first too)
    if ((first && c == 0) || (last && c == 1 && !(first && g.nc == 1))) {
      const uint64_t dc = g.lo + 16 * (c == 0 ? 0ull : g.nc - 1);
      if (!(dc >= g.Df && dc + 16 <= g.Ef)) enc_chunk_partial(dc, g);
    }
  }
  const uint64_t gt = blockIdx.x * (uint64_t)kEncLongBlock + threadIdx.x, gs = (uint64_t)gridDim.x * kEncLongBlock;
  for (uint64_t e = gt; e < ents; e += gs) {
    const uint32_t i = lg.entry[e];
    const uint32_t L = len[i];
    const uint64_t D = (uint64_t)(uintptr_t)(dst + dst_off[i]) + (uint32_t)T;
    gstore4(D + L, __builtin_bswap32(lg.digest[e]));  // the trailer, big-endian
    const uint64_t hdr = (uint64_t)L + 4, hp = D - (uint64_t)T;
    if (T == 1) gstore1(hp, (uint32_t)hdr);
    else if (T == 2) gstore2(hp, __builtin_bswap32((uint32_t)hdr) >> 16);
    else if (T == 4) gstore4(hp, __builtin_bswap32((uint32_t)hdr));
    else gstore8(hp, __builtin_bswap64(hdr));
  }
}

// 512 lanes per block (2 waves per SIMD over the one LDS image). 768 lanes (3 per SIMD) measured 0.588 against
// 0.637 ms on chat frames and 0.676 against 0.682 on mixed ones, but spill (the kernel needs ~175 VGPRs of 168).
constexpr int kEncBlock = 512;
//   PROBE (A/B builds only, microbench: wrong frames): bit 0 = no copy stores, bit 1 = no CRC (the data are xored
//   into the register, the trailer still stored), bit 2 = no partial-chunk pieces, bit 3 = no whole-chunk stores,
//   bit 5 = whole chunks always stored temporally (the product stores those of frames >= 2 KiB nontemporally).
//   G: lanes per frame, 8 (rounds of 1 KiB) or 4 (rounds of 512 bytes: a frame of up to 4 lines - 408-byte chat
//   frames - fills its round instead of half of it). With G = 4 a coalesced 1 KiB load (block i) carries the rounds
//   of two groups, lines 0-3 and 4-7: groups 2 m(i) and 2 m(i) + 1.
template <int PROBE, int G>
__device__ __forceinline__ void encode_frames(uint4* lds4, const uint8_t* __restrict__ src,
                                              const uint64_t* __restrict__ src_off, const uint32_t* __restrict__ len,
                                              size_t n, int T, int64_t enc_min, int64_t enc_max,
                                              uint8_t* __restrict__ dst, const uint64_t* __restrict__ dst_off,
                                              uint64_t zero_line, const uint4* __restrict__ img_slice,
                                              const uint4* __restrict__ img_w8, const EncLong& lg) {
  static_assert(G == 8 || G == 4, "lane groups of 8 or 4");
  constexpr uint32_t kImg = G == 8 ? kLdsW8ImageBytes : kLdsEnc4ImageBytes;
  constexpr uint32_t kRoundOff = G == 8 ? kLdsW8RoundOff : kLdsW8Round4Off;  // byte tables of shift_{(G-1)*128}
  constexpr uint32_t kRound = 128u * G;                                      // bytes per round
  const uint32_t* lds = reinterpret_cast<const uint32_t*>(lds4);
  // j: this lane's line in its group's round; hi: (G = 4) the lane's line is in the second group of its block
  const uint32_t l = threadIdx.x & 63, l3 = (l >> 3) & 1, j = l & (G - 1);
  const bool hi = G == 4 && (l & 4u) != 0;
  const size_t gid = group_id<kEncBlock, G, kVwg>();
  const size_t ngroups = ((size_t)gridDim.x * kEncBlock) / G;
  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = 0;
  // line l & 7, chunk 4 l3 + 2 l5 + l4 of a 1 KiB block; its offset in the lane's group's round
  const uint32_t voff = coalesced_lane_offset(l) - (hi ? 512u : 0u);
  auto fetch = [&](size_t t, uint64_t& so, uint32_t& ln, uint64_t& fo) __attribute__((always_inline)) {
    const size_t tc = t < n ? t : n - 1;  // unconditional: past the end re-read the last frame's fields
    so = src_off[tc];
    ln = len[tc];
    fo = dst_off[tc];
  };
  // a frame of more than kEncLongMin bytes that finds room on the long path (crc32_kernels.h EncLong) is handed
  // over there and idles here (decoded as an empty frame); called with the group's 8 lanes alike
  auto dec = [&](size_t t, uint64_t so, uint32_t ln, uint64_t fo) __attribute__((always_inline)) {
    EncW d = decode_encw<G>(src, dst, so, ln, fo, T, enc_min, enc_max, t < n, zero_line);
    const bool want = d.valid && d.L > kEncLongMin;
    if (__builtin_amdgcn_ballot_w64(want) != 0 && enc_hand_over<G>(lg, d.A, d.Dp, d.L, (uint32_t)t, want, l))
      d = decode_encw<G>(src, dst, so, 0u, fo, T, enc_min, enc_max, t < n, zero_line);
    return d;
  };
  // Load i reads the round of group m(i) = (i >> 2) + 2 (i & 1) + 4 ((i >> 1) & 1) (var_class_w8's order); a lane's
  // chunk past the group's last one re-reads that one (lim: the last chunk's offset in the round)
  // pc: lane 0 of a group loads the payload's first chunk in the head round, lane 1 its last one in the last round
  // (the partial chunks, stored piecewise), the other lanes the round's first chunk (unused)
  auto load = [&](const EncW& tk, uint32_t r, uint4 (&v)[8], uint4& pc) __attribute__((always_inline)) {
    const uint64_t rb = encw_round<G>(tk, r);
    pc = gload16(j == 0 && r == 0 ? tk.a0() : (j == 1 && r + 1 == tk.R ? (tk.E() - 1) & ~15ull : rb));
    const uint64_t last = ((tk.E() - 1) & ~15ull) - rb;
    const uint32_t lim = last < kRound - 16 ? (uint32_t)last : kRound - 16;
    const uint32_t lo = (uint32_t)rb, hw = (uint32_t)(rb >> 32);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int sl = 8 * ((i >> 2) + 2 * (i & 1) + 4 * ((i >> 1) & 1));
      if constexpr (G == 8) {
        const uint64_t g = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hw, sl) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)lo, sl);
        const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)lim, sl);
        v[i] = gload16_nt(g, min(voff, c));
      } else {  // the block's two groups: lanes sl .. sl + 3 and sl + 4 .. sl + 7
        const uint64_t g0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hw, sl) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)lo, sl);
        const uint64_t g1 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hw, sl + 4) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)lo, sl + 4);
        const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)lim, sl);
        const uint32_t c1 = (uint32_t)__builtin_amdgcn_readlane((int)lim, sl + 4);
        v[i] = gload16_nt_at((hi ? g1 : g0) + min(voff, hi ? c1 : c0));
      }
    }
  };

  size_t tL = gid;
  if (!__syncthreads_or(tL < n)) return;
  uint64_t so, fo;
  uint32_t ln;
  fetch(tL, so, ln, fo);
  EncW dL = dec(tL, so, ln, fo);
  uint64_t sn, fn;
  uint32_t lnn;
  fetch(tL + ngroups, sn, lnn, fn);
  uint4 A[8], B[8], pA, pB;
  load(dL, 0, A, pA);
  EncW dC = dL;
  uint32_t rC = 0, rL = 1;
  load_image<kImg, kEncBlock, kLdsCommonBytes>(lds4, img_slice, nullptr, img_w8);
  __syncthreads();

  // bytes [lo, hi) of x (lo < hi <= 16) to addr .. addr + hi - lo, as 8/4/2/1-byte pieces
  auto store_piece = [&](uint64_t addr, uint4 x, uint32_t lo, uint32_t hi, bool on) __attribute__((always_inline)) {
    // x >> 8 lo: dword q + (lo >> 2) funnel-shifted by lo & 3 bytes
    const uint32_t w[8] = {x.x, x.y, x.z, x.w, 0u, 0u, 0u, 0u};
    const uint32_t q = lo >> 2, sh = lo & 3;
    uint32_t y[5];
#pragma unroll
    for (int d = 0; d < 5; d++) y[d] = q == 0 ? w[d] : (q == 1 ? w[d + 1] : (q == 2 ? w[d + 2] : w[d + 3]));
    uint32_t z[4];
#pragma unroll
    for (int d = 0; d < 4; d++) z[d] = __builtin_amdgcn_alignbyte(y[d + 1], y[d], sh);
    const uint32_t cnt = on ? hi - lo : 0u;
    uint32_t o = 0;
    if (__builtin_amdgcn_ballot_w64(cnt & 8u) != 0 && (cnt & 8u)) {
      gstore8(addr, ((uint64_t)z[1] << 32) | z[0]);
      o = 8;
    }
    const uint32_t d4 = o == 8 ? z[2] : z[0], d4n = o == 8 ? z[3] : z[1];
    uint32_t rest = d4;
    if (__builtin_amdgcn_ballot_w64(cnt & 4u) != 0 && (cnt & 4u)) {
      gstore4(addr + o, d4);
      o += 4;
      rest = d4n;
    }
    if (__builtin_amdgcn_ballot_w64(cnt & 2u) != 0 && (cnt & 2u)) {
      gstore2(addr + o, rest);
      o += 2;
      rest >>= 16;
    }
    if (__builtin_amdgcn_ballot_w64(cnt & 1u) != 0 && (cnt & 1u)) gstore1(addr + o, rest);
  };

  uint32_t s = 0;
  auto fold = [&](uint4 (&v)[8]) __attribute__((always_inline)) {
    const uint32_t sin = byte_map64(s, lds, kRoundOff);
    const uint32_t sp = (uint32_t)__builtin_amdgcn_mov_dpp((int)sin, 0x128, 0xF, 0xF, false);  // lane ^ 8's
    v[0].x ^= l3 ? 0u : sin;
    v[4].x ^= l3 ? 0u : sp;
    s = fold_halves(v, k, lds, l3, kLdsW8HalfOff);
  };
  auto compute = [&](uint4 (&v)[8], uint4 pc, EncW cur, uint32_t r_c) __attribute__((always_inline)) {
    const bool live = cur.valid && r_c < cur.R;
    // the copy: this lane's chunk of each load, source offset voff in its group's round; the payload's bytes
    // in the round are [plo, phi) (a head round keeps only its first h lines)
    if constexpr ((PROBE & 1) == 0) {
      const uint64_t rb = encw_round<G>(cur, r_c);
      const uint64_t drb = rb + (cur.Dp - cur.A);
      const int64_t lo64 = (int64_t)(cur.A - rb), hi64 = (int64_t)(cur.E() - rb);
      uint32_t plo = lo64 > 0 ? (uint32_t)lo64 : 0u;
      uint32_t phi = hi64 < (int64_t)kRound ? (uint32_t)hi64 : kRound;
      if (r_c == 0 && phi > 128u * cur.h) phi = 128u * cur.h;
      if (!live) phi = 0;
      const uint32_t dlo = (uint32_t)drb, dhi = (uint32_t)(drb >> 32);
#pragma unroll
      for (int i = 0; i < 8; i++) {
        // the group whose round load i carried to this lane (G = 4: the first or second of block i's two)
        const int sl = 8 * ((i >> 2) + 2 * (i & 1) + 4 * ((i >> 1) & 1)) + (hi ? 4 : 0);
        uint64_t d;
        uint32_t a, b, Lg;
        if constexpr (G == 8) {
          d = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)dhi, sl) << 32) |
              (uint32_t)__builtin_amdgcn_readlane((int)dlo, sl);
          a = (uint32_t)__builtin_amdgcn_readlane((int)plo, sl);
          b = (uint32_t)__builtin_amdgcn_readlane((int)phi, sl);
          Lg = (uint32_t)__builtin_amdgcn_readlane((int)cur.L, sl);
        } else {  // both groups' values (scalar), then this lane's
          const int s0 = sl & ~4, s1 = s0 + 4;
          auto pick = [&](uint32_t x) {
            const uint32_t x0 = (uint32_t)__builtin_amdgcn_readlane((int)x, s0);
            const uint32_t x1 = (uint32_t)__builtin_amdgcn_readlane((int)x, s1);
            return hi ? x1 : x0;
          };
          d = ((uint64_t)pick(dhi) << 32) | pick(dlo);
          a = pick(plo);
          b = pick(phi);
          Lg = pick(cur.L);
        }
        // nontemporal for frames of >= 2 KiB (256K frames of 4000 B: 466 against 520 us per call), temporal for
        // smaller ones, whose edge lines two groups complete in L2 (2M mixed frames: 631 against 666)
        const bool nt = Lg >= 2048u;
        if ((PROBE & 8) == 0 && voff >= a && voff + 16 <= b) {
          if ((PROBE & 32) == 0 && nt)
            gstore16_nt(d + voff, v[i]);
          else
            gstore16(d + voff, v[i]);
        }
      }
      // the partial chunks: the first (bytes [lead, ...) when the payload does not start on a chunk) by lane 0,
      // the last (bytes [0, E - chunk) when it does not end on one, and it is not the first) by lane 1
      const uint64_t tc = (cur.E() - 1) & ~15ull;
      const bool hp = live && j == 0 && r_c == 0 && cur.lead() > 0;
      const bool tp = live && j == 1 && r_c + 1 == cur.R && (cur.E() & 15) != 0 && !(tc == cur.a0() && cur.lead() > 0);
      if ((PROBE & 4) == 0 && __builtin_amdgcn_ballot_w64(hp || tp) != 0) {
        const uint32_t lo = hp ? cur.lead() : 0u;
        const uint32_t hi = hp ? min(16u, cur.lead() + cur.L) : (uint32_t)(cur.E() - tc);
        store_piece(hp ? cur.Dp : tc + (cur.Dp - cur.A), pc, lo, hi, hp || tp);
      }
    }
    transpose_blocks(v);
    if constexpr ((PROBE & 2) != 0) {
      uint32_t x = s;
#pragma unroll
      for (int i = 0; i < 8; i++) x ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
      s = x;
      if (live && r_c + 1 == cur.R && j == G - 1) gstore4(cur.Dp + cur.L, s);
      if (live && r_c + 1 == cur.R) s = 0;
      return;
    }
    const bool body = live && r_c > 0 && r_c + 1 < cur.R;
    if (__builtin_amdgcn_ballot_w64(!body) == 0) {  // every group in a body round: no masks
      fold(v);
      return;
    }
    // masked round (var_class_w8): keep bytes [lo, hi) of half q of line j; lanes ^ 8 exchange bounds
    const bool head = live && r_c == 0, last = live && r_c + 1 == cur.R;
    const int32_t line_lo = head && j == 0 ? (int32_t)cur.lead() : 0;
    const int32_t line_hi =
        !live || (head && j >= cur.h) ? 0 : (last && j == (head ? cur.h - 1 : G - 1u) ? (int32_t)cur.te : 128);
    const int32_t lo_own = min(max(line_lo - 64 * (int32_t)l3, 0), 64), hi_own = min(max(line_hi - 64 * (int32_t)l3, 0), 64);
    const int32_t lo_oth = min(max(line_lo - 64 * (int32_t)(l3 ^ 1), 0), 64),
                  hi_oth = min(max(line_hi - 64 * (int32_t)(l3 ^ 1), 0), 64);
    const int32_t lo_par = lane_xor8(lo_oth), hi_par = lane_xor8(hi_oth);
    const int32_t lo_a = l3 ? lo_par : lo_own, hi_a = l3 ? hi_par : hi_own;
    const int32_t lo_b = l3 ? lo_own : lo_par, hi_b = l3 ? hi_own : hi_par;
    if (__builtin_amdgcn_ballot_w64(lo_a > 0 || hi_a < 64 || lo_b > 0 || hi_b < 64) != 0) {
      uint4 va[4] = {v[0], v[1], v[2], v[3]}, vb[4] = {v[4], v[5], v[6], v[7]};
      mask_chunks<4>(va, lo_a, hi_a, lds);
      mask_chunks<4>(vb, lo_b, hi_b, lds);
#pragma unroll
      for (int i = 0; i < 4; i++) {
        v[i] = va[i];
        v[4 + i] = vb[i];
      }
    }
    fold(v);
    if (__builtin_amdgcn_ballot_w64(head) != 0) {  // lines [0, h) to the group's last h lanes, then the init
      const uint32_t up = G - cur.h;
      const bool from = head && j >= up;
      const int src_l = (int)(head ? (from ? l - up : l) : l);
      const uint32_t moved = (uint32_t)__builtin_amdgcn_ds_bpermute(4 * src_l, (int)s);
      s = head ? (from ? moved : 0u) : s;
      if (head && j == up) s ^= lds[kLdsW8InitOff / 4 + cur.lead()];  // shift_{128-lead}(kInit)
    }
    if (__builtin_amdgcn_ballot_w64(last) != 0) {
      const uint32_t t = group_xor_reduce<G>(w8_join(s, lds, j + 8 - G));  // shift_{(G-1-j)*128}, xor over the group
      if (last && j == G - 1) {
        const uint32_t over = 128 - cur.te;
        const uint32_t crc = ~(over ? w8_unshift(t, over, lds) : t);
        gstore4(cur.Dp + cur.L, __builtin_bswap32(crc));  // the trailer, big-endian (unaligned store)
        const uint64_t hdr = (uint64_t)cur.L + 4;         // append_intT(length + 4), big-endian
        const uint64_t hp = cur.Dp - (uint64_t)T;
        if (T == 1) gstore1(hp, (uint32_t)hdr);
        else if (T == 2) gstore2(hp, __builtin_bswap32((uint32_t)hdr) >> 16);
        else if (T == 4) gstore4(hp, __builtin_bswap32((uint32_t)hdr));
        else gstore8(hp, __builtin_bswap64(hdr));
      }
      s = last ? 0u : s;
    }
  };
  auto step = [&](uint4 (&cur)[8], uint4 cpc, uint4 (&nxt)[8], uint4& npc) __attribute__((always_inline)) {
    if (__builtin_amdgcn_ballot_w64(rL >= dL.R) != 0) {
      if (rL >= dL.R) {
        tL += ngroups;
        dL = dec(tL, sn, lnn, fn);
        rL = 0;
      }
    }
    fetch(tL + ngroups, sn, lnn, fn);  // unconditional: the same addresses until dL ends
    ANNETY_PRIO_HI();
    load(dL, rL < dL.R ? rL : 0u, nxt, npc);
    __builtin_amdgcn_sched_barrier(0);
    ANNETY_PRIO_LO();
    compute(cur, cpc, dC, rC);
    dC = dL;
    rC = rL;
    rL++;
  };
  while (__builtin_amdgcn_ballot_w64(dC.live) != 0) {
    step(A, pA, B, pB);
    step(B, pB, A, pA);
  }
}

// lanes: 4 or 8 lanes per frame, or 0: chosen here from 512 frame lengths sampled evenly over the batch (the same
// samples and rule in every block): 4 when at least 3/4 of the sampled frames that are written fit one 4-line round
// whatever their lead (<= 496 bytes; 2M 408-byte chat frames: 0.594 -> 0.427 ms), else 8 (2M frames of 16 B - 1 KiB:
// 0.646 ms, against 0.83 with 4: their 5-9-line frames take two or three 4-line rounds).
template <int PROBE = 0>
__global__ __launch_bounds__(kEncBlock) void lhc_encode_fused_kernel(const uint8_t* __restrict__ src,
                                                                  const uint64_t* __restrict__ src_off,
                                                                  const uint32_t* __restrict__ len, size_t n, int T,
                                                                  int64_t enc_min, int64_t enc_max,
                                                                  uint8_t* __restrict__ dst,
                                                                  const uint64_t* __restrict__ dst_off,
                                                                  uint64_t zero_line,
                                                                  const uint4* __restrict__ img_slice,
                                                                  const uint4* __restrict__ img_w8,
                                                                  EncLong lg, int lanes) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsEnc4ImageBytes / 16];
  if (lanes == 0) {
    const uint32_t L = len[(size_t)(((uint64_t)threadIdx.x * n) / kEncBlock)];
    const bool written = L > 0 && (int64_t)L >= enc_min && !(enc_max > 0 && (int64_t)L > enc_max);
    const int nw = __syncthreads_count(written), n4 = __syncthreads_count(written && L <= 496);
    lanes = (int64_t)n4 * 4 >= (int64_t)nw * 3 && nw > 0 ? 4 : 8;
  }
  if (PROBE == 0 && lanes == 4)
    encode_frames<PROBE, 4>(lds4, src, src_off, len, n, T, enc_min, enc_max, dst, dst_off, zero_line, img_slice,
                            img_w8, lg);
  else
    encode_frames<PROBE, 8>(lds4, src, src_off, len, n, T, enc_min, enc_max, dst, dst_off, zero_line, img_slice,
                            img_w8, lg);
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
                                   const void* zero_line, const void* img_slice, const void* img_w8,
                                   const EncLong& lg, size_t max_blocks, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const size_t want = (n * 8 + kEncBlock - 1) / kEncBlock;
  const unsigned blocks = (unsigned)std::max<size_t>(1, std::min(max_blocks, want));
  note_kernel("lhc_encode_fused_kernel");
#define ANNETY_ENC_LAUNCH(P) ANNETY_ENC_LAUNCH_G(P, 8)
#define ANNETY_ENC_LAUNCH_G(P, LANES)                                                                               \
  hipLaunchKernelGGL((lhc_encode_fused_kernel<P>), dim3(blocks), dim3(kEncBlock), 0, stream,                           \
                     static_cast<const uint8_t*>(src), src_off, len, n, T, enc_min, enc_max, static_cast<uint8_t*>(dst), \
                     dst_off, (uint64_t)(uintptr_t)zero_line, static_cast<const uint4*>(img_slice),                 \
                     static_cast<const uint4*>(img_w8), lg, LANES)
#ifdef ANNETY_CRC_AB
  static const int probe = ANNETY_AB_KNOB("ANNETY_CRC_ENC_PROBE", 0);
  static const int enc_g = ANNETY_AB_KNOB("ANNETY_CRC_ENC_G", 0);  // lanes per frame 4 or 8; 0: sampled (product)
  if (probe == 0) ANNETY_ENC_LAUNCH_G(0, enc_g);
  else if (probe == 1) ANNETY_ENC_LAUNCH(1);
  else if (probe == 2) ANNETY_ENC_LAUNCH(2);
  else if (probe == 3) ANNETY_ENC_LAUNCH(3);
  else if (probe == 6) ANNETY_ENC_LAUNCH(6);
  else if (probe == 32) ANNETY_ENC_LAUNCH(32);
  else if (probe == 10) ANNETY_ENC_LAUNCH(10);
  else ANNETY_ENC_LAUNCH_G(0, 0);
#else
  ANNETY_ENC_LAUNCH_G(0, 0);  // lanes per frame sampled on the device
#endif
#undef ANNETY_ENC_LAUNCH
#undef ANNETY_ENC_LAUNCH_G
  return hipGetLastError();
}

hipError_t launch_lhc_encode_long(const uint32_t* len, int T, void* dst, const uint64_t* dst_off, const EncLong& lg,
                                  size_t max_blocks, hipStream_t stream) {
  note_kernel("lhc_encode_long_kernel");
  hipLaunchKernelGGL(lhc_encode_long_kernel, dim3((unsigned)std::max<size_t>(1, 8 * max_blocks)), dim3(kEncLongBlock), 0,
                     stream, len, T, static_cast<uint8_t*>(dst), dst_off, lg);
  return hipGetLastError();
}

}  // namespace annety_crc
