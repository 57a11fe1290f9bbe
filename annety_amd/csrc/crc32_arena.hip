// Arena path for variable-length batches whose payloads lie in one buffer (a NetBuffer, a frame
// stream, a packed batch: BASELINE config 3). Two launches, no sort:
//
//  1. The line pass (crc32_arena_lines_kernel, crc32_arena_lines.h) streams EVERY 128-byte line of the
//     arena, payload-agnostic, in the access shape of the config-1 kernel (a wave reads 64 consecutive
//     lines = one 8 KiB superblock per round). Per line j of a 1 KiB block it stores the
//     block-suffix CRC S[j] = raw(lines j..7) (register 0, no init), per block g of a superblock the
//     superblock-suffix SB[g] = raw(blocks g..7). No payload state: the arena runs at the fixed-batch
//     rate whatever the length mix.
//  2. crc32_arena_stitch_kernel gives one lane per payload. With V(x) the register after the bytes
//     before address x, taken as data (a "virtual" register that equals the payload's register inside
//     it), the payload [A, E) reads as
//         V at a line boundary  ->  whole lines I0..I1 from S/SB  ->  V(E)
//     and only two half-line (64-byte) windows are folded from the data:
//       head: lead = A % 128 < 64: the bytes [line start, A) of the first line, which fix V(first line
//             start) = shift_{-lead}(s ^ raw(them)); else the payload's bytes [A, line end), which give
//             V(first line end) = shift_{128-lead}(s) ^ raw(them);
//       tail: te = bytes of the last line up to E >= 64: the bytes [E, line end), removed from V(last
//             line end) as V(E) = shift_{-(128-te)}(V ^ raw(them)); else the payload's bytes [line start,
//             E), appended to V(last line start).
//     The whole lines between take at most four steps acc = M1(acc) ^ M2(S[a] ^ S[b]) (the head block,
//     the partial superblocks' block runs, the tail block: M1 = shift by the unit, M2 = the inverse
//     shift that cuts a suffix difference down to the unit); the whole superblocks between are a chain
//     acc = shift_8KiB(acc) ^ SB[q, 0], shared by the lanes running the stitch once a run is longer than
//     kLongMid superblocks (mid_join).
//     A config-3 payload (6.5 KiB on average) costs 64 + 64 bytes of window folds and about six map
//     steps of 8 nibble-table lookups, with every load issued before the first fold.
//     s = 0xFFFFFFFF (crc32_long) or the caller's register (crc32_update, include/Crc32c.h:71-82).
//     Bytes outside the arena [byte_lo, byte_hi) sharing a line with it are zeros to both launches.
//
// Reference semantics: crc32_long include/Crc32c.h:58-69 (digests), crc32_update :71-82 (update
// mode); the math identities are in crc32_math.h. DESIGN.md §2.6.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "crc32_arena_lines.h"
#include "crc32_device.h"
#include "crc32_kernels.h"
#include "crc32_math.h"

namespace annety_crc {
namespace {

// 512 lanes per block (one block per CU, LDS-bound), which leaves 256 VGPRs per lane; a config-3 batch
// (165k payloads) is 1.26 payloads per lane. (1024-lane blocks, which cap a kernel at 128 VGPRs,
// returned wrong digests for whole waves now and then on the MI355X with the previous stitch - a
// register-pressure-dependent fault we did not pin down)
constexpr int kStitchBlock = 512;
constexpr uint32_t kMidChunk = 7;  // whole superblocks between a payload's partial ones whose SB words load with its plan
// Runs of more whole superblocks than this (a payload of more than ~512 KiB) are joined by the whole wave (mid_join)
constexpr uint32_t kLongMid = 64;

// (nibble_map_set: crc32_device.h)
// shift_{-m} for m in [0, 128): U_hi[m >> 4] o U_lo[m & 15]
__device__ __forceinline__ uint32_t unshift(uint32_t t, uint32_t m, const uint32_t* lds) {
  t = nibble_map_set<16>(t, lds, kLdsStitchUnshiftOff, m & 15u);
  return nibble_map_set<8>(t, lds, kLdsStitchUnshiftOff + 8192, m >> 4);
}
__device__ __forceinline__ uint32_t seg_map(uint32_t t, uint32_t idx, const uint32_t* lds) {
  return nibble_map_set<32>(t, lds, kLdsMapOff, idx);
}
// Two 64-byte windows from register 0, four 32-byte chains: raw(window) = shift_32(raw(first half)) ^
// raw(second half).
__device__ __forceinline__ void absorb_two_windows(const uint4 (&v)[4], const uint4 (&w)[4], const LaneCtx& k,
                                                   const uint32_t* lds, uint32_t& rv, uint32_t& rw) {
  uint32_t xa = v[0].x, xb = v[2].x, xc = w[0].x, xd = w[2].x;
#pragma unroll
  for (int i = 0; i < 2; i++) {
    word4x4(xa, v[i].y, xb, v[2 + i].y, xc, w[i].y, xd, w[2 + i].y, k);
    word4x4(xa, v[i].z, xb, v[2 + i].z, xc, w[i].z, xd, w[2 + i].z, k);
    word4x4(xa, v[i].w, xb, v[2 + i].w, xc, w[i].w, xd, w[2 + i].w, k);
    word4x4(xa, i == 0 ? v[1].x : 0u, xb, i == 0 ? v[3].x : 0u, xc, i == 0 ? w[1].x : 0u, xd, i == 0 ? w[3].x : 0u, k);
  }
  rv = nibble_map_uniform(xa, lds, kLdsQuarterOff) ^ xb;
  rw = nibble_map_uniform(xc, lds, kLdsQuarterOff) ^ xd;
}

// Where the stitch finds a call's batch and the line pass's outputs (layout: crc32_kernels.h).
struct StitchGeo {
  const uint8_t* base;
  uint64_t byte_lo, byte_hi, line_lo, line_hi, sb0, fs0, fs1;
  uint64_t W;   // line-pass waves = 8 * L
  uint32_t L;   // line-pass workgroups (64 L lane groups)
  const uint32_t *S, *SB, *S_edge, *SB_edge;
  // the stitch addresses the line pass's outputs as 32-bit word indices from W0 (= S; when the call has no
  // arena, g.len: index 0 is then a valid word for the dummy loads); sb_word / edge_word = SB / S_edge - S
  const uint32_t* W0;
  uint32_t sb_word, edge_word;
  uint64_t Lmagic;  // ceil(2^40 / L): (x * Lmagic) >> 40 == x / L for x < 2^26 (s_addr's task division)
  const uint64_t* off;
  const uint32_t* len;
  size_t n;
  uint64_t zero_line;
  uint32_t* out;
  uint8_t* ok;            // ArenaLaunch::ok (read only by the VER stitch)
  const uint64_t* check;  // ArenaLaunch::check
  uint32_t check_parts;
  uint64_t check_lo, check_hi;
  bool check_any_order;
  ExtentHint* record;
  uint64_t record_seq;
  AutoChoice choice;  // ArenaLaunch::choice: W0 = the scratch, the geometry from the device's span
  const uint32_t* pow8k;  // ArenaLaunch::pow8k
  // lanes per payload: 1, or 64 for batches of few payloads (stitch_spread): a wave per payload, whose 63 other lanes
  // help with its long superblock runs (mid_join)
  uint32_t spread;
};

// The stitch's geometry for the span the device chose (AutoChoice; the host's stitch_geo below).
__device__ __forceinline__ void stitch_geo_chosen(StitchGeo& s, const ArenaSpan& sp, const ArenaGeom& geo) {
  uint32_t* scratch = const_cast<uint32_t*>(s.W0);
  s.byte_lo = sp.byte_lo;
  s.byte_hi = sp.byte_hi;
  s.line_lo = sp.line_lo;
  s.line_hi = sp.line_hi;
  s.sb0 = sp.sb0;
  s.fs0 = sp.fs0;
  s.fs1 = sp.fs1;
  s.S = scratch;  // (W, L and Lmagic: the host's, from choice.blocks)
  s.SB = scratch + geo.sb_off;
  s.S_edge = scratch + geo.edge_off;
  s.SB_edge = scratch + geo.edge_off + 128;
  s.sb_word = (uint32_t)geo.sb_off;
  s.edge_word = (uint32_t)geo.edge_off;
  s.check = nullptr;
}

// One payload's loads and the plan that consumes them. Steps 0..3 = head block, first partial
// superblock's blocks, last partial superblock's blocks, tail block; mid = whole superblocks between.
struct Plan {
  uint64_t A, E;
  uint32_t len;
  bool fast, headX, tailX;
  uint32_t lead, te;
  uint32_t hlo, hhi, tlo, thi;  // window byte ranges kept, relative to the window start
  uint32_t m1, m2;              // step q's maps (seg_map index < 32) in byte q
  uint32_t act, yzero;          // per step bit: active / second operand is zero
  uint32_t nmid;
  uint32_t mid_s;               // first whole superblock between (relative to sb0)
  uint32_t xa[4], ya[4];        // step operand word indices from g.W0
};
struct Vals {
  uint4 h[4], t[4];
  uint32_t x[4], y[4], mid[kMidChunk];
  uint32_t s0;
  uint32_t tr0, tr1;  // VER: the two dwords holding the trailer
  uint32_t tsh;       // VER: the trailer's byte offset inside tr0
  __device__ __forceinline__ uint32_t tr_shift() const { return tsh; }
};

// The per-payload stitch (file comment). Phase A issues everything the line pass did not write, phase
// B the S/SB words.
//   PROBE (microbench only; product = 0): 1 = descriptors and stores only, 2 = + all loads,
//   3 = + window folds (no map steps), 4 = the product with every S/SB word from one address, 5 = the product with
//   every window chunk from the zero line - wrong digests, used to measure what the stages cost.
//   VER: LengthHeaderCodec verify (LengthHeaderCodec::decode, include/codec/LengthHeaderCodec.h:107-121): the
//   4-byte big-endian trailer after each payload is loaded with the plan and compared with the digest here,
//   ok[p] = 1 on a match (the digest itself is stored only when out is set).
template <bool UPD, int PROBE, bool VER = false>
struct Stitcher {
  const StitchGeo& g;
  const uint32_t* lds;
  LaneCtx k;

  __device__ __forceinline__ void put(size_t p, uint32_t digest, const Vals& v) const {
    if constexpr (VER) {
      if (g.out) g.out[p] = digest;
      // bytes [E, E + 4) of the trailer's two dwords, as a big-endian integer
      const uint32_t le = __builtin_amdgcn_alignbyte(v.tr1, v.tr0, v.tr_shift());
      g.ok[p] = __builtin_bswap32(le) == digest ? 1 : 0;
    } else {
      g.out[p] = digest;
    }
  }

  __device__ __forceinline__ uint32_t word(uint32_t idx) const {
    return gload4((uint64_t)(uintptr_t)g.W0 + 4ull * idx);
  }
  // word index of S for line a (0..7) of block rb (relative to superblock sb0)
  __device__ __forceinline__ uint32_t s_addr(uint64_t rb, uint32_t a) const {
    const uint64_t sb = g.sb0 + (rb >> 3);
    const bool edge = sb < g.fs0 || sb >= g.fs1;
    const uint32_t r = (uint32_t)(rb - (g.fs0 - g.sb0) * 8);               // block of the full range (< 2^32)
    const uint32_t t = (uint32_t)(((uint64_t)(r >> 6) * g.Lmagic) >> 40);  // task = (r >> 6) / L
    const uint32_t full = (uint32_t)arena_s_word(t, r - t * 64 * g.L, a, g.W);  // lane group = r - t * 64 L
    const uint32_t ed = g.edge_word + (sb == g.sb0 ? 0u : 64u) + (uint32_t)(rb & 7) * 8 + a;
    return edge ? ed : full;
  }
  // word index of SB for block gg of superblock sbr (relative to sb0)
  __device__ __forceinline__ uint32_t sb_addr(uint64_t sbr, uint32_t gg) const {
    const uint64_t sb = g.sb0 + sbr;
    const bool edge = sb < g.fs0 || sb >= g.fs1;
    const uint32_t full = g.sb_word + (uint32_t)(sb - g.fs0) * 8 + gg;
    const uint32_t ed = g.edge_word + 128u + (sb == g.sb0 ? 0u : 8u) + gg;
    return edge ? ed : full;
  }

  // SB[., 0] word indices of the whole superblocks mid_s .. mid_s + cnt - 1 (relative to sb0, cnt <= kMidChunk),
  // the rest 0. Whole superblocks between two partial ones are never the arena's edge superblocks, and SB is linear
  // in the superblock, so no edge selects.
  __device__ __forceinline__ void mid_addrs(uint32_t mid_s, uint32_t cnt, uint32_t (&a)[kMidChunk]) const {
    const uint32_t w0 = g.sb_word + (uint32_t)(g.sb0 + mid_s - g.fs0) * 8;
#pragma unroll
    for (uint32_t c = 0; c < kMidChunk; c++) a[c] = c < cnt ? w0 + 8 * c : 0u;
  }

  // Phase A: descriptor, plan, window and register loads (nothing the line pass writes).
  __device__ __forceinline__ void plan_a(size_t p, Plan& y, Vals& v) const { plan_a(p, g.len[p], g.off[p], y, v); }
  __device__ __forceinline__ void plan_a(size_t p, uint32_t len, uint64_t off, Plan& y, Vals& v) const {
    y.len = len;
    y.A = (uint64_t)(uintptr_t)g.base + off;
    y.E = y.A + y.len;
    y.fast = y.len > 0 && y.A >= g.byte_lo && y.E <= g.byte_hi;
    const uint64_t L0 = y.A >> 7, L1 = (y.E - (y.len ? 1 : 0)) >> 7;
    y.lead = (uint32_t)(y.A & 127);
    y.te = (uint32_t)((y.E - (y.len ? 1 : 0)) & 127) + (y.len ? 1u : 0u);
    y.headX = y.lead < 64;
    y.tailX = y.te >= 64;
    const uint32_t cl0 = L0 == g.line_lo ? (uint32_t)(g.byte_lo & 127) : 0u;
    const uint32_t ch0 = L0 == g.line_hi ? (uint32_t)(((g.byte_hi - 1) & 127) + 1) : 128u;
    const uint32_t cl1 = L1 == g.line_lo ? (uint32_t)(g.byte_lo & 127) : 0u;
    const uint32_t ch1 = L1 == g.line_hi ? (uint32_t)(((g.byte_hi - 1) & 127) + 1) : 128u;
    // windows: head [0,64) keeps [cl, lead) or [64,128) keeps [lead, ch); tail [64,128) keeps [te, ch) or
    // [0,64) keeps [cl, te)
    const uint32_t oh = y.headX ? 0u : 64u, ot = y.tailX ? 64u : 0u;
    y.hlo = (y.headX ? cl0 : y.lead) - oh;
    y.hhi = (y.headX ? y.lead : ch0) - oh;
    y.tlo = (y.tailX ? y.te : cl1) - ot;
    y.thi = (y.tailX ? ch1 : y.te) - ot;
    const uint64_t hsrc = y.len ? (L0 << 7) + oh : g.zero_line;
    const uint64_t tsrc = y.len ? (L1 << 7) + ot : g.zero_line;
    // only the 16-byte chunks that hold kept bytes come from the batch; the rest read the zero line (an L2 hit):
    // on average half of each window, which the fold masks to zero anyway
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const bool keep = PROBE != 5 && 16u * i < y.hhi && 16u * i + 16 > y.hlo;
      v.h[i] = gload16((keep ? hsrc : g.zero_line) + 16 * i);
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const bool keep = PROBE != 5 && 16u * i < y.thi && 16u * i + 16 > y.tlo;
      v.t[i] = gload16((keep ? tsrc : g.zero_line) + 16 * i);
    }
    v.s0 = UPD ? gload4((uint64_t)(uintptr_t)(g.out + p)) : kInit;
    if constexpr (VER) {  // the trailer [E, E + 4): the dword holding E and, when it is unaligned, the next one
      const uint64_t ea = y.E & ~3ull;
      v.tsh = (uint32_t)(y.E & 3);
      v.tr0 = gload4(ea);
      v.tr1 = gload4(v.tsh ? ea + 4 : ea);
    }

    // whole lines I0..I1 (empty when I1 < I0)
    const int64_t I0 = (int64_t)L0 + (y.headX ? 0 : 1), I1 = (int64_t)L1 - (y.tailX ? 0 : 1);
    const bool seg = y.fast && I1 >= I0;
    const uint64_t b0 = (uint64_t)I0 >> 3, b1 = (uint64_t)I1 >> 3;
    const uint32_t a = (uint32_t)I0 & 7, z = (uint32_t)I1 & 7;
    const uint64_t rb0 = b0 - g.sb0 * 8, rb1 = b1 - g.sb0 * 8;
    const bool same = b0 == b1;
    const bool blocks = seg && b1 >= b0 + 2;
    const uint64_t B0 = rb0 + 1, B1 = rb1 - 1;
    const uint64_t s0 = B0 >> 3, s1 = B1 >> 3;
    const uint32_t g0 = (uint32_t)B0 & 7, g1 = (uint32_t)B1 & 7;
    const bool one = s0 == s1;
    // step 0: head block (or the whole run when it stays in one block)
    y.m1 = kMapF + (same ? z - a + 1 : 8 - a) - 1;
    y.m2 = kMapUL + (same ? 7 - z : 0);
    y.xa[0] = s_addr(rb0, a);
    y.ya[0] = s_addr(rb0, z + 1 < 8 ? z + 1 : 0);
    const bool yz0 = !same || z == 7;
    // step 1: blocks of the first partial superblock (or all of them when they stay in one)
    y.m1 |= (kMapG + (one ? g1 - g0 + 1 : 8 - g0) - 1) << 8;
    y.m2 |= (kMapUB + (one ? 7 - g1 : 0)) << 8;
    y.xa[1] = sb_addr(s0, g0);
    y.ya[1] = sb_addr(s0, g1 + 1 < 8 ? g1 + 1 : 0);
    const bool yz1 = !one || g1 == 7;
    // step 2: blocks 0..g1 of the last partial superblock
    y.m1 |= (kMapG + g1) << 16;
    y.m2 |= (kMapUB + (7 - g1)) << 16;
    y.xa[2] = sb_addr(s1, 0);
    y.ya[2] = sb_addr(s1, g1 + 1 < 8 ? g1 + 1 : 0);
    const bool yz2 = g1 == 7;
    // step 3: lines 0..z of the tail block
    y.m1 |= (kMapF + z) << 24;
    y.m2 |= (kMapUL + (7 - z)) << 24;
    y.xa[3] = s_addr(rb1, 0);
    y.ya[3] = s_addr(rb1, z + 1 < 8 ? z + 1 : 0);
    const bool yz3 = z == 7;
    y.act = (seg ? 1u : 0u) | (blocks ? 2u : 0u) | (blocks && !one ? 4u : 0u) | (seg && !same ? 8u : 0u);
    y.yzero = (yz0 ? 1u : 0u) | (yz1 ? 2u : 0u) | (yz2 ? 4u : 0u) | (yz3 ? 8u : 0u);
    y.nmid = blocks && !one ? (uint32_t)(s1 - s0 - 1) : 0u;
    y.mid_s = (uint32_t)(s0 + 1);
  }

  // Phase B: the S/SB words of the plan.
  __device__ __forceinline__ void plan_b(size_t /*p*/, const Plan& y, Vals& v) const {
    const uint32_t dummy = 0;  // g.W0[0]: a valid word (the loads of inactive steps are not used)
    // a wave whose payloads all stay within two blocks (frames, short payloads) has steps 1-2 and the whole
    // superblocks between empty: it loads only steps 0 and 3 (frames verify 0.290 -> 0.287 ms per step, config 3
    // unchanged; profiles/r06/abshort/)
    if (__builtin_amdgcn_ballot_w64((y.act & 6u) != 0 || y.nmid != 0) == 0) {
#pragma unroll
      for (int q = 0; q < 4; q += 3) {
        const bool on = PROBE != 4 && ((y.act >> q) & 1u);
        v.x[q] = word(on ? y.xa[q] : dummy);
        v.y[q] = word(on && !((y.yzero >> q) & 1u) ? y.ya[q] : dummy);
      }
      v.x[1] = v.x[2] = v.y[1] = v.y[2] = 0;
#pragma unroll
      for (uint32_t c = 0; c < kMidChunk; c++) v.mid[c] = 0;
      return;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const bool on = PROBE != 4 && ((y.act >> q) & 1u);
      v.x[q] = word(on ? y.xa[q] : dummy);
      v.y[q] = word(on && !((y.yzero >> q) & 1u) ? y.ya[q] : dummy);
    }
    uint32_t ma[kMidChunk];
    mid_addrs(y.mid_s, y.nmid < kMidChunk ? y.nmid : kMidChunk, ma);  // (dummy = 0)
#pragma unroll
    for (uint32_t c = 0; c < kMidChunk; c++) v.mid[c] = word(ma[c]);
  }

  // shift_{m * 8 KiB}(x) from the power table (ArenaLaunch::pow8k; m beyond its reach in several applications)
  __device__ __forceinline__ uint32_t pow8k(uint32_t x, uint32_t m) const {
    while (m) {
      const uint32_t e = m < kSplitMaxSegs - 1 ? m : kSplitMaxSegs - 1;
      const uint32_t* P = g.pow8k + (size_t)(e - 1) * 32;
      uint32_t r = 0;
#pragma unroll 8
      for (int b = 0; b < 32; b++) r ^= P[b] & (0u - ((x >> b) & 1u));  // (8 loads at a time: few VGPRs)
      x = r;
      m -= e;
    }
    return x;
  }

  // The whole superblocks between a payload's partial ones (y.nmid of them from y.mid_s): acc = V before them ->
  // V after them = shift_{n 8KiB}(acc) ^ xor_q shift_{(n-1-q) 8KiB}(SB[q, 0]). Runs of up to kLongMid superblocks
  // are a chain of shift_8KiB steps on the payload's lane; longer runs (a payload of more than ~512 KiB; up to 8k
  // superblocks for one of the codec's 64 MiB frames) are taken by all the lanes running this, one run after another:
  // each chains its share of the run, which enters as shift_{(superblocks after it) 8KiB} from the power table, and a
  // scalar xor over the lanes gives the run's lane V after it (the chain was serial). `on`: this
  // lane's payload has a run to join.
  __device__ __forceinline__ uint32_t mid_join(uint32_t acc, bool on, const Plan& y, Vals& v) const {
    const bool lng = on && y.nmid > kLongMid;
    if (on && !lng && y.nmid) {  // acc = shift_8KiB(acc) ^ SB[s, 0], superblock by superblock
      for (uint32_t i = 0; i < y.nmid; i += kMidChunk) {
        if (i > 0) {
          uint32_t ma[kMidChunk];
          mid_addrs(y.mid_s + i, y.nmid - i < kMidChunk ? y.nmid - i : kMidChunk, ma);
#pragma unroll
          for (uint32_t c = 0; c < kMidChunk; c++) v.mid[c] = word(ma[c]);
        }
#pragma unroll
        for (uint32_t c = 0; c < kMidChunk; c++)
          if (i + c < y.nmid) acc = seg_map(acc, kMapG + 7, lds) ^ v.mid[c];
      }
    }
    // the lanes running this (the payload loop leaves a wave's last lanes behind at the end of a block's range): they
    // share each run, rank = this lane's place among them
    const uint64_t act = __builtin_amdgcn_ballot_w64(true);
    const uint32_t nact = (uint32_t)__builtin_popcountll(act);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
    const uint32_t l = threadIdx.x & 63;
    uint64_t todo = __builtin_amdgcn_ballot_w64(lng);
    while (todo) {
      const int src = __builtin_ffsll((long long)todo) - 1;
      todo &= todo - 1;
      const uint32_t n = (uint32_t)__builtin_amdgcn_readlane((int)y.nmid, src);
      const uint32_t ms = (uint32_t)__builtin_amdgcn_readlane((int)y.mid_s, src);
      const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)acc, src);
      // (whole superblocks between two partial ones are never the arena's edge ones: SB at sb_word + 8 (sb - fs0))
      const uint32_t w0 = g.sb_word + (uint32_t)(g.sb0 + ms - g.fs0) * 8;
      const uint32_t per = (n + nact - 1) / nact, lo = min(n, rank * per), hi = min(n, lo + per);
      uint32_t r = 0;
      for (uint32_t q = lo; q < hi; q += 4) {  // 4 loads in flight, then their 4 steps
        uint32_t w[4];
#pragma unroll
        for (uint32_t c = 0; c < 4; c++) w[c] = word(q + c < hi ? w0 + 8 * (q + c) : 0u);
#pragma unroll
        for (uint32_t c = 0; c < 4; c++)
          if (q + c < hi) r = seg_map(r, kMapG + 7, lds) ^ w[c];
      }
      uint32_t x = pow8k(r, n - hi);     // this lane's share, seen from the run's end
      if (rank == 0) x ^= pow8k(a0, n);  // the register before the run
      uint32_t tot = 0;                  // xor over the running lanes (scalar: no read of a lane left behind)
      for (uint64_t m = act; m; m &= m - 1)
        tot ^= (uint32_t)__builtin_amdgcn_readlane((int)x, __builtin_ffsll((long long)m) - 1);
      if (l == (uint32_t)src) acc = tot;
    }
    return acc;
  }

  // Payload p's digest (or register); mid_join shares long superblock runs among the lanes running this. `own`: this
  // lane writes the result (with StitchGeo::spread > 1 the payload's other lanes only help with its runs).
  __device__ __forceinline__ void process(size_t p, const Plan& y, Vals& v, bool own = true) const {
    bool live = false;  // a payload on the arena path, to finish after the whole superblocks
    uint32_t acc = 0, wt = 0;
    if (own) {
      if (y.len == 0) {  // crc of the empty string is 0; update mode leaves the register alone
        if constexpr (!UPD) put(p, 0u, v);
      } else if constexpr (PROBE == 1) {
        g.out[p] = (uint32_t)y.A ^ y.lead ^ v.s0;
      } else if constexpr (PROBE == 2) {
        uint32_t t = v.s0;
#pragma unroll
        for (int q = 0; q < 4; q++) t ^= v.h[q].x ^ v.t[q].y ^ v.x[q] ^ v.y[q];
#pragma unroll
        for (uint32_t c = 0; c < kMidChunk; c++) t ^= v.mid[c];
        g.out[p] = t;
      } else if (y.fast) {
        live = true;
        // (byte masks from the image's chunk tables: 2 LDS reads and 4 ands per chunk where mask_line's per-dword
        // clamps and 64-bit shifts took about 200 VALU instructions per payload)
        mask_chunks<4>(v.h, (int32_t)y.hlo, (int32_t)y.hhi, lds, kLdsStitchMaskOff);
        mask_chunks<4>(v.t, (int32_t)y.tlo, (int32_t)y.thi, lds, kLdsStitchMaskOff);
        uint32_t wh;
        absorb_two_windows(v.h, v.t, k, lds, wh, wt);
        // head: V(first line start) = shift_{-lead}(s0) ^ shift_{-64}(wh), or
        //       V(first line end) = shift_{-lead}(shift_128(s0)) ^ wh
        const uint32_t f1s = seg_map(v.s0, kMapF, lds);
        const uint32_t u64 = nibble_map_set<8>(wh, lds, kLdsStitchUnshiftOff + 8192, 4);  // shift_{-64}
        acc = unshift(y.headX ? v.s0 : f1s, y.lead, lds) ^ (y.headX ? u64 : wh);
        if constexpr (PROBE != 3) {
#pragma unroll
          for (int q = 0; q < 2; q++) {
            if ((y.act >> q) & 1u) {
              const uint32_t d = v.x[q] ^ (((y.yzero >> q) & 1u) ? 0u : v.y[q]);
              acc = seg_map(acc, __builtin_amdgcn_ubfe(y.m1, 8 * q, 5), lds) ^
                    seg_map(d, __builtin_amdgcn_ubfe(y.m2, 8 * q, 5), lds);
            }
          }
        }
      } else {
        // payload reaches outside the arena the caller declared (or there is none): fold its lines directly
        const uint64_t L0 = y.A >> 7, L1 = (y.E - 1) >> 7;
        acc = unshift(v.s0, y.lead, lds);  // V(first line start): the lead bytes are zeros here
        for (uint64_t i = L0; i <= L1; i++) {
          uint4 u[8];
#pragma unroll
          for (int q = 0; q < 8; q++) u[q] = gload16((i << 7) + 16 * q);
          mask_line<8>(u, i == L0 ? (int32_t)y.lead * 8 : 0, i == L1 ? (int32_t)y.te * 8 : 1024);
          const uint32_t r = absorb_line(0u, u, k, lds);
          acc = seg_map(acc, kMapF, lds) ^ r;
        }
        acc = unshift(acc, 128 - y.te, lds);  // drop the zero bytes after the payload end
        put(p, UPD ? acc : ~acc, v);
      }
    }
    // whole superblocks between the partial ones, in one level per kMidChunk of them (the first chunk's words were
    // loaded with the plan; payloads past 7 whole superblocks load the next chunks here), long runs by the wave
    if constexpr (PROBE != 3) acc = mid_join(acc, live, y, v);
    if (!live) return;
    if constexpr (PROBE != 3) {
#pragma unroll
      for (int q = 2; q < 4; q++) {
        if ((y.act >> q) & 1u) {
          const uint32_t d = v.x[q] ^ (((y.yzero >> q) & 1u) ? 0u : v.y[q]);
          acc = seg_map(acc, __builtin_amdgcn_ubfe(y.m1, 8 * q, 5), lds) ^
                seg_map(d, __builtin_amdgcn_ubfe(y.m2, 8 * q, 5), lds);
        }
      }
    }
    // tail: V(E) = shift_{-(128-te)}(V(last line end) ^ wt), or
    //       shift_{-(128-te)}(shift_128(V(last line start)) ^ shift_64(wt))
    const uint32_t f1a = seg_map(acc, kMapF, lds);
    const uint32_t h64 = nibble_map_uniform(wt, lds, kLdsHalfOff);
    acc = unshift(y.tailX ? acc ^ wt : f1a ^ h64, 128 - y.te, lds);
    put(p, UPD ? acc : ~acc, v);
  }
};

__device__ __forceinline__ LaneCtx lane_ctx() {
  LaneCtx k;
  k.L0 = (threadIdx.x & 31) << 3;
  k.L1 = k.L0 | (1u << 16);
  k.slot4 = (threadIdx.x & 31) << 2;
  return k;
}

// Relaxed system-scope stores of the extent record and its check word (crc32_kernels.h ExtentHint).
__device__ __forceinline__ void publish_extent(ExtentHint* host, uint64_t lo, uint64_t hi, uint64_t sum, uint64_t bad,
                                               uint64_t seq) {
  const uint64_t f[6] = {lo, hi, sum, bad, seq, lo ^ hi ^ sum ^ bad ^ seq ^ kExtentCheck};
  uint64_t* h = reinterpret_cast<uint64_t*>(host);
#pragma unroll
  for (int i = 0; i < 6; i++) __hip_atomic_store(h + i, f[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Second launch of the two-launch path: contiguous payload ranges per block (coalesced descriptor loads),
// the same count for every block; the first payload's loads are in flight while the LDS image is staged.
//   PIPE (microbench A/B, product = 0): 1 = the next payload's loads are issued before the
//   current one is folded; 2 = a lane's first two payloads' descriptors and plan loads issued together.
template <bool UPD, int BLK = kStitchBlock, int PROBE = 0, int PIPE = 0, bool VER = false>
__global__ __launch_bounds__(BLK) void crc32_arena_stitch_kernel(StitchGeo g0, const uint4* __restrict__ img_slice,
                                                                 const uint4* __restrict__ img_stitch) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[kLdsStitchImageBytes / 16];
  StitchGeo g = g0;
  if (g.choice.ws) {  // the device's choice: the arena's span (or return: the sorted path runs this call)
    ArenaSpan sp;
    if (!choose_arena(g.choice, sp)) return;
    stitch_geo_chosen(g, sp, arena_geom_of(sp.fs1 - sp.fs0, g.choice.blocks));
    // the next calls' record (crc32_kernels.h): extent_of reduces across the wave, so every lane takes part
    uint64_t lo, hi, sum, bad;
    extent_of(g.choice.ws, g.choice.parts, lo, hi, sum, bad);
    if (blockIdx.x == 0 && threadIdx.x == 0 && g.record) publish_extent(g.record, lo, hi, sum, bad, g.record_seq);
  }
  // automatic path: this call's extent, reduced by every wave from the partials; on a mismatch with the
  // declared arena the line pass did nothing, and every payload is folded directly
  if (g.check) {
    uint64_t lo, hi, sum, bad;
    extent_of(g.check, g.check_parts, lo, hi, sum, bad);
    if (!(lo == g.check_lo && hi == g.check_hi && (bad == 0 || g.check_any_order))) g.byte_lo = g.byte_hi = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0 && g.record)  // the next calls' record (crc32_kernels.h)
      publish_extent(g.record, lo, hi, sum, bad, g.record_seq);
  }
  const Stitcher<UPD, PROBE, VER> st{g, reinterpret_cast<const uint32_t*>(lds4), lane_ctx()};
  const size_t per = (g.n + gridDim.x - 1) / gridDim.x;
  const size_t p_end = std::min(g.n, (size_t)(blockIdx.x + 1) * per);
  Plan y{};
  Vals v{};
  if (g.spread > 1) {  // a wave per payload (few payloads: the wave helps with its long runs)
    load_image<kLdsStitchImageBytes, BLK, kLdsCommonBytes>(lds4, img_slice, nullptr, img_stitch);
    __syncthreads();
    for (size_t p = (size_t)blockIdx.x * per + threadIdx.x / 64; p < p_end; p += BLK / 64) {
      st.plan_a(p, y, v);
      st.plan_b(p, y, v);
      st.process(p, y, v, (threadIdx.x & 63) == 0);
    }
    return;
  }
  const size_t p_first = (size_t)blockIdx.x * per + threadIdx.x;
  if (p_first < p_end) {
    st.plan_a(p_first, y, v);
    st.plan_b(p_first, y, v);
  }
  if constexpr (PIPE == 1) {
    Plan y2{};
    Vals v2{};
    if (p_first + BLK < p_end) {
      st.plan_a(p_first + BLK, y2, v2);
      st.plan_b(p_first + BLK, y2, v2);
    }
    load_image<kLdsStitchImageBytes, BLK, kLdsCommonBytes>(lds4, img_slice, nullptr, img_stitch);
    __syncthreads();
    // (y, v) holds payload p, (y2, v2) payload p + BLK; each refills while the other folds
    for (size_t p = p_first; p < p_end; p += 2 * BLK) {
      st.process(p, y, v);
      if (p + 2 * BLK < p_end) {
        st.plan_a(p + 2 * BLK, y, v);
        st.plan_b(p + 2 * BLK, y, v);
      }
      if (p + BLK < p_end) st.process(p + BLK, y2, v2);
      if (p + 3 * BLK < p_end) {
        st.plan_a(p + 3 * BLK, y2, v2);
        st.plan_b(p + 3 * BLK, y2, v2);
      }
    }
  } else if constexpr (PIPE == 2) {
    // the block's first two payloads per lane: both descriptors in flight together, then both plans'
    // loads, all before the LDS image is staged. Loads are unconditional (a lane without a payload reads
    // a valid one's) so the wait counts stay exact; the rest of a long batch runs one payload at a time.
    const size_t last = p_end > 0 ? p_end - 1 : 0;
    const size_t p2 = p_first + BLK;
    const size_t q1 = p_first < p_end ? p_first : last, q2 = p2 < p_end ? p2 : last;
    Plan y2{};
    Vals v2{};
    const uint32_t l1 = g.len[q1], l2 = g.len[q2];
    const uint64_t o1 = g.off[q1], o2 = g.off[q2];
    st.plan_a(q1, l1, o1, y, v);
    st.plan_b(q1, y, v);
    st.plan_a(q2, l2, o2, y2, v2);
    st.plan_b(q2, y2, v2);
    load_image<kLdsStitchImageBytes, BLK, kLdsCommonBytes>(lds4, img_slice, nullptr, img_stitch);
    __syncthreads();
    if (p_first < p_end) st.process(p_first, y, v);
    if (p2 < p_end) st.process(p2, y2, v2);
    for (size_t p = p2 + BLK; p < p_end; p += BLK) {
      st.plan_a(p, y, v);
      st.plan_b(p, y, v);
      st.process(p, y, v);
    }
  } else {
    load_image<kLdsStitchImageBytes, BLK, kLdsCommonBytes>(lds4, img_slice, nullptr, img_stitch);
    __syncthreads();
    for (size_t p = p_first; p < p_end; p += BLK) {
      if (p != p_first) {
        st.plan_a(p, y, v);
        st.plan_b(p, y, v);
      }
      st.process(p, y, v);
    }
  }
}

// First launch: the line pass.
// `base` = the first full superblock (fs0 * 8192); with a device choice (ar.choice.ws) the batch's base, from which
// the pass moves to the chosen span's first full superblock (or returns: the sorted path runs this call).
template <int PROBE = 0, bool NT = true>
__global__ __launch_bounds__(kBlock) void crc32_arena_lines_kernel(const uint8_t* __restrict__ base, LineOut ar,
                                                                   const uint4* __restrict__ img_slice,
                                                                   const uint4* __restrict__ img_group8,
                                                                   const uint4* __restrict__ img_sb) {
  __shared__ __attribute__((aligned(16))) uint4 lds4[(NT ? kLdsArenaNtImageBytes : kLdsArenaImageBytes) / 16];
  if (ar.choice.ws) {
    ArenaSpan sp;
    if (!choose_arena(ar.choice, sp)) return;  // uniform over the grid
    line_out_chosen(ar, sp, arena_geom_of(sp.fs1 - sp.fs0, gridDim.x));
    base += (int64_t)(sp.fs0 * 8192 - (uint64_t)(uintptr_t)base);
  }
  arena_line_pass<PROBE, NT>(base, ar, blockIdx.x, gridDim.x, lds4, img_slice, img_group8, img_sb);
}

// Extent of a variable batch (crc32_kernels.h launch_extent), no fences: every block writes its partial
// {lo, hi, sum, bad} with plain stores; the next launches on the stream (the kernel boundary orders them)
// reduce the partials themselves, one wave at a time (extent_of): the line pass and the stitch check the
// declared arena against them, and the stitch (or, on the sorted path, crc32_bucket_place) publishes the
// result to the pinned host record with relaxed system-scope stores plus a check word over the fields,
// which is how the host tells a complete record from a torn one. (A first version reduced in the last
// block to arrive, behind device-scope fences, and published with a system-scope release: 11.4 us per
// call, every release writing back the dirty L2 lines of the launches before it.) At most kExtentMaxParts
// partials: every block of the line pass and of the stitch reduces them all (510 partials of 256-thread
// blocks cost the config-3 line pass 3.5 us and the stitch 3.6).
// ws layout (uint64): [8 + 4b ...] block b's partial; bytes [kCursorOff, +8 KiB) the bucket cursors.
constexpr int kExtentBlock = kBucketThreads;
__device__ __forceinline__ uint64_t wave_min(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = min(v, (uint64_t)__shfl_xor((unsigned long long)v, d));
  return v;
}
__device__ __forceinline__ uint64_t wave_max(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = max(v, (uint64_t)__shfl_xor((unsigned long long)v, d));
  return v;
}
__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, d);
  return v;
}
// {lo, hi, sum, bad} of this thread's values, reduced over the block into out[0..3] by thread 0
__device__ __forceinline__ void block_reduce4(uint64_t lo, uint64_t hi, uint64_t sum, uint64_t bad, uint64_t* out) {
  __shared__ uint64_t red[4][kExtentBlock / 64];
  lo = wave_min(lo);
  hi = wave_max(hi);
  sum = wave_sum(sum);
  bad = wave_max(bad);
  const uint32_t w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = lo;
    red[1][w] = hi;
    red[2][w] = sum;
    red[3][w] = bad;
  }
  __syncthreads();
  if (threadIdx.x == 0 && out) {
    for (int k = 1; k < kExtentBlock / 64; k++) {
      lo = min(lo, red[0][k]);
      hi = max(hi, red[1][k]);
      sum += red[2][k];
      bad = max(bad, red[3][k]);
    }
    out[0] = lo;
    out[1] = hi;
    out[2] = sum;
    out[3] = bad;
  }
}

// Bucket of a non-empty payload at absolute address a: 1023 - its 128-byte line count (longest first).
// key: the payload's rounds in the sorted path (crc32_kernels.hip var_class_w8), R = ceil(lines / 8), descending
// (payloads of equal R run in lockstep; up to 8184 lines sort exactly, longer ones share bucket 0). Keying on R
// rather than on lines gives config 3 about 65 distinct buckets instead of about 520, so step 1 issues that many
// fewer global atomics per block.
__device__ __forceinline__ uint32_t bucket_of(uint64_t a, uint32_t len) {
  const uint32_t nl = (uint32_t)(((a + len - 1) >> 7) - (a >> 7) + 1);
  const uint32_t r = (nl + 7) >> 3;
  return (kBucketCount - 1) - (r < kBucketCount - 1 ? r : kBucketCount - 1);
}

// A payload the sorted path may run as segments (crc32_kernels.h kSplitSeg): longer than kSplitMin, with an index
// that fits the segment descriptors; its segment size (a uint32 length is < 4096 big segments, within the power
// tables' reach).
__device__ __forceinline__ bool split_eligible(const BucketArgs& bk, size_t i, uint32_t l) {
  return bk.split_slot && l > kSplitMin && i <= kSegIndexMask;
}
__device__ __forceinline__ uint32_t split_seg(uint32_t l) {
  return (uint64_t)l > (uint64_t)kSplitSeg * (kSplitMaxSegs - 1) ? kSplitSegBig : kSplitSeg;
}

// COUNT: step 1 of the counting sort (crc32_kernels.h BucketArgs) beside the extent.
template <bool COUNT>
__global__ __launch_bounds__(kExtentBlock) void crc32_extent_kernel(const uint64_t* __restrict__ off,
                                                                    const uint32_t* __restrict__ len, size_t n,
                                                                    uint64_t* ws, BucketArgs bk) {
  __shared__ uint32_t h[COUNT ? kBucketCount : 1];
  if constexpr (COUNT) {
    if (bk.choice.ws) {  // the device's choice (AutoChoice): nothing to do when it is the arena
      ArenaSpan sp;
      if (choose_arena(bk.choice, sp)) return;
    }
    for (uint32_t i = threadIdx.x; i < kBucketCount; i += kExtentBlock) h[i] = 0;
    __syncthreads();
  }
  uint64_t lo = ~0ull, hi = 0, sum = 0, bad = 0;
  const size_t stride = (size_t)gridDim.x * kExtentBlock;
  size_t i = blockIdx.x * (size_t)kExtentBlock + threadIdx.x;
  if constexpr (!COUNT) {
    // the extent alone: four payloads' descriptors in flight per thread (one at a time, a 2M-payload batch is 16
    // dependent rounds per thread on the 128-block grid: ~20 us; crc32_capi.cpp run_var_auto's device choice)
    for (; i + 3 * stride < n; i += 4 * stride) {
      uint64_t o[4], nx[4];
      uint32_t l[4];
      const bool has_next = i + 3 * stride + 1 < n;  // (only the fourth can be the batch's last payload)
#pragma unroll
      for (int u = 0; u < 4; u++) {
        o[u] = off[i + u * stride];
        l[u] = len[i + u * stride];
        nx[u] = off[u < 3 || has_next ? i + u * stride + 1 : i + u * stride];
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const bool last = u == 3 && !has_next;
        if (l[u]) {
          lo = min(lo, o[u]);
          hi = max(hi, o[u] + l[u]);
          sum += l[u];
        }
        if (!last) bad |= (nx[u] < o[u] || (nx[u] >= o[u] + l[u] && nx[u] - (o[u] + l[u]) >= 4096)) ? 1u : 0u;
      }
    }
  }
  for (; i < n; i += stride) {
    const uint64_t o = off[i], l = len[i];
    if (l) {
      lo = min(lo, o);
      hi = max(hi, o + l);
      sum += l;
    }
    if (i + 1 < n) {
      const uint64_t o2 = off[i + 1];
      bad |= (o2 < o || (o2 >= o + l && o2 - (o + l) >= 4096)) ? 1u : 0u;
    }
    if constexpr (COUNT) {
      if (l) {
        const uint64_t a = (uint64_t)(uintptr_t)bk.base + o;
        bool split = false;
        if (split_eligible(bk, i, (uint32_t)l)) {  // a long payload: claim its extra descriptors
          const uint32_t seg = split_seg((uint32_t)l);
          const uint32_t S = (uint32_t)((l + seg - 1) / seg);
          split = atomicAdd(bk.split_ctr, (unsigned long long)(S - 1)) + (S - 1) <= bk.split_cap;
          bk.split_slot[i] = split ? 1u : 0u;
          if (split) {  // the first segment, then S - 1 of seg bytes with the same alignment, one bucket
            if (bk.state) {  // update mode: the first segment starts from the register, the segments xor into 0
              bk.split_state[i] = bk.state[i];
              bk.state[i] = 0u;
            } else {
              bk.out[i] = ~0u;  // the segments xor into it (the complement of the init's)
            }
            const uint32_t l0 = (uint32_t)l - (S - 1) * seg;
            atomicAdd(&h[bucket_of(a, l0)], 1u);
            atomicAdd(&h[bucket_of(a + l0, seg)], S - 1);
          }
        }
        if (!split) atomicAdd(&h[bucket_of(a, (uint32_t)l)], 1u);
      } else if (bk.out) {
        bk.out[i] = 0u;  // crc of the empty string (update mode: the register is unchanged)
      }
    }
  }
  // (its barrier also orders h; with a device choice the partials are the extent kernel's, already in ws)
  block_reduce4(lo, hi, sum, bad, COUNT && bk.choice.ws ? nullptr : ws + 8 + 4 * (size_t)blockIdx.x);
  if constexpr (COUNT) {
    __syncthreads();
    uint32_t* row = bk.rows + (size_t)blockIdx.x * kBucketCount;
    for (uint32_t i = threadIdx.x; i < kBucketCount; i += kExtentBlock) {
      const uint32_t c = h[i];
      if (c) row[i] = __hip_atomic_fetch_add(bk.cursor + i, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Step 2 of the counting sort (crc32_kernels.h); the same grid and payload-to-block map as step 1.
__global__ __launch_bounds__(kBucketThreads) void crc32_bucket_place(const uint64_t* __restrict__ off,
                                                                     const uint32_t* __restrict__ len, size_t n,
                                                                     const uint64_t* ws, uint32_t parts, BucketArgs bk,
                                                                     ExtentHint* record, uint64_t seq) {
  static_assert(kBucketThreads == kBucketCount, "one bucket per thread");
  __shared__ uint32_t basep[kBucketCount];
  __shared__ uint32_t wtot[kBucketThreads / 64];
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (bk.choice.ws) {  // the device's choice (AutoChoice): when it is the arena, only the next call's sets are zeroed
    ArenaSpan sp;
    if (choose_arena(bk.choice, sp)) {
      if (blockIdx.x == 0) {
        bk.cursor_next[t] = 0u;
        if (bk.split_ctr_next && t == 0) *bk.split_ctr_next = 0ull;
      }
      return;
    }
  }
  // bucket totals (step 1's atomics, finished at the kernel boundary) -> exclusive bucket bases
  const uint32_t tot = __hip_atomic_load(bk.cursor + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t mine = bk.rows[(size_t)blockIdx.x * kBucketCount + t];  // valid where this block has payloads
  uint32_t v = tot;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t u = (uint32_t)__shfl_up((int)v, d);
    if (lane >= (uint32_t)d) v += u;
  }
  if (lane == 63) wtot[w] = v;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t k = 0; k < w; k++) before += wtot[k];
  const uint32_t start = before + v - tot;
  basep[t] = start + mine;
  if (blockIdx.x == 0) {
    bk.cursor_next[t] = 0u;
    if (bk.split_ctr_next && t == 0) *bk.split_ctr_next = 0ull;
    // one class: every non-empty payload (crc32_kernels.hip var_class_w8); ranges[2..5] empty
    if (t == 0) bk.ranges[0] = 0u;
    if (t == kBucketCount - 1)
      bk.ranges[1] = bk.ranges[2] = bk.ranges[3] = bk.ranges[4] = bk.ranges[5] = start + tot;
    if (record && w == 0) {
      uint64_t lo, hi, sum, bad;
      extent_of(ws, parts, lo, hi, sum, bad);
      if (t == 0) publish_extent(record, lo, hi, sum, bad, seq);
    }
  }
  __syncthreads();
  uint4* desc = static_cast<uint4*>(bk.desc);
  // every thread of the block runs the same iterations (the segment writes below take the whole wave)
  for (size_t i0 = blockIdx.x * (size_t)kBucketThreads; i0 < n; i0 += (size_t)gridDim.x * kBucketThreads) {
    const size_t i = i0 + t;
    const uint32_t l = i < n ? len[i] : 0u;
    const uint64_t a = (uint64_t)(uintptr_t)bk.base + (l ? off[i] : 0ull);
    const bool split = l && split_eligible(bk, i, l) && bk.split_slot[i];
    // segments: the first (the remainder), then S - 1 of seg bytes
    const uint32_t seg = split ? split_seg(l) : 1u, S = split ? (l + seg - 1) / seg : 1u, l0 = l - (S - 1) * seg;
    uint32_t pk = 0;
    if (l) {
      const uint32_t pos = atomicAdd(&basep[bucket_of(a, split ? l0 : l)], 1u);  // LDS atomic: rank in the block's slots
      desc[pos] = split ? make_uint4((uint32_t)a, (uint32_t)(a >> 32) | ((S - 1) << 16), l0,
                                     kSegFlag | kSegFirst | (seg == kSplitSegBig ? kSegBig : 0u) | (uint32_t)i)
                        : make_uint4((uint32_t)a, (uint32_t)(a >> 32), l, (uint32_t)i);
      if (split) pk = atomicAdd(&basep[bucket_of(a + l0, seg)], S - 1);
    }
    // the later S - 1 segments of each split payload, written by the whole wave (one thread wrote up to
    // 16k descriptors of a payload just under 256 MiB in a serial loop)
    uint64_t pend = __builtin_amdgcn_ballot_w64(split);
    while (pend) {
      const int src = __builtin_ffsll((long long)pend) - 1;
      pend &= pend - 1;
      const uint32_t sS = (uint32_t)__builtin_amdgcn_readlane((int)S, src);
      const uint32_t sseg = (uint32_t)__builtin_amdgcn_readlane((int)seg, src);
      const uint32_t spk = (uint32_t)__builtin_amdgcn_readlane((int)pk, src);
      const uint32_t si = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)i, src);
      const uint64_t a1 = a + l0;
      const uint64_t sa1 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(a1 >> 32), src) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a1, src);
      const uint32_t big = sseg == kSplitSegBig ? kSegBig : 0u;
      for (uint32_t k = 1 + lane; k < sS; k += 64) {
        const uint64_t ak = sa1 + (uint64_t)(k - 1) * sseg;
        desc[spk + k - 1] = make_uint4((uint32_t)ak, (uint32_t)(ak >> 32) | ((sS - 1 - k) << 16), sseg,
                                       kSegFlag | big | si);
      }
    }
  }
}

}  // namespace

unsigned bucket_grid(size_t n) {
  // about one payload per thread (the launches are latency-bound), up to kExtentMaxParts blocks
  static const size_t per = (size_t)std::max(1, ANNETY_AB_KNOB("ANNETY_CRC_BUCKET_PER", 1));  // A/B: payloads per thread
  const size_t chunk = per * kExtentBlock;
  return (unsigned)std::max<size_t>(1, std::min<size_t>((n + chunk - 1) / chunk, kExtentMaxParts));
}

hipError_t launch_extent(const uint64_t* off, const uint32_t* len, size_t n, void* ws, uint32_t* parts,
                         const BucketArgs* bk, hipStream_t stream) {
  const unsigned blocks = bucket_grid(n);
  *parts = blocks;
  note_kernel(bk ? "crc32_extent_kernel<count>" : "crc32_extent_kernel");
  if (bk)
    hipLaunchKernelGGL(crc32_extent_kernel<true>, dim3(blocks), dim3(kExtentBlock), 0, stream, off, len, n,
                       static_cast<uint64_t*>(ws), *bk);
  else
    hipLaunchKernelGGL(crc32_extent_kernel<false>, dim3(blocks), dim3(kExtentBlock), 0, stream, off, len, n,
                       static_cast<uint64_t*>(ws), BucketArgs{});
  return hipGetLastError();
}

hipError_t launch_bucket_place(const uint64_t* off, const uint32_t* len, size_t n, const void* ws, uint32_t parts,
                               const BucketArgs& bk, ExtentHint* record, uint64_t seq, hipStream_t stream) {
  note_kernel("crc32_bucket_place");
  hipLaunchKernelGGL(crc32_bucket_place, dim3(bucket_grid(n)), dim3(kBucketThreads), 0, stream, off, len, n,
                     static_cast<const uint64_t*>(ws), parts, bk, record, seq);
  return hipGetLastError();
}

LineOut line_out(const ArenaLaunch& a, const ArenaGeom& geo) {
  LineOut ar;
  ar.S = a.scratch;
  ar.SB = a.scratch + geo.sb_off;
  ar.S_edge = a.scratch + geo.edge_off;
  ar.SB_edge = ar.S_edge + 128;
  ar.W = geo.W;
  ar.byte_lo = a.byte_lo;
  ar.byte_hi = a.byte_hi;
  ar.line_lo = a.line_lo;
  ar.line_hi = a.line_hi;
  ar.sb0 = a.sb0;
  ar.nsb = a.nsb;
  ar.fs0 = a.fs0;
  ar.fs1 = a.fs1;
  ar.zero_line = (uint64_t)(uintptr_t)a.zero_line;
  ar.check = a.check;
  ar.check_parts = a.check_parts;
  ar.check_lo = a.check_lo;
  ar.check_any_order = a.check_any_order;
  ar.check_hi = a.check_hi;
  ar.choice = a.choice;  // (with a device choice the kernel derives the geometry from S = the scratch)
  ar.probe_delta = 0;
  return ar;
}

// Lanes per payload in the stitch: a wave each when the batch has few payloads (at most 8 per CU), so that the wave
// can share a long payload's superblock runs (mid_join; 16 frames of 64 MiB ran their runs on 16 lanes of one wave
// in ~1.3 ms); one lane each otherwise.
uint32_t stitch_spread(const ArenaLaunch& a) { return a.n <= a.max_blocks * (kStitchBlock / 64) ? 64u : 1u; }

size_t stitch_blocks(const ArenaLaunch& a, size_t blk = kStitchBlock) {
  return std::max<size_t>(1, std::min<size_t>(a.max_blocks, (a.n * stitch_spread(a) + blk - 1) / blk));
}

StitchGeo stitch_geo(const ArenaLaunch& a, const ArenaGeom& geo) {
  StitchGeo s;
  s.base = static_cast<const uint8_t*>(a.base);
  s.byte_lo = a.byte_lo;
  s.byte_hi = a.byte_hi;
  s.line_lo = a.line_lo;
  s.line_hi = a.line_hi;
  s.sb0 = a.sb0;
  s.fs0 = a.fs0;
  s.fs1 = a.fs1;
  s.W = geo.W;
  s.L = (uint32_t)geo.blocks;
  s.S = a.scratch;
  s.SB = a.scratch ? a.scratch + geo.sb_off : nullptr;
  s.S_edge = a.scratch ? a.scratch + geo.edge_off : nullptr;
  s.SB_edge = a.scratch ? a.scratch + geo.edge_off + 128 : nullptr;
  s.W0 = a.scratch ? a.scratch : a.len;
  s.sb_word = (uint32_t)geo.sb_off;
  s.edge_word = (uint32_t)geo.edge_off;
  s.Lmagic = ((1ull << 40) + geo.blocks - 1) / geo.blocks;
  s.off = a.off;
  s.len = a.len;
  s.n = a.n;
  s.zero_line = (uint64_t)(uintptr_t)a.zero_line;
  s.out = a.out;
  s.ok = a.ok;
  s.check = a.check;
  s.check_parts = a.check_parts;
  s.check_lo = a.check_lo;
  s.check_any_order = a.check_any_order;
  s.check_hi = a.check_hi;
  s.record = a.record;
  s.record_seq = a.record_seq;
  s.choice = a.choice;  // (with a device choice the kernel derives the geometry from W0 = the scratch)
  s.pow8k = static_cast<const uint32_t*>(a.pow8k);
  s.spread = stitch_spread(a);
  return s;
}

// The geometry the host launches with: the arena's, or with a device choice (ArenaLaunch::choice) the line pass on
// choice.blocks workgroups over a span the kernels find themselves.
ArenaGeom launch_geom(const ArenaLaunch& a) {
  return a.choice.ws ? arena_geom_of(0, a.choice.blocks) : arena_geom(a);
}

template <int PROBE, int PIPE = 0, int BLK = kStitchBlock>
hipError_t launch_stitch_p(const ArenaLaunch& a, hipStream_t stream) {
  const StitchGeo s = stitch_geo(a, launch_geom(a));
  const size_t blocks = stitch_blocks(a, BLK);
  const uint4* img_slice = static_cast<const uint4*>(a.img_slice);
  const uint4* img_stitch = static_cast<const uint4*>(a.img_stitch);
  if (a.ok && !a.update) {  // LengthHeaderCodec verify: the trailer compare in the stitch
    note_kernel("crc32_arena_stitch_kernel<verify>");
    hipLaunchKernelGGL((crc32_arena_stitch_kernel<false, BLK, PROBE, PIPE, true>), dim3((unsigned)blocks),
                       dim3(BLK), 0, stream, s, img_slice, img_stitch);
    return hipGetLastError();
  }
  note_kernel("crc32_arena_stitch_kernel");
  if (a.update)
    hipLaunchKernelGGL((crc32_arena_stitch_kernel<true, BLK, PROBE, PIPE>), dim3((unsigned)blocks), dim3(BLK), 0,
                       stream, s, img_slice, img_stitch);
  else
    hipLaunchKernelGGL((crc32_arena_stitch_kernel<false, BLK, PROBE, PIPE>), dim3((unsigned)blocks), dim3(BLK), 0,
                       stream, s, img_slice, img_stitch);
  return hipGetLastError();
}

template <int PROBE, bool NT = true>
hipError_t launch_arena_lines_p(const ArenaLaunch& a, hipStream_t stream) {
  static_assert(kBlock / 8 == 64 && kSTasks % 4 == 0, "arena_geom / arena_s_word assume 64 groups per block, bursts of 4k tasks");
  const ArenaGeom geo = launch_geom(a);
  // the first full superblock, or with a device choice the batch's base (the kernel moves to the span it finds)
  const uint8_t* base = a.choice.ws ? static_cast<const uint8_t*>(a.base)
                                    : reinterpret_cast<const uint8_t*>((uintptr_t)(a.fs0 * 8192));
  note_kernel("crc32_arena_lines_kernel");
  hipLaunchKernelGGL((crc32_arena_lines_kernel<PROBE, NT>), dim3((unsigned)geo.blocks), dim3(kBlock), 0, stream, base,
                     line_out(a, geo), static_cast<const uint4*>(a.img_slice), static_cast<const uint4*>(a.img_group8),
                     static_cast<const uint4*>(a.img_sb));
  return hipGetLastError();
}

// The line pass reads each superblock as 8 coalesced nontemporal 1 KiB loads (crc32_arena_lines.h); A/B builds
// select the per-line loads with ANNETY_CRC_LINES_NT=0.
hipError_t launch_arena_lines(const ArenaLaunch& a, hipStream_t stream) {
#ifdef ANNETY_CRC_AB
  static const bool nt = ANNETY_AB_KNOB("ANNETY_CRC_LINES_NT", 1) != 0;
  static const int probe = ANNETY_AB_KNOB("ANNETY_CRC_LINES_PROBE", 0);  // 1: no S stores (wrong digests)
  if (!nt) return launch_arena_lines_p<0, false>(a, stream);
  if (probe == 1) return launch_arena_lines_p<1, true>(a, stream);
#endif
  return launch_arena_lines_p<0, true>(a, stream);
}

hipError_t launch_arena(const ArenaLaunch& a, hipStream_t stream) {
  if (a.nsb || a.choice.ws) {
    const hipError_t e = launch_arena_lines(a, stream);
    if (e != hipSuccess) return e;
  }
  // The stitch issues a lane's next payload loads before folding the current one (PIPE 1): config-3 step
  // 0.2139-0.2142 ms vs 0.2144-0.2151 without, same box, three alternating pairs
  // (profiles/r02/stitch_pipe_bench_ab/). 768-lane blocks with one payload in flight (3 waves per SIMD under a
  // 168-VGPR cap, no spill) measured 21.3 us against 20.4 for this 512-lane form (profiles/r03/stitch_ab/):
  // occupancy is not what bounds it. A/B builds: ANNETY_CRC_STITCH_PIPE=0 (one payload at a time). (A one-level join
  // of up to 7 whole superblocks from a table of shift_{c 8KiB} maps measured no faster than the chain, and was
  // dropped in round 6 for the window masks' tables.)
#ifdef ANNETY_CRC_AB
  static const bool pipe = ANNETY_AB_KNOB("ANNETY_CRC_STITCH_PIPE", 1) != 0;
  static const int probe = ANNETY_AB_KNOB("ANNETY_CRC_STITCH_PROBE", 0);  // Stitcher PROBE (wrong digests)
  if (probe == 1) return launch_stitch_p<1, 1>(a, stream);
  if (probe == 2) return launch_stitch_p<2, 1>(a, stream);
  if (probe == 3) return launch_stitch_p<3, 1>(a, stream);
  if (probe == 4) return launch_stitch_p<4, 1>(a, stream);
  if (probe == 5) return launch_stitch_p<5, 1>(a, stream);
  if (!pipe) return launch_stitch_p<0>(a, stream);
#endif
  return launch_stitch_p<0, 1>(a, stream);
}

}  // namespace annety_crc
