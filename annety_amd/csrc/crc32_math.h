// Shared host/device arithmetic for annety's checksum (reflected CRC-32/ISO-HDLC, poly 0xEDB88320).
//
// Reference semantics (restated, not copied):
//   include/Crc32c.h:58-69  crc32_long  : c = ~0; for each byte c = T[(c ^ b) & 0xff] ^ (c >> 8); return ~c
//   include/Crc32c.h:41-55  crc32_short : same value via two 16-entry nibble steps per byte
//   include/Crc32c.h:71-82  crc32_update: the raw register loop without init / final xor
//   src/Crc32c.cc:20-92     the 16- and 256-entry tables (generated here from the polynomial)
//
// Everything on the batch path is linear algebra over GF(2) on the 32-bit raw register:
//   raw(M, s)         = register after absorbing bytes M from state s
//   raw(A||B, s)      = shift_|B|(raw(A, s)) ^ raw(B, 0)
//   shift_n(s)        = register after absorbing n zero bytes = the linear map x^(8n) mod P
// The GPU kernels split each payload into 128-byte chunks owned by different lanes and re-join the
// per-lane registers with precomputed shift_n maps.
#pragma once

#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define ANNETY_HD __host__ __device__
#else
#define ANNETY_HD
#endif

namespace annety_crc {

constexpr uint32_t kPoly = 0xEDB88320u;  // reflected IEEE 802.3 polynomial (src/Crc32c.cc:8-9, table256[1])
constexpr uint32_t kInit = 0xFFFFFFFFu;  // include/Crc32c.h:62
constexpr uint32_t kXorOut = 0xFFFFFFFFu;  // include/Crc32c.h:68

// One zero bit through the reflected register.
ANNETY_HD constexpr uint32_t step_bit(uint32_t c) { return (c >> 1) ^ (kPoly & (0u - (c & 1u))); }

// Register after n zero BITS (bit-serial; used for table generation and small shifts only).
ANNETY_HD constexpr uint32_t shift_bits(uint32_t c, uint64_t nbits) {
  for (uint64_t i = 0; i < nbits; i++) c = step_bit(c);
  return c;
}

// table256[i] (src/Crc32c.cc:27-92) and the slicing tables T_k[e] = register after byte e followed by
// k more zero bytes, i.e. 8*(k+1) bit steps from e.
ANNETY_HD constexpr uint32_t table256_entry(uint32_t e) { return shift_bits(e, 8); }
ANNETY_HD constexpr uint32_t slice_entry(int k, uint32_t e) { return shift_bits(e, 8u * (unsigned)(k + 1)); }

// ---- GF(2) 32x32 matrices (columns = image of each bit) for arbitrary byte shifts, host side ----
struct Gf2Mat {
  uint32_t col[32];
};

ANNETY_HD inline uint32_t gf2_apply(const Gf2Mat& m, uint32_t v) {
  uint32_t r = 0;
  for (int i = 0; v; i++, v >>= 1)
    if (v & 1u) r ^= m.col[i];
  return r;
}

ANNETY_HD inline Gf2Mat gf2_mul(const Gf2Mat& a, const Gf2Mat& b) {  // a after b
  Gf2Mat r{};
  for (int i = 0; i < 32; i++) r.col[i] = gf2_apply(a, b.col[i]);
  return r;
}

// Matrix of shift by n zero bytes, by binary powering of the one-byte map. O(32*32*log n).
inline Gf2Mat shift_matrix(uint64_t nbytes) {
  Gf2Mat byte{}, acc{};
  for (int i = 0; i < 32; i++) {
    byte.col[i] = shift_bits(1u << i, 8);
    acc.col[i] = 1u << i;
  }
  while (nbytes) {
    if (nbytes & 1) acc = gf2_mul(byte, acc);
    byte = gf2_mul(byte, byte);
    nbytes >>= 1;
  }
  return acc;
}

inline uint32_t shift_bytes(uint32_t c, uint64_t nbytes) { return gf2_apply(shift_matrix(nbytes), c); }

// crc(A||B) from the FINAL values crc(A), crc(B) and |B| (zlib's identity; the init/xorout terms cancel).
inline uint32_t combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) { return shift_bytes(crc_a, len_b) ^ crc_b; }

// ---- LDS image layout of the batch kernels (bytes); see DESIGN.md §2 ----
// [0, 128 KiB)          slicing-by-4 tables as two paired slots, 32 replicas:
//                         pair P, entry e, replica r at P*65536 + e*256 + r*8 = {lo, hi}
//                         P=0: {T3[e], T2[e]}   P=1: {T1[e], T0[e]}
//                       read with ds_read_b64: address = one v_perm_b32, 32 lanes hit 32 distinct
//                       8-byte slots of the 64-bank row -> conflict-free.
// [128 KiB, +512 B)     half-line join: (k, v) = shift_64(v << 4k), uniform (broadcast reads). A line is
//                       folded as two independent 64-byte chains (2x ILP) joined by this map.
// [+512 B, +16 KiB)     lane-position join tables for a lane-group of G lanes, 32 replicas:
//                         (k nibble, v value, slot s) at kLdsJoinOff + k*2048 + v*128 + s*4
//                         = shift_{(G-1-j)*128}(v << 4k), j = s & (G-1)
// [.., +512 B)          round-advance tables (uniform across lanes -> broadcast reads):
//                         (k, v) at kLdsRoundOff + k*64 + v*4 = shift_{(G-1)*128}(v << 4k)
constexpr uint32_t kLdsSliceBytes = 131072;
constexpr uint32_t kLdsHalfOff = 131072;
constexpr uint32_t kLdsCommonBytes = kLdsHalfOff + 512;  // slicing + half-line join: same for every G
constexpr uint32_t kLdsJoinOff = kLdsCommonBytes;        // 131584
constexpr uint32_t kLdsJoinBytes = 16384;
constexpr uint32_t kLdsRoundOff = kLdsJoinOff + kLdsJoinBytes;  // 147968
constexpr uint32_t kLdsRoundBytes = 512;
constexpr uint32_t kLdsImageBytes = kLdsRoundOff + kLdsRoundBytes;  // 148480
constexpr uint32_t kGroupImageBytes = kLdsJoinBytes + kLdsRoundBytes;  // per-G part
// Variable-length kernel only: two-level inverse-shift tables (8 x 16 nibble entries per map)
//   [kLdsUnshiftOff, +8 KiB)  U_lo[m] = shift_{-m} bytes, m = 0..15
//   [+8 KiB, +4 KiB)          U_hi[h] = shift_{-16h} bytes, h = 0..7 -> shift_{-over} = U_hi[over>>4] o U_lo[over&15]
constexpr uint32_t kLdsUnshiftOff = kLdsImageBytes;
constexpr uint32_t kLdsUnshiftBytes = 24 * 512;
constexpr uint32_t kLdsVarImageBytes = kLdsUnshiftOff + kLdsUnshiftBytes;  // 160768 <= 163840
constexpr uint32_t kChunkBytes = 128;  // one cache line per lane per round
// Arena path (crc32_arena.hip), bulk line kernel: common + G=8 group part + superblock join
//   [kLdsImageBytes, +4 KiB)  (k nibble, v value, g group) at k*512 + v*32 + g*4 = shift_{(7-g)*1024}(v << 4k)
constexpr uint32_t kLdsSbJoinOff = kLdsImageBytes;
constexpr uint32_t kLdsSbJoinBytes = 4096;
constexpr uint32_t kLdsArenaImageBytes = kLdsSbJoinOff + kLdsSbJoinBytes;  // 152576
// Half-line join as byte tables for the coalesced nontemporal kernels (crc32_device.h fold_halves): 4 tables
// x 256 words, B_k[e] = shift_64(e << 8k), after the fixed image or after the arena image (the device buffer
// holding the superblock join holds it right behind, so the arena stages both in one piece).
constexpr uint32_t kLdsByteMapBytes = 4096;
constexpr uint32_t kLdsFixedNtImageBytes = kLdsImageBytes + kLdsByteMapBytes;     // 152576
// G = 32 rounds (crc32_fixed32_nt_kernel): the round advance shift_{31*128} as byte tables too, after the
// half-line join's
constexpr uint32_t kLdsFixed32NtImageBytes = kLdsFixedNtImageBytes + kLdsByteMapBytes;  // 156672
constexpr uint32_t kLdsArenaNtImageBytes = kLdsArenaImageBytes + kLdsByteMapBytes;  // 156672
// Arena path, stitch kernel: common + segment maps + inverse shifts + quarter-line join (no group part)
//   [kLdsMapOff, +16 KiB)  set of 32 maps, (k, i, v) at (k*32 + i)*64 + v*4: i = m-1: F(m) = shift_{128m}
//                          (m = 1..8), 7+m: G(m) = shift_{1024m}, 16+q: UL(q) = shift_{-128q},
//                          24+q: UB(q) = shift_{-1024q} (q = 0..7)
//   [kLdsStitchUnshiftOff, +8 KiB)  set U_lo[m] = shift_{-m}, (k, m, v) at (k*16 + m)*64 + v*4
//   [+8 KiB, +12 KiB)                set U_hi[h] = shift_{-16h}, (k, h, v) at (k*8 + h)*64 + v*4
//   [kLdsQuarterOff, +512)  shift_32 (joins the two 32-byte chains of a half-line window)
//   [kLdsStitchMaskOff, +544 B)  byte masks of a 16-byte chunk (as kLdsW8MaskOff): the windows' kept bytes
constexpr uint32_t kLdsMapOff = kLdsCommonBytes;
constexpr uint32_t kLdsMapBytes = 32 * 512;
constexpr uint32_t kMapF = 0, kMapG = 8, kMapUL = 16, kMapUB = 24;  // map index of F(1), G(1), UL(0), UB(0)
constexpr uint32_t kLdsStitchUnshiftOff = kLdsMapOff + kLdsMapBytes;
constexpr uint32_t kLdsQuarterOff = kLdsStitchUnshiftOff + kLdsUnshiftBytes;
constexpr uint32_t kLdsStitchMaskOff = kLdsQuarterOff + 512;
constexpr uint32_t kLdsStitchImageBytes = kLdsStitchMaskOff + 544;  // 161312
// Length-sorted path (crc32_kernels.hip var_class_w8): common part, then the
// device image "w8" (kW8ImgBytes):
//   [kLdsW8JoinOff, +4 KiB)     lane-position join, unreplicated: (k, v, j) at (k*16 + v)*32 + j*4 =
//                               shift_{(7-j)*128}(v << 4k) (used once per payload: bank conflicts are harmless)
//   [kLdsW8HalfOff, +4 KiB)     byte tables of the half-line join shift_64 (crc32_device.h byte_map64)
//   [kLdsW8RoundOff, +4 KiB)    byte tables of the round advance shift_{7*128}
//   [kLdsW8UnshiftOff, +12 KiB) U_lo[m] = shift_{-m} (m = 0..15), U_hi[h] = shift_{-16h} (h = 0..7), 512 B each
//   [kLdsW8InitOff, +512 B)     shift_{128-lead}(kInit), lead = 0..127: the init as a register at line 0's end
//   [kLdsW8MaskOff, +544 B)     byte masks of a 16-byte chunk: KEEP_FROM[a] = bytes [a, 16), a = 0..16, then
//                               KEEP_TO[b] = bytes [0, b), b = 0..16 (crc32_device.h mask_chunks)
constexpr uint32_t kLdsW8JoinOff = kLdsCommonBytes;
constexpr uint32_t kLdsW8HalfOff = kLdsW8JoinOff + 4096;
constexpr uint32_t kLdsW8RoundOff = kLdsW8HalfOff + 4096;
constexpr uint32_t kLdsW8UnshiftOff = kLdsW8RoundOff + 4096;
constexpr uint32_t kLdsW8InitOff = kLdsW8UnshiftOff + kLdsUnshiftBytes;
constexpr uint32_t kLdsW8MaskOff = kLdsW8InitOff + 512;
constexpr uint32_t kLdsW8ImageBytes = kLdsW8MaskOff + 544;            // 157216
constexpr uint32_t kW8ImgBytes = kLdsW8ImageBytes - kLdsCommonBytes;  // 25632
// The frame encode with lane groups of 4 (crc32_frames.hip lhc_encode_fused_kernel<P, 4>) advances its columns by 4
// lines per round: byte tables of shift_{3*128} right after the w8 image (the device buffer holds them behind it;
// the sorted kernel stages only kLdsW8ImageBytes)
constexpr uint32_t kLdsW8Round4Off = kLdsW8ImageBytes;
constexpr uint32_t kLdsEnc4ImageBytes = kLdsW8Round4Off + 4096;  // 161312
constexpr uint32_t kW8ImgAllBytes = kLdsEnc4ImageBytes - kLdsCommonBytes;
// after the image: each wave's ring of 4 claimed sets' descriptors (8 x 16 B a set), their set indices, and the
// block's set counters (front, back: 2 x 32 bits of one 64-bit word)
// The sorted kernel's block: 768 threads (12 waves: 3 per SIMD at <= 168 VGPRs) share the one LDS image.
constexpr int kW8Block = 768;
constexpr uint32_t kW8MaxWaves = 12;
constexpr uint32_t kLdsW8RingOff = kLdsW8ImageBytes;
constexpr uint32_t kLdsW8RingSetOff = kLdsW8RingOff + kW8MaxWaves * 4 * 128;
constexpr uint32_t kLdsW8CounterOff = kLdsW8RingSetOff + kW8MaxWaves * 4 * 4;
constexpr uint32_t kLdsW8TotalBytes = kLdsW8CounterOff + 16;  // 163568 <= 163840

}  // namespace annety_crc
