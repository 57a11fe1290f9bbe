// Internal launcher interface between the C-ABI shim (crc32_capi.cpp) and the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

// A/B switches of the design-space harnesses (microbench/): the environment is read only in builds compiled
// with -DANNETY_CRC_AB. The product library always runs the measured defaults, so no environment variable can
// change a digest or a kernel choice (probe modes that wrote wrong digests were reachable from the
// environment). ANNETY_AB_KNOB(name, default) is the integer value of environment variable `name`.
#ifdef ANNETY_CRC_AB
#include <cstdlib>
#define ANNETY_AB_KNOB(name, dflt)                 \
  ([]() -> int {                                   \
    const char* e_ = std::getenv(name);            \
    return e_ && *e_ ? std::atoi(e_) : (int)(dflt); \
  }())
#else
#define ANNETY_AB_KNOB(name, dflt) ((int)(dflt))
#endif

namespace annety_crc {

struct ShiftCols {
  uint32_t c[32];  // columns of a GF(2) 32x32 matrix (passed by value in the kernarg segment)
};

// The automatic variable path's choice ON THE DEVICE (annety_crc32_batch_var with offset/length arrays the host has
// no record for): one call enqueues the extent kernel, then both paths' launches; each launch reduces this call's
// extent from the extent partials (ws, parts) and runs only if the choice is its own (crc32_device.h choose_arena):
// the arena path iff the batch is dense (payload bytes >= 2/3 of the span), sorted with gaps < 4 KiB (every byte of
// the span then lies on a page holding payload bytes) and its scratch fits cap_words; else the sorted path. The
// arena launches derive their geometry from the span (line pass on `blocks` workgroups). ws == null: no choice
// (the host chose).
struct AutoChoice {
  const uint64_t* ws;  // launch_extent's partials
  uint32_t parts;
  uint32_t blocks;     // the arena line pass's workgroups (its grid)
  uint64_t base;       // the batch's base address (payload offsets are relative to it)
  uint64_t cap_words;  // scratch words the arena path may use
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
  const void* img_bytemap; // kLdsByteMapBytes of half-line join byte tables (the nontemporal kernels)
  ShiftCols raw_shift_cols;  // raw only: shift_len columns
  uint32_t* out;           // digests (device)
  size_t max_blocks;       // persistent grid size (one workgroup per CU)
};

hipError_t launch_fixed(const FixedLaunch& a, hipStream_t stream);

struct VarLaunch {
  const void* base;          // device base pointer
  size_t n;                  // payload count
  uint64_t fixed_stride;     // direct mode (desc == null): payload i at base + i*fixed_stride,
  uint32_t fixed_len;        //   fixed_len bytes
  const void* desc;          // sorted mode: uint4 {addr lo, addr hi, len, index} per task (launch_bucket_place)
  const uint32_t* range;     // sorted mode: device [begin, end) into desc for this class
  uint32_t group;            // lanes per payload
  const void* img_slice;
  const void* img_group;
  const void* img_unshift;   // 12 KiB two-level inverse-shift tables (LDS image part 3)
  uint32_t* out;             // digests, or (update) the register array, read and written in place
  size_t max_blocks;
  bool update;               // crc32_update semantics instead of crc32_long
  AutoChoice choice;         // the sorted kernel: run only if the device chose the sorted path (ws null: always)
};

hipError_t launch_var(const VarLaunch& a, hipStream_t stream);
// Long payloads on the sorted path (digest mode): a payload of more than kSplitMin bytes runs as end-aligned
// segments of kSplitSeg bytes (kSplitSegBig past kSplitSeg * kSplitMaxSegs; the first segment takes the
// remainder), each a task of the sorted list, so that one long payload no longer serialises its rounds on one lane
// group. A segment's descriptor carries kSegFlag (| kSegFirst for the first, | kSegBig) | the payload's index in
// .w and m = the segments after it in bits 16-31 of .y (addresses are 48-bit). The group that finishes a segment
// applies shift_{m seg} to its raw register (the first from the init, the others from 0) from the power table and
// xors it into out[payload], which the count step preset to ~0, so the digest = ~xor_k shift_{m_k seg}(raw_k)
// needs no join. Update mode (crc32_update, include/Crc32c.h:71-82) splits the same way: the count step moves the
// payload's register to SortedSplit::state and presets out[payload] to 0, the first segment starts from that
// register, and the segments' xor is the new register (no final complement). Extra descriptors are claimed in the
// count step up to BucketArgs::split_cap (<= kSplitSegCap) per call; a payload that finds none runs whole.
// Payload indices are 31-bit (bit 31 = kSegFlag); only payloads with index <= kSegIndexMask can split.
constexpr uint32_t kSplitSeg = 16384;
constexpr uint32_t kSplitSegBig = 1u << 20;
constexpr uint32_t kSplitMin = 131072;
constexpr uint32_t kSplitMaxSegs = 16384;      // the power tables' reach (crc32_capi.cpp kMaxSegs)
constexpr uint32_t kSplitSegCap = 1u << 18;    // extra descriptors per call, at most
constexpr uint32_t kSegFlag = 0x80000000u, kSegFirst = 0x40000000u, kSegBig = 0x20000000u,
                   kSegIndexMask = 0x1FFFFFFFu;
constexpr uint64_t kSortedMaxPayloads = 0x7FFFFFFFull;  // the sorted list's descriptor indices (bit 31 = kSegFlag)
struct SortedSplit {
  const uint32_t* powers;      // powers[(m-1)*32 + bit] = shift_{m*kSplitSeg}(1 << bit), m = 1..kSplitMaxSegs-1
  const uint32_t* powers_big;  // the same for kSplitSegBig
  const uint32_t* state;       // update mode: a split payload's register before it (BucketArgs::split_state)
};
// The sorted path in one launch (a.range[0..1] = the sorted list's bounds in a.desc); img_w8 = the w8 image
// (kW8ImgBytes, crc32_math.h); a.group, a.img_group and a.img_unshift are ignored.
hipError_t launch_var_sorted(const VarLaunch& a, const void* img_w8, const SortedSplit& split, hipStream_t stream);

// Long payloads cut into end-aligned segments (crc32_kernels.hip): descriptors for the variable kernel,
// then the combine fold with powers[(m-1)*32 + bit] = shift_{m*seg}(1 << bit), m = 1..S-1.
hipError_t launch_split_desc(const void* base, size_t n, uint64_t len, uint64_t stride, uint64_t seg, uint32_t S,
                             void* desc, uint32_t* range, hipStream_t stream);
hipError_t launch_split_join(const uint32_t* seg_crc, size_t n, uint32_t S, const uint32_t* powers, uint32_t* out,
                             hipStream_t stream);

// Extent of a variable batch, for the automatic choice between the arena and the sorted path: over the
// non-empty payloads lo = min offset, hi = max end, sum = total bytes; bad != 0 unless every payload starts
// at or after the previous one and within 4 KiB of its end (then every byte of [lo, hi) lies on a page that
// also holds payload bytes, so the arena path reads only mapped memory). ExtentResult = {lo, hi, sum, bad}.
// Written to the device scratch `ws` (kExtentScratchBytes) and to the pinned host record `host`
// (ExtentHint), whose `chk` = lo ^ hi ^ sum ^ bad ^ seq ^ kExtentCheck lets the host reject a record it read
// while the device was rewriting it.
constexpr size_t kExtentScratchBytes = 16384 + 64;  // + the sorted path's two split counter sets (kSplitCtrOff)
constexpr uint32_t kExtentMaxParts = 128;  // partials (uint64 {lo, hi, sum, bad} at word 8 + 4b)
constexpr uint64_t kExtentCheck = 0x9E3779B97F4A7C15ull;
struct ExtentHint {
  uint64_t lo, hi, sum, bad;
  uint64_t seq, chk;
};
// Arena path (crc32_arena.hip): bulk line pass over the arena [byte_lo, byte_hi) (absolute 128-byte
// lines line_lo..line_hi, superblocks of 64 lines from sb0, nsb of them; nsb = 0 skips the pass), then
// the per-payload stitch. DESIGN.md §2.8.
struct ArenaLaunch {
  const void* base;          // payload offsets are relative to this pointer
  uint64_t byte_lo, byte_hi; // the arena, absolute addresses (byte_lo == byte_hi: none, every payload folded directly)
  uint64_t line_lo, line_hi; // its lines
  uint64_t sb0, nsb;         // superblocks (64 lines) overlapping the arena
  uint64_t fs0, fs1;         // the ones wholly inside it: [fs0, fs1), absolute superblock indices
  const uint64_t* off;       // device, n entries
  const uint32_t* len;       // device, n entries
  size_t n;
  uint32_t* scratch;         // arena_geom(*this).words words (device)
  const void* img_slice;     // common image part (slicing tables + half-line join)
  const void* img_group8;    // G = 8 group part (lane join + round maps)
  const void* img_sb;        // superblock join, kLdsSbJoinBytes, then the half-line join byte tables
  const void* img_stitch;    // stitch maps, kLdsStitchImageBytes - kLdsCommonBytes
  const void* zero_line;     // 128 zero bytes (device), read in place of lines outside the arena
  uint32_t* out;             // digests, or (update) registers in place; may be null when ok is set
  // LengthHeaderCodec verify (crc32_frames.hip): ok[p] = (digest == the big-endian 4-byte trailer at the payload's
  // end), written by the stitch; null = digests only
  uint8_t* ok;
  size_t max_blocks;
  bool update;
  // automatic path selection (annety_crc32_batch_var): the arena was declared from an earlier call's
  // extent; both launches first reduce this call's extent from the launch_extent partials (check,
  // check_parts; same stream) and compare it with [check_lo, check_hi) - on any difference the line pass
  // does nothing and every payload is folded directly from its own bytes (no read outside the payloads).
  // The stitch also publishes the reduced extent to `record` (seq = record_seq). null = no check.
  const uint64_t* check;
  uint32_t check_parts;
  uint64_t check_lo, check_hi;
  bool check_any_order;      // the recorded span lies in one allocation: unsorted or gapped batches qualify
  ExtentHint* record;
  uint64_t record_seq;
  // the device's choice (AutoChoice): the launches run only if it is the arena, with the geometry of this call's span
  // (byte_lo .. fs1 above are then unused) and `scratch` of choice.cap_words words
  AutoChoice choice;
  // pow8k[(m-1)*32 + bit] = shift_{m*8KiB}(1 << bit), m = 1..kSplitMaxSegs-1: the stitch's long superblock runs
  const void* pow8k;
};

// Counting sort of a variable batch by rounds (ceil(128-byte lines / 8)), longest first, for the sorted path:
// two launches, no host round trip and no memset per call.
//  1. launch_extent with `bk`: besides the extent partials, each block histograms its payloads by that key in
//     LDS and claims its slots in every bucket it uses with one agent-scope atomic add on that bucket's cursor
//     (rows[b][i] = the value returned = block b's first slot inside bucket i, in arrival order),
//     and writes out[p] = 0 for zero-length payloads (out null in update mode: their registers stay).
//  2. launch_bucket_place: every block scans the 1024 cursor totals into bucket bases, ranks its payloads
//     inside its slots with LDS atomics and writes desc[] (16 B per non-empty payload); block 0 writes the
//     class ranges and zeroes the other cursor set for the next call (the two sets alternate per call, so
//     the cursors are zero when a call's first launch starts), and, with `record`, publishes the extent.
// The order of payloads inside a bucket depends on arrival order; the digests do not.
constexpr uint32_t kBucketCount = 1024;
constexpr uint32_t kBucketThreads = 1024;  // both launches; one payload per thread per grid stride
constexpr size_t kCursorOff = 8192;        // the two cursor sets, in the extent scratch (2 x 4 KiB)
constexpr size_t kSplitCtrOff = kCursorOff + 2 * 4 * kBucketCount;  // 2 sets of 4 uint64 (split counters)
static_assert((8 + 4 * kExtentMaxParts) * 8 <= kCursorOff && kSplitCtrOff + 2 * 32 <= kExtentScratchBytes,
              "extent scratch layout");
// The ranges area (BucketArgs::ranges): the classes' bounds and two spare words
constexpr uint32_t kRangeWords = 8;
struct BucketArgs {
  const void* base;       // payload offsets are relative to this pointer
  uint32_t* rows;         // bucket_grid(n) * kBucketCount words
  uint32_t* cursor;       // this call's set (zero on entry)
  uint32_t* cursor_next;  // the other set: zeroed by launch_bucket_place
  uint32_t* ranges;       // kRangeWords: [0, 1] = {begin, end} of the sorted list in desc, [2..5] empty
  void* desc;             // uint4 {addr lo, addr hi, len, index} per non-empty payload (or segment)
  uint32_t* out;          // zero-length digests; null in update mode
  uint32_t* state;        // update mode: the registers (null in digest mode)
  // long payloads (launch_var_sorted): null split_slot = no splitting
  unsigned long long* split_ctr;       // this call's counter set (zero on entry)
  unsigned long long* split_ctr_next;  // the other set: zeroed by launch_bucket_place
  uint32_t* split_slot;                // n words: 1 when a long payload runs as segments, else 0
  uint32_t* split_state;               // update mode, n words: a split payload's register (SortedSplit::state)
  uint32_t split_cap;                  // extra descriptors this call may claim (<= kSplitSegCap)
  AutoChoice choice;  // both launches run only if the device chose the sorted path (ws null: always)
};
unsigned bucket_grid(size_t n);  // blocks of both launches (= the extent partials: at most kExtentMaxParts)

// The per-block extent partials (their count in *parts), and with `bk` step 1 of the counting sort.
hipError_t launch_extent(const uint64_t* off, const uint32_t* len, size_t n, void* ws, uint32_t* parts,
                         const BucketArgs* bk, hipStream_t stream);
// Step 2 of the counting sort; `record` (nullable) receives the extent reduced from ws's partials.
hipError_t launch_bucket_place(const uint64_t* off, const uint32_t* len, size_t n, const void* ws, uint32_t parts,
                               const BucketArgs& bk, ExtentHint* record, uint64_t seq, hipStream_t stream);

// Line-pass layout. L line-pass workgroups of 512 lanes = W = 8L waves = 64L lane groups;
// wave w's task t is full superblock fs0 + t*W + w (lane group g = 8w + block). Per line of a full
// superblock the block-suffix CRC S leaves in bursts of K = kSTasks tasks, K / 4 16-byte stores per lane
// that each cover 1 KiB contiguously: task t of group g, line a at word
//   ((((t / K) * W + g / 8) * (K / 4) + (t / 4) % (K / 4)) * 256 + ((g % 8) * 8 + a) * 4 + t % 4.
// SB (superblock suffix per block) of full superblock fs0 + i, block g at word i * 8 + g: a 128-byte line
// holds 4 superblocks of one task (W is a multiple of 4), so no line mixes two tasks' stores. The (at
// most two) partial superblocks keep S in S_edge[2][64] and SB in SB_edge[2][8].
#ifndef ANNETY_S_TASKS
#define ANNETY_S_TASKS 16
#endif
constexpr uint32_t kSTasks = ANNETY_S_TASKS;  // tasks per S burst (kSTasks / 4 stores of 1 KiB per wave)
inline __host__ __device__ uint64_t arena_s_word(uint64_t t, uint64_t group, uint32_t a, uint64_t W) {
  return ((((t / kSTasks) * W + (group >> 3)) * (kSTasks / 4) + ((t >> 2) % (kSTasks / 4))) << 8) +
         (((group & 7) * 8 + a) << 2) + (t & 3);
}

// Geometry of one arena call: the line pass on `blocks` workgroups, and the scratch layout
// [S | SB | S_edge 128 | SB_edge 16].
struct ArenaGeom {
  size_t blocks;         // line-pass workgroups L
  uint64_t W;            // line-pass waves = 8L
  uint64_t ntasks;       // tasks of the busiest wave
  uint64_t nbursts;      // ceil(ntasks / kSTasks)
  uint64_t sb_off, edge_off, words;
};
inline __host__ __device__ ArenaGeom arena_geom_of(uint64_t nsbf /* full superblocks */, size_t line_blocks) {
  ArenaGeom g{};
  g.blocks = line_blocks ? line_blocks : 1;
  g.W = 8 * (uint64_t)g.blocks;
  g.ntasks = (nsbf + g.W - 1) / g.W;
  g.nbursts = (g.ntasks + kSTasks - 1) / kSTasks;
  g.sb_off = g.nbursts * g.W * 64 * kSTasks;
  g.edge_off = g.sb_off + nsbf * 8;
  g.words = g.edge_off + 144;
  return g;
}
inline ArenaGeom arena_geom(const ArenaLaunch& a, size_t line_blocks) {  // line_blocks >= 1
  return arena_geom_of(a.fs1 - a.fs0, line_blocks);
}
// The lines and superblocks of the arena [byte_lo, byte_hi) (absolute addresses, byte_hi > byte_lo).
struct ArenaSpan {
  uint64_t byte_lo, byte_hi, line_lo, line_hi, sb0, nsb, fs0, fs1;
};
inline __host__ __device__ ArenaSpan arena_span(uint64_t byte_lo, uint64_t byte_hi) {
  ArenaSpan s;
  s.byte_lo = byte_lo;
  s.byte_hi = byte_hi;
  s.line_lo = byte_lo >> 7;
  s.line_hi = (byte_hi - 1) >> 7;
  s.sb0 = s.line_lo >> 6;
  s.nsb = (s.line_hi >> 6) - s.sb0 + 1;
  s.fs0 = (byte_lo + 8191) >> 13;  // superblocks wholly inside the arena
  s.fs1 = byte_hi >> 13;
  if (s.fs1 < s.fs0) s.fs1 = s.fs0;
  return s;
}
// The line pass on min(max_blocks, what the arena fills) workgroups.
inline ArenaGeom arena_geom(const ArenaLaunch& a) {
  const uint64_t nsbf = a.fs1 - a.fs0;
  uint64_t want = nsbf / 8 + 1;  // a wave per superblock per task, 8 waves per workgroup
  if (want > a.max_blocks) want = a.max_blocks;
  return arena_geom(a, (size_t)want);
}

hipError_t launch_arena(const ArenaLaunch& a, hipStream_t stream);
// the line pass alone (crc32_arena.hip, crc32_arena_lines.h)
hipError_t launch_arena_lines(const ArenaLaunch& a, hipStream_t stream);

// LengthHeaderCodec frames (crc32_frames.hip)
hipError_t launch_lhc_compare(const void* stream_base, const uint64_t* off, const uint32_t* len, size_t n,
                              const uint32_t* digest, uint8_t* ok, hipStream_t stream);
// One pass per frame: CRC, header, payload copy and trailer (crc32_frames.hip lhc_encode_fused_kernel). zero_line:
// 128 zero bytes (device); img_w8 = the sorted path's image part (kW8ImgBytes, crc32_math.h).
//
// Long frames (more than kEncLongMin payload bytes) do not run on one lane group (a 64 MiB frame would be 65k serial
// rounds): the group claims an entry and the frame's segment descriptors (kSplitSeg, the sorted path's segment
// format) from this call's counter, writes them and moves on; crc32_var_sorted_kernel then computes the claimed
// frames' digests, and lhc_encode_long_kernel copies them with the whole grid and writes their headers and trailers.
// Frames past the caps run on their groups as before. The counters live in the stream slot's extent scratch at
// kEncCtrOff, one 16-byte set per call parity: {unused, 0 (the sorted kernel's ranges[0]), uint64 {segments (its
// ranges[1]), frames}}; the long kernel zeroes the next call's set.
constexpr uint32_t kEncLongMin = 262144;
constexpr uint32_t kEncLongCap = 4096;         // frames per call
constexpr uint32_t kEncLongSegCap = 1u << 16;  // segment descriptors per call
constexpr size_t kEncCtrOff = 8192 - 64;       // after the extent partials, before the bucket cursors
static_assert((8 + 4 * kExtentMaxParts) * 8 <= kEncCtrOff && kEncCtrOff + 32 <= kCursorOff, "encode counters");
struct EncLong {
  unsigned long long* ctr;       // this call's {segments, frames}
  unsigned long long* ctr_next;  // the next call's (zeroed by lhc_encode_long_kernel)
  uint32_t* digest;              // [kEncLongCap] preset to ~0, the segments xor into it
  uint32_t* entry;               // [kEncLongCap] frame index
  void* desc;                    // [kEncLongSegCap] uint4 segment descriptors
  uint64_t* seg_dst;             // [kEncLongSegCap] each segment's destination address
};
constexpr size_t kEncLongScratchBytes = 8ull * kEncLongCap + 24ull * kEncLongSegCap;  // digest, entry, desc, seg_dst
hipError_t launch_lhc_encode_fused(const void* src, const uint64_t* src_off, const uint32_t* len, size_t n, int T,
                                   int64_t enc_min, int64_t enc_max, void* dst, const uint64_t* dst_off,
                                   const void* zero_line, const void* img_slice, const void* img_w8,
                                   const EncLong& lg, size_t max_blocks, hipStream_t stream);
// The claimed long frames: payload copy (16-byte stores over the whole grid, by segment), header and trailer.
hipError_t launch_lhc_encode_long(const uint32_t* len, int T, void* dst, const uint64_t* dst_off, const EncLong& lg,
                                  size_t max_blocks, hipStream_t stream);
int fixed_kernel_block();
// Records, for annety_crc_last_kernels, that the current entry point enqueued `name` (crc32_capi.cpp).
void note_kernel(const char* name);

}  // namespace annety_crc
