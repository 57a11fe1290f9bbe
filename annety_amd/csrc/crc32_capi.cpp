// C-ABI shim of the MI355X checksum engine: argument checks, per-device table images, launch
// selection, the host-memory staging pipeline, and the host scalar replacements of annety::Crc32c.
// Declared in include/annety_crc.h; every entry point is reentrant and returns a status, never aborts.
#include "annety_crc.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "crc32_host.h"
#include "crc32_kernels.h"
#include "crc32_math.h"

using namespace annety_crc;
using host::ConnWalk;
using host::FrameRules;
using host::FrameWalks;
using host::kPbcRules;
using host::lhc_rules;
using host::lhc_type_ok;
using host::parallel_pack;

namespace {

// ---------------- error and launch records (per calling thread) ----------------
thread_local int t_last_hip = 0;
// The stage a host path is in (verify_host_iov names its steps), and the stage of the last failing HIP call:
// annety_crc_last_error_stage. A failure of queued work surfaces at the next synchronising call, so with
// ANNETY_CRC_SYNC_STAGES=1 the host paths synchronise after every stage to name the one that failed.
thread_local const char* t_stage = "";
thread_local const char* t_fail_stage = "";
// The kernels the latest device entry point of this thread launched, in order (annety_crc_last_kernels).
thread_local std::string t_kernels;

void set_stage(const char* s) { t_stage = s; }

bool sync_stages() {
  static const bool on = [] {
    const char* e = std::getenv("ANNETY_CRC_SYNC_STAGES");
    return e && e[0] == '1';
  }();
  return on;
}

int hip_fail(hipError_t e) {
  t_last_hip = static_cast<int>(e);
  t_fail_stage = t_stage;
  return e == hipErrorOutOfMemory ? ANNETY_CRC_ENOMEM : ANNETY_CRC_EHIP;
}

#define HIP_TRY(expr)                          \
  do {                                         \
    hipError_t e_ = (expr);                    \
    if (e_ != hipSuccess) return hip_fail(e_); \
  } while (0)

// true if [p, p + bytes) lies inside one range this library pinned (annety_crc_host_register), so the DMA
// engines can read it in place. The runtime's pointer attributes are not asked: they classify a range by
// single bytes and cannot tell a stale or partly overlapping registration from a live one.
bool host_pinned(const void* p, size_t bytes) { return host::host_registry().covers(p, bytes); }

// ---------------- host-built LDS images ----------------
constexpr int kGroups[] = {1, 2, 4, 8, 16, 32};
constexpr int kNumGroups = 6;

int group_index(uint32_t g) {
  for (int i = 0; i < kNumGroups; i++)
    if ((uint32_t)kGroups[i] == g) return i;
  return -1;
}

struct HostImages {
  std::vector<uint32_t> slice;   // common part: slicing tables (32768 words) + half-line join (128 words)
  std::vector<uint32_t> groups;  // kNumGroups * (kGroupImageBytes / 4)
  std::vector<uint32_t> unshift; // 24 maps x 128 words (U_lo[0..15], U_hi[0..7])
  std::vector<uint32_t> sb;      // arena superblock join: (k, v, g) = shift_{(7-g)*1024}(v << 4k); byte map
  std::vector<uint32_t> stitch;  // arena stitch: segment maps F/G/UL/UB, unshift, shift_32 (crc32_math.h)
  std::vector<uint32_t> w8;      // sorted path (var_class_w8): join, byte maps, unshift (crc32_math.h kLdsW8*)
};

// Apply matrix m to (v << 4k) for every nibble value: the 16-entry table of one nibble position.
void nibble_tables(const Gf2Mat& m, uint32_t* out /* [8][16] */) {
  for (int kk = 0; kk < 8; kk++)
    for (uint32_t v = 0; v < 16; v++) out[kk * 16 + v] = gf2_apply(m, v << (4 * kk));
}

// A set of T maps stored [k][i][v] (crc32_device.h nibble_map_set) from maps stored [i][k][v].
void put_set(uint32_t* dst, const uint32_t* maps, uint32_t T) {
  for (uint32_t i = 0; i < T; i++)
    for (uint32_t kk = 0; kk < 8; kk++)
      for (uint32_t v = 0; v < 16; v++) dst[(kk * T + i) * 16 + v] = maps[i * 128 + kk * 16 + v];
}

// Byte masks of a 16-byte chunk (crc32_device.h mask_chunks): KEEP_FROM[a] = bytes [a, 16) for a = 0..16, then
// KEEP_TO[b] = bytes [0, b) for b = 0..16, 4 words each (544 bytes; dst zeroed).
void chunk_masks(uint32_t* mk) {
  for (uint32_t a = 0; a <= 16; a++)
    for (uint32_t byte = 0; byte < 16; byte++) {
      if (byte >= a) mk[a * 4 + byte / 4] |= 0xFFu << (8 * (byte % 4));
      if (byte < a) mk[(17 + a) * 4 + byte / 4] |= 0xFFu << (8 * (byte % 4));
    }
}

Gf2Mat gf2_inverse(const Gf2Mat& m) {
  // Gauss-Jordan over GF(2) on rows of the 32x32 matrix (row r = bit r of every column)
  uint64_t rows[32];
  for (int r = 0; r < 32; r++) {
    uint32_t row = 0;
    for (int c = 0; c < 32; c++) row |= ((m.col[c] >> r) & 1u) << c;
    rows[r] = (uint64_t)row | ((uint64_t)1 << (32 + r));  // [A | I]
  }
  for (int c = 0; c < 32; c++) {
    int piv = c;
    while (piv < 32 && !((rows[piv] >> c) & 1)) piv++;
    std::swap(rows[c], rows[piv]);
    for (int r = 0; r < 32; r++)
      if (r != c && ((rows[r] >> c) & 1)) rows[r] ^= rows[c];
  }
  Gf2Mat inv{};
  for (int c = 0; c < 32; c++) {
    uint32_t col = 0;
    for (int r = 0; r < 32; r++) col |= (uint32_t)((rows[r] >> (32 + c)) & 1u) << r;
    inv.col[c] = col;
  }
  return inv;
}

const HostImages& host_images() {
  static HostImages img;
  static std::once_flag once;
  std::call_once(once, [] {
    img.slice.assign(kLdsCommonBytes / 4, 0);
    uint32_t t[4][256];
    for (int kk = 0; kk < 4; kk++)
      for (uint32_t e = 0; e < 256; e++) t[kk][e] = slice_entry(kk, e);
    for (int P = 0; P < 2; P++)
      for (uint32_t e = 0; e < 256; e++)
        for (uint32_t r = 0; r < 32; r++) {
          const uint32_t w = (P * 65536 + e * 256 + r * 8) / 4;
          img.slice[w] = t[3 - 2 * P][e];      // P0: T3, P1: T1
          img.slice[w + 1] = t[2 - 2 * P][e];  // P0: T2, P1: T0
        }
    nibble_tables(shift_matrix(64), img.slice.data() + kLdsHalfOff / 4);  // half-line join
    const uint32_t gw = kGroupImageBytes / 4;
    img.groups.assign((size_t)kNumGroups * gw, 0);
    for (int gi = 0; gi < kNumGroups; gi++) {
      const uint32_t G = kGroups[gi];
      uint32_t* g = img.groups.data() + (size_t)gi * gw;
      uint32_t nt[8 * 16];
      for (uint32_t jj = 0; jj < G; jj++) {
        nibble_tables(shift_matrix((uint64_t)(G - 1 - jj) * kChunkBytes), nt);
        for (uint32_t slot = 0; slot < 32; slot++) {
          if ((slot & (G - 1)) != jj) continue;
          for (int kk = 0; kk < 8; kk++)
            for (int v = 0; v < 16; v++) g[(kk * 2048 + v * 128 + slot * 4) / 4] = nt[kk * 16 + v];
        }
      }
      nibble_tables(shift_matrix((uint64_t)(G - 1) * kChunkBytes), nt);
      std::memcpy(g + kLdsJoinBytes / 4, nt, sizeof nt);
    }
    img.unshift.assign(24 * 128, 0);
    const Gf2Mat inv1 = gf2_inverse(shift_matrix(1));
    Gf2Mat acc{};
    for (int i = 0; i < 32; i++) acc.col[i] = 1u << i;
    Gf2Mat inv16{};
    for (int m = 0; m < 16; m++) {  // U_lo[m] = shift_{-m}
      nibble_tables(acc, img.unshift.data() + m * 128);
      acc = gf2_mul(inv1, acc);
    }
    inv16 = acc;  // shift_{-16}
    for (int i = 0; i < 32; i++) acc.col[i] = 1u << i;
    for (int h = 0; h < 8; h++) {  // U_hi[h] = shift_{-16h}
      nibble_tables(acc, img.unshift.data() + (16 + h) * 128);
      acc = gf2_mul(inv16, acc);
    }
    img.sb.assign((kLdsSbJoinBytes + 2 * kLdsByteMapBytes) / 4, 0);
    {  // then byte tables B_k[e] = shift(e << 8k) (crc32_device.h byte_map64): the half-line join shift_64,
       // and the G = 32 round advance shift_{31*128} (crc32_fixed32_nt_kernel)
      const uint64_t shifts[2] = {64, 31 * kChunkBytes};
      for (int m_i = 0; m_i < 2; m_i++) {
        const Gf2Mat m = shift_matrix(shifts[m_i]);
        uint32_t* bm = img.sb.data() + (kLdsSbJoinBytes + m_i * kLdsByteMapBytes) / 4;
        for (uint32_t kk = 0; kk < 4; kk++)
          for (uint32_t e = 0; e < 256; e++) bm[kk * 256 + e] = gf2_apply(m, e << (8 * kk));
      }
    }
    for (uint32_t g = 0; g < 8; g++) {
      uint32_t nt[8 * 16];
      nibble_tables(shift_matrix((uint64_t)(7 - g) * 1024), nt);
      for (int kk = 0; kk < 8; kk++)
        for (int v = 0; v < 16; v++) img.sb[kk * 128 + v * 8 + g] = nt[kk * 16 + v];
    }
    img.stitch.assign((kLdsStitchImageBytes - kLdsCommonBytes) / 4, 0);
    {
      std::vector<uint32_t> seg(32 * 128);
      const Gf2Mat inv128 = gf2_inverse(shift_matrix(128)), inv1024 = gf2_inverse(shift_matrix(1024));
      Gf2Mat ul{}, ub{};
      for (int i = 0; i < 32; i++) ul.col[i] = ub.col[i] = 1u << i;
      for (uint32_t q = 0; q < 8; q++) {
        nibble_tables(shift_matrix((uint64_t)128 * (q + 1)), seg.data() + (kMapF + q) * 128);   // F(q+1)
        nibble_tables(shift_matrix((uint64_t)1024 * (q + 1)), seg.data() + (kMapG + q) * 128);  // G(q+1)
        nibble_tables(ul, seg.data() + (kMapUL + q) * 128);                                      // UL(q)
        nibble_tables(ub, seg.data() + (kMapUB + q) * 128);                                      // UB(q)
        ul = gf2_mul(inv128, ul);
        ub = gf2_mul(inv1024, ub);
      }
      uint32_t* m = img.stitch.data();
      put_set(m, seg.data(), 32);
      put_set(m + (kLdsStitchUnshiftOff - kLdsMapOff) / 4, img.unshift.data(), 16);                  // U_lo
      put_set(m + (kLdsStitchUnshiftOff + 8192 - kLdsMapOff) / 4, img.unshift.data() + 16 * 128, 8);  // U_hi
      nibble_tables(shift_matrix(32), m + (kLdsQuarterOff - kLdsMapOff) / 4);
      chunk_masks(m + (kLdsStitchMaskOff - kLdsMapOff) / 4);
    }
    img.w8.assign(kW8ImgAllBytes / 4, 0);
    {
      uint32_t* m = img.w8.data();
      for (uint32_t jj = 0; jj < 8; jj++) {  // (k, v, j) at (k*16 + v)*8 + j words
        uint32_t nt[8 * 16];
        nibble_tables(shift_matrix((uint64_t)(7 - jj) * kChunkBytes), nt);
        for (int kk = 0; kk < 8; kk++)
          for (int v = 0; v < 16; v++) m[(kk * 16 + v) * 8 + jj] = nt[kk * 16 + v];
      }
      // byte tables: half-line join, round advance (8-lane groups), round advance of 4-lane groups (the encode)
      const uint64_t shifts[3] = {64, 7 * kChunkBytes, 3 * kChunkBytes};
      const uint32_t offs[3] = {kLdsW8HalfOff, kLdsW8RoundOff, kLdsW8Round4Off};
      for (int m_i = 0; m_i < 3; m_i++) {
        const Gf2Mat sm = shift_matrix(shifts[m_i]);
        uint32_t* bm = m + (offs[m_i] - kLdsCommonBytes) / 4;
        for (uint32_t kk = 0; kk < 4; kk++)
          for (uint32_t e = 0; e < 256; e++) bm[kk * 256 + e] = gf2_apply(sm, e << (8 * kk));
      }
      std::memcpy(m + (kLdsW8UnshiftOff - kLdsCommonBytes) / 4, img.unshift.data(), img.unshift.size() * 4);
      for (uint32_t lead = 0; lead < 128; lead++)
        m[(kLdsW8InitOff - kLdsCommonBytes) / 4 + lead] = gf2_apply(shift_matrix(128 - lead), kInit);
      chunk_masks(m + (kLdsW8MaskOff - kLdsCommonBytes) / 4);
    }
  });
  return img;
}

// ---------------- per-device state ----------------
struct Staging {
  void* h_pinned[2] = {nullptr, nullptr};  // pinned host ring
  void* d_buf[2] = {nullptr, nullptr};
  uint32_t* d_out[2] = {nullptr, nullptr};
  uint32_t* h_out[2] = {nullptr, nullptr};
  hipStream_t stream[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  size_t bytes = 0, outs = 0;
  // frame path (annety_lhc_verify_host): the received stream and its per-frame metadata on the device
  char* d_stream = nullptr;
  size_t stream_cap = 0;
  char* d_meta = nullptr;  // off (8 B) + len (4 B) + digest (4 B) + ok (1 B) per frame
  size_t meta_cap = 0;     // frames
  // pinned bounce buffer of that metadata: off + len up, ok down. The runtime's copies from and to the
  // caller's pageable arrays cost time that grows with the size of the ARRAYS, not of the copy (frame
  // verify of config 3 through 110 MB output arrays: 28.6 against 49 GiB/s)
  char* h_meta = nullptr;
  size_t h_meta_cap = 0;   // frames
};

// The scratch a stream's slot carries (crc32_host.h Slot<Scratch>::data).
struct Scratch {
  void* ptr = nullptr;
  size_t bytes = 0;
  // automatic variable-path choice (run_var_auto): the extent kernels' area is the slot's first
  // kExtentScratchBytes; the paths' scratch follows
  ExtentHint* hint = nullptr;  // pinned: the extent of this slot's latest completed auto call
  uint64_t calls = 0;          // extent kernels launched from this slot (hint->seq numbers them)
  // the sorted path's bucket cursors (crc32_kernels.h BucketArgs): set (sorts & 1) is this call's
  uint64_t sorts = 0;
  bool cursors_clean = false;  // both sets zero (false after an allocation or a failed sort)
  // the fused encode's long-frame counters (crc32_kernels.h EncLong): set (encodes & 1) is this call's
  uint64_t encodes = 0;
  bool enc_clean = false;  // both sets zero (false after an allocation or a failed encode)
  struct Key {
    const void *base, *off, *len;
    size_t n;
    bool update;
    bool operator==(const Key& o) const {
      return base == o.base && off == o.off && len == o.len && n == o.n && update == o.update;
    }
  } key{};
  uint64_t arena_want = 0;                // scratch bytes the densest span recorded in this slot needs (any key)
  uint64_t key_since = 0;                 // first call (seq) with the current key
  uint64_t since_extent = 0;              // arena calls since the last one that recorded its extent
  uint64_t seen_seq = 0, prev_seq = 0;    // the two latest completed hints read for this key
  ExtentHint seen{}, prev{};
};
using ScratchSlot = host::Slot<Scratch>;

// Up to ANNETY_CRC_STREAM_SLOTS (default 64) slots per device, read once.
size_t stream_slot_cap() {
  static const size_t cap = [] {
    const char* e = std::getenv("ANNETY_CRC_STREAM_SLOTS");
    const long v = e && *e ? std::atol(e) : 64;
    return (size_t)std::max(1L, std::min(4096L, v));
  }();
  return cap;
}

// The runtime operations the slot table needs, on the current device.
struct HipSlotOps {
  int make_fence(void** ev) {
    hipEvent_t e = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    *ev = e;
    return ANNETY_CRC_OK;
  }
  void destroy_fence(void* ev) {
    if (ev) (void)hipEventDestroy(static_cast<hipEvent_t>(ev));
  }
  int record(void* ev, const void* stream) {
    HIP_TRY(hipEventRecord(static_cast<hipEvent_t>(ev), static_cast<hipStream_t>(const_cast<void*>(stream))));
    return ANNETY_CRC_OK;
  }
  int wait(const void* stream, void* ev) {
    HIP_TRY(hipStreamWaitEvent(static_cast<hipStream_t>(const_cast<void*>(stream)), static_cast<hipEvent_t>(ev), 0));
    return ANNETY_CRC_OK;
  }
  int drain() {
    HIP_TRY(hipDeviceSynchronize());
    return ANNETY_CRC_OK;
  }
};

struct DeviceCtx {
  std::atomic<bool> ready{false};
  int cus = 0;
  void* d_slice = nullptr;
  void* d_groups = nullptr;
  uint32_t* d_unshift = nullptr;
  void* d_sb = nullptr;
  void* d_stitch = nullptr;
  void* d_w8 = nullptr;
  void* d_zero = nullptr;  // 256 zero bytes
  Staging stg;
  std::mutex stg_mu;  // one host-staged batch at a time per device
  std::mutex pow_mu;  // split-path power tables, one per segment size
  std::vector<std::pair<uint64_t, uint32_t*>> powers;
  // per-call scratch of the arena, split and sorted paths, reused across calls: one slot per stream
  // (crc32_host.h SlotTable: stream order while the table has room, fences or one drain past it)
  std::mutex arena_mu;  // held while a call picks a slot and enqueues its launches
  host::SlotTable<Scratch> slots{stream_slot_cap()};
  // test-visible counters (annety_crc_scratch_stats): drains at shutdown (the table counts its own)
  std::atomic<uint64_t> shutdown_syncs{0};
  std::atomic<uint64_t> auto_arena{0}, auto_sorted{0};  // run_var_auto's choices
  std::atomic<uint64_t> auto_unchecked{0};              // arena calls without the extent kernel
  std::atomic<uint64_t> auto_device{0};                 // calls whose path the device chose (AutoChoice)
};

constexpr int kMaxDev = 64;
DeviceCtx g_dev[kMaxDev];
// CUs left free by the batch kernels (annety_crc_reserve_cus): room for work on other streams, e.g. the
// RCCL kernels of a digest gather that runs beside the next chunk's checksums
std::atomic<int> g_reserved_cus{0};
size_t grid_cus(const DeviceCtx& c) { return (size_t)std::max(1, c.cus - g_reserved_cus.load()); }
std::mutex g_init_mu;

void free_images(DeviceCtx& c) {
  void* bufs[] = {c.d_slice, c.d_groups, c.d_unshift, c.d_sb, c.d_stitch, c.d_w8, c.d_zero};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  c.d_slice = c.d_groups = nullptr;
  c.d_unshift = nullptr;
  c.d_sb = c.d_stitch = c.d_w8 = c.d_zero = nullptr;
}

int init_device_locked(int dev) {
  DeviceCtx& c = g_dev[dev];
  if (c.ready) return ANNETY_CRC_OK;
  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (dev < 0 || dev >= ndev) return ANNETY_CRC_ENODEV;
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, dev));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return ANNETY_CRC_ENODEV;  // built for gfx950 only
  int prev = 0;
  HIP_TRY(hipGetDevice(&prev));
  HIP_TRY(hipSetDevice(dev));
  const HostImages& img = host_images();
  int rc = ANNETY_CRC_OK;
  do {
    hipError_t e;
    if ((e = hipMalloc(&c.d_slice, img.slice.size() * 4)) != hipSuccess) { rc = hip_fail(e); break; }
    if ((e = hipMalloc(&c.d_groups, img.groups.size() * 4)) != hipSuccess) { rc = hip_fail(e); break; }
    if ((e = hipMalloc(&c.d_unshift, img.unshift.size() * 4)) != hipSuccess) { rc = hip_fail(e); break; }
    if ((e = hipMalloc(&c.d_sb, img.sb.size() * 4)) != hipSuccess) { rc = hip_fail(e); break; }
    if ((e = hipMalloc(&c.d_stitch, img.stitch.size() * 4)) != hipSuccess) { rc = hip_fail(e); break; }
    if ((e = hipMalloc(&c.d_w8, img.w8.size() * 4)) != hipSuccess) { rc = hip_fail(e); break; }
    if ((e = hipMemcpy(c.d_w8, img.w8.data(), img.w8.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) { rc = hip_fail(e); break; }
    if ((e = hipMalloc(&c.d_zero, 256)) != hipSuccess) { rc = hip_fail(e); break; }
    if ((e = hipMemset(c.d_zero, 0, 256)) != hipSuccess) { rc = hip_fail(e); break; }
    if ((e = hipMemcpy(c.d_sb, img.sb.data(), img.sb.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) { rc = hip_fail(e); break; }
    if ((e = hipMemcpy(c.d_stitch, img.stitch.data(), img.stitch.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) { rc = hip_fail(e); break; }
    if ((e = hipMemcpy(c.d_slice, img.slice.data(), img.slice.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) { rc = hip_fail(e); break; }
    if ((e = hipMemcpy(c.d_groups, img.groups.data(), img.groups.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) { rc = hip_fail(e); break; }
    if ((e = hipMemcpy(c.d_unshift, img.unshift.data(), img.unshift.size() * 4, hipMemcpyHostToDevice)) != hipSuccess) { rc = hip_fail(e); break; }
    c.cus = prop.multiProcessorCount;
    c.ready = true;
  } while (0);
  if (rc != ANNETY_CRC_OK) free_images(c);  // nothing half-built survives a failed init
  (void)hipSetDevice(prev);
  return rc;
}

DeviceCtx* ensure_ctx(int dev, int* rc) {
  if (dev < 0 || dev >= kMaxDev) {
    *rc = ANNETY_CRC_ENODEV;
    return nullptr;
  }
  DeviceCtx& c = g_dev[dev];
  if (!c.ready) {
    std::lock_guard<std::mutex> lk(g_init_mu);
    *rc = init_device_locked(dev);
    if (*rc != ANNETY_CRC_OK) return nullptr;
  }
  *rc = ANNETY_CRC_OK;
  return &c;
}

// The context of the device a call runs on: the current device, which must also own `stream`. A stream
// of another device is refused (ANNETY_CRC_EINVAL) rather than given this device's tables and scratch:
// a process driving several GPUs from one thread must hipSetDevice to the stream's device first. The NULL
// stream and the per-thread / legacy handles belong to the current device by definition.
bool special_stream(hipStream_t s) { return s == nullptr || s == hipStreamPerThread || s == hipStreamLegacy; }

int stream_ctx(hipStream_t stream, DeviceCtx** out) {
  t_kernels.clear();  // a device entry point starts: its launches are recorded from here
  set_stage("launch");
  int dev = 0;
  HIP_TRY(hipGetDevice(&dev));
  if (!special_stream(stream)) {
    hipDevice_t sdev = -1;
    const hipError_t e = hipStreamGetDevice(stream, &sdev);
    if (e != hipSuccess) {
      t_last_hip = static_cast<int>(e);
      (void)hipGetLastError();
      return ANNETY_CRC_EINVAL;  // not a stream handle
    }
    if (sdev != dev) return ANNETY_CRC_EINVAL;
  }
  int rc = 0;
  DeviceCtx* c = ensure_ctx(dev, &rc);
  if (!c) return rc;
  *out = c;
  return ANNETY_CRC_OK;
}

// The current device's context (microbench harnesses, which include this file).
[[maybe_unused]] int current_ctx(DeviceCtx** out) { return stream_ctx(nullptr, out); }

const void* group_image(const DeviceCtx& c, uint32_t g) {
  return static_cast<const char*>(c.d_groups) + (size_t)group_index(g) * kGroupImageBytes;
}

uint32_t pick_group(uint64_t lines, size_t n, int cus) {
  // Largest power of two <= lines, capped at 32 lanes; one more doubling (fewer rounds, same number of
  // virtual lines) when the batch is too small to fill the chip.
  uint32_t g = 1;
  while (g < 32 && (uint64_t)g * 2 <= lines) g *= 2;
  const size_t lanes_chip = (size_t)cus * fixed_kernel_block();
  if (g < 32 && (uint64_t)g < lines && n * (size_t)g * 2 <= lanes_chip) g *= 2;
  return g;
}

int run_fixed(DeviceCtx& c, const void* d_base, size_t n, size_t len, size_t stride, uint32_t* d_out, bool raw,
              hipStream_t stream) {
  FixedLaunch a{};
  a.base = d_base;
  a.n = n;
  a.stride = stride;
  a.len_blocks = (uint32_t)(len / 16);
  const uint64_t lines = (len + kChunkBytes - 1) / kChunkBytes;
  a.group = pick_group(lines, n, c.cus);
  a.rounds = (uint32_t)((lines + a.group - 1) / a.group);
  a.vlead = a.rounds * a.group * 8 - a.len_blocks;
  a.full = a.vlead == 0;
  a.raw = raw;
  a.img_slice = c.d_slice;
  a.img_group = group_image(c, a.group);
  a.img_bytemap = static_cast<const char*>(c.d_sb) + kLdsSbJoinBytes;
  if (raw) {
    const Gf2Mat m = shift_matrix(len);
    std::memcpy(a.raw_shift_cols.c, m.col, sizeof m.col);
  }
  a.out = d_out;
  a.max_blocks = grid_cus(c);
  HIP_TRY(launch_fixed(a, stream));
  return ANNETY_CRC_OK;
}

int run_var(DeviceCtx& c, const void* d_base, size_t n, uint64_t fstride, uint32_t flen, uint32_t group,
            const void* desc, const uint32_t* range, uint32_t* d_out, hipStream_t stream, bool update = false) {
  VarLaunch a{};
  a.update = update;
  a.base = d_base;
  a.n = n;
  a.fixed_stride = fstride;
  a.fixed_len = flen;
  a.desc = desc;
  a.range = range;
  a.group = group;
  a.img_slice = c.d_slice;
  a.img_group = group_image(c, group);
  a.img_unshift = c.d_unshift;
  a.out = d_out;
  a.max_blocks = grid_cus(c);
  HIP_TRY(launch_var(a, stream));
  return ANNETY_CRC_OK;
}

// Per-call device scratch of the arena, split and sorted paths: the stream's slot (crc32_host.h SlotTable),
// grown in stream order with the stream-ordered allocator (one allocation per growth; per call it would cost
// ~3.6 us). The caller holds c.arena_mu from here until its launches are enqueued, then calls scratch_done.
int scratch_slot(DeviceCtx& c, hipStream_t stream, size_t bytes, ScratchSlot** out) {
  HipSlotOps ops;
  ScratchSlot* slot = nullptr;
  const int rc = c.slots.acquire(ops, stream, stream == hipStreamPerThread, &slot);
  if (rc) return rc;
  Scratch& d = slot->data;
  if (d.bytes < bytes) {
    if (d.ptr) HIP_TRY(hipFreeAsync(d.ptr, stream));
    d.ptr = nullptr;
    d.bytes = 0;
    HIP_TRY(hipMallocAsync(&d.ptr, kExtentScratchBytes + bytes, stream));
    d.bytes = bytes;
    d.cursors_clean = false;
    d.enc_clean = false;
  }
  *out = slot;
  return ANNETY_CRC_OK;
}

// The paths' scratch inside a slot (after the extent kernel's area).
char* path_scratch(const ScratchSlot* slot) { return static_cast<char*>(slot->data.ptr) + kExtentScratchBytes; }

// After the call's launches (arena_mu still held): the table fences the call when a later hand-over could
// need it (crc32_host.h SlotTable::done).
int scratch_done(DeviceCtx& c, ScratchSlot* slot) {
  HipSlotOps ops;
  return c.slots.done(ops, slot);
}

// Variable batch: counting sort by rounds (ceil(lines / 8)) on the device (no host round trip; two launches,
// crc32_kernels.h BucketArgs), then one launch per length class with its own lane-group width. Scratch:
// the stream's slot (scratch_slot): the bucket cursors in the extent area, rows + ranges + descriptors
// after it.
// Layout after rows + ranges: descriptors (n, plus split_cap(n) for long payloads' extra segments), then
// split_slot and split_state (n words each; crc32_kernels.h kSplitSeg).
// Extra segment descriptors per call (annety_crc_set_split_cap; default and maximum kSplitSegCap).
std::atomic<uint32_t> g_split_cap{kSplitSegCap};
// A batch of n payloads never needs more than n * (kSplitMaxSegs - 1) (small batches reserved 4 MiB).
uint32_t split_cap(size_t n) {
  return (uint32_t)std::min<uint64_t>(g_split_cap.load(std::memory_order_relaxed), (uint64_t)n * (kSplitMaxSegs - 1));
}
size_t sorted_desc_count(size_t n, uint32_t cap) { return n + cap; }
size_t sorted_scratch_bytes(size_t n, uint32_t cap) {
  const size_t rows_words = (size_t)bucket_grid(n) * kBucketCount;
  return (rows_words + kRangeWords) * sizeof(uint32_t) + 16 * sorted_desc_count(n, cap) + 8 * n;
}
size_t sorted_scratch_bytes(size_t n) { return sorted_scratch_bytes(n, split_cap(n)); }
int split_powers(DeviceCtx& c, uint64_t seg, const uint32_t** out);

// The length classes in one launch (the product) or one launch each (A/B builds: ANNETY_CRC_SORTED_FUSED=0).
bool sorted_fused() {
  static const bool on = ANNETY_AB_KNOB("ANNETY_CRC_SORTED_FUSED", 1) != 0;
  return on;
}

// The sorted path's launches into `slot` (sized by sorted_scratch_bytes; c.arena_mu held). `record`
// (automatic path): the extent record the bucket pass publishes, numbered `seq`.
int run_var_sorted_in(DeviceCtx& c, ScratchSlot* slot, const void* d_base, size_t n, const uint64_t* d_off,
                      const uint32_t* d_len, uint32_t* d_out, hipStream_t stream, bool update,
                      ExtentHint* record = nullptr, uint64_t seq = 0, const AutoChoice* choice = nullptr) {
  // descriptor indices keep bit 31 for segments (and payloads past kSegIndexMask run whole)
  if (n > kSortedMaxPayloads) return ANNETY_CRC_EINVAL;
  // extra segment descriptors: the cap, within what the slot holds (a setter racing with the sizing cannot overflow it)
  const size_t fixed = ((size_t)bucket_grid(n) * kBucketCount + kRangeWords) * sizeof(uint32_t) + 24 * n;
  const uint64_t room = slot->data.bytes > fixed ? (slot->data.bytes - fixed) / 16 : 0;
  const uint32_t cap = (uint32_t)std::min<uint64_t>(split_cap(n), room);
  uint32_t* cursors = reinterpret_cast<uint32_t*>(static_cast<char*>(slot->data.ptr) + kCursorOff);
  if (!slot->data.cursors_clean) {  // both cursor sets and both split counter sets (contiguous)
    const hipError_t z = hipMemsetAsync(cursors, 0, 2 * kBucketCount * sizeof(uint32_t) + 64, stream);
    if (z != hipSuccess) return hip_fail(z);
    slot->data.cursors_clean = true;
  }
  SortedSplit split{};  // the long payloads' power tables (built once per device)
  if (sorted_fused()) {
    int pr = split_powers(c, kSplitSeg, &split.powers);
    if (pr == ANNETY_CRC_OK) pr = split_powers(c, kSplitSegBig, &split.powers_big);
    if (pr) return pr;
  }
  const size_t rows_words = (size_t)bucket_grid(n) * kBucketCount;
  char* scratch = path_scratch(slot);
  BucketArgs bk{};
  bk.base = d_base;
  bk.rows = reinterpret_cast<uint32_t*>(scratch);
  bk.ranges = bk.rows + rows_words;
  bk.desc = scratch + (rows_words + kRangeWords) * sizeof(uint32_t);
  const uint32_t set = (uint32_t)(slot->data.sorts & 1);
  bk.cursor = cursors + set * kBucketCount;
  bk.cursor_next = cursors + (set ^ 1) * kBucketCount;
  bk.out = update ? nullptr : d_out;
  bk.state = update ? d_out : nullptr;
  if (choice) bk.choice = *choice;
  unsigned long long* sctr =
      reinterpret_cast<unsigned long long*>(static_cast<char*>(slot->data.ptr) + kSplitCtrOff);
  if (sorted_fused()) {  // (the A/B per-class launches take no segments)
    bk.split_ctr = sctr + 4 * set;
    bk.split_ctr_next = sctr + 4 * (set ^ 1);
    bk.split_slot = reinterpret_cast<uint32_t*>(static_cast<char*>(bk.desc) + 16 * sorted_desc_count(n, cap));
    bk.split_state = bk.split_slot + n;
    bk.split_cap = cap;
    split.state = bk.split_state;
  }
  uint32_t parts = 0;
  hipError_t e = launch_extent(d_off, d_len, n, slot->data.ptr, &parts, &bk, stream);
  if (e == hipSuccess) e = launch_bucket_place(d_off, d_len, n, slot->data.ptr, parts, bk, record, seq, stream);
  if (e != hipSuccess) {
    slot->data.cursors_clean = false;  // the next sort zeroes both sets first
    return hip_fail(e);
  }
  slot->data.sorts++;
  int rc = ANNETY_CRC_OK;
  if (sorted_fused()) {  // the length classes in one launch (crc32_var_sorted_kernel)
    VarLaunch a{};
    a.update = update;
    a.base = d_base;
    a.n = n;
    a.desc = bk.desc;
    a.range = bk.ranges;
    a.img_slice = c.d_slice;
    a.img_unshift = c.d_unshift;
    a.out = d_out;
    a.max_blocks = grid_cus(c);
    if (choice) a.choice = *choice;
    const hipError_t e = launch_var_sorted(a, c.d_w8, split, stream);
    return e == hipSuccess ? ANNETY_CRC_OK : hip_fail(e);
  }
  // (A/B builds) the per-task var kernel over the sorted list, 32 lanes per payload (no device choice)
  if (choice) return ANNETY_CRC_EINVAL;
  rc = run_var(c, d_base, n, 0, 0, 32, bk.desc, bk.ranges, d_out, stream, update);
  return rc;
}

int run_var_sorted(DeviceCtx& c, const void* d_base, size_t n, const uint64_t* d_off, const uint32_t* d_len,
                   uint32_t* d_out, hipStream_t stream, bool update = false) {
  std::lock_guard<std::mutex> lk(c.arena_mu);
  ScratchSlot* slot = nullptr;
  int rc = scratch_slot(c, stream, sorted_scratch_bytes(n), &slot);
  if (rc) return rc;
  rc = run_var_sorted_in(c, slot, d_base, n, d_off, d_len, d_out, stream, update);
  const int rd = scratch_done(c, slot);
  return rc ? rc : rd;
}

// Arena path (crc32_arena.hip): one bulk pass over every line of [d_base, d_base + arena_bytes),
// then one lane per payload. Scratch (S quads, S_edge, SB: ~33 words per 1 KiB block, ~3.3 % of the
// arena) comes from the stream-ordered allocator.
// Arena geometry and images for [d_base, d_base + arena_bytes) (everything but the batch and scratch).
void arena_fill_range(const DeviceCtx& c, const void* d_base, uint64_t byte_lo, uint64_t byte_hi, ArenaLaunch& a) {
  a.base = d_base;
  a.img_slice = c.d_slice;
  a.img_group8 = group_image(c, 8);
  a.img_sb = c.d_sb;
  a.img_stitch = c.d_stitch;
  a.zero_line = c.d_zero;
  a.max_blocks = grid_cus(c);
  if (byte_hi <= byte_lo) return;
  const ArenaSpan sp = arena_span(byte_lo, byte_hi);
  a.byte_lo = sp.byte_lo;
  a.byte_hi = sp.byte_hi;
  a.line_lo = sp.line_lo;
  a.line_hi = sp.line_hi;
  a.sb0 = sp.sb0;
  a.nsb = sp.nsb;
  a.fs0 = sp.fs0;
  a.fs1 = sp.fs1;
}

void arena_fill(const DeviceCtx& c, const void* d_base, size_t arena_bytes, ArenaLaunch& a) {
  const uint64_t lo = (uint64_t)(uintptr_t)d_base;
  arena_fill_range(c, d_base, lo, lo + arena_bytes, a);
}

// d_ok: LengthHeaderCodec verify - the stitch compares every digest with the trailer after its payload and writes
// the verdicts (d_out may then be null: no digests)
// The stitch's power table for long runs of whole superblocks (ArenaLaunch::pow8k), built once per device.
int arena_powers(DeviceCtx& c, ArenaLaunch& a) {
  const uint32_t* p = nullptr;
  const int rc = split_powers(c, 8192, &p);
  a.pow8k = p;
  return rc;
}

int run_arena(DeviceCtx& c, const void* d_base, size_t arena_bytes, const uint64_t* d_off, const uint32_t* d_len,
              size_t n, uint32_t* d_out, hipStream_t stream, bool update, uint8_t* d_ok = nullptr) {
  ArenaLaunch a{};
  arena_fill(c, d_base, arena_bytes, a);
  if (const int pr = arena_powers(c, a)) return pr;
  a.off = d_off;
  a.len = d_len;
  a.n = n;
  a.out = d_out;
  a.ok = d_ok;
  a.update = update;
  if (n == 0) return ANNETY_CRC_OK;
  if (!a.nsb) {
    const hipError_t e = launch_arena(a, stream);
    return e == hipSuccess ? ANNETY_CRC_OK : hip_fail(e);
  }
  const size_t bytes = arena_geom(a).words * sizeof(uint32_t);
  if (bytes / sizeof(uint32_t) >= (1ull << 32)) return ANNETY_CRC_EINVAL;  // the stitch's 32-bit word indices
  std::lock_guard<std::mutex> lk(c.arena_mu);
  ScratchSlot* slot = nullptr;
  const int rc = scratch_slot(c, stream, bytes, &slot);
  if (rc) return rc;
  a.scratch = reinterpret_cast<uint32_t*>(path_scratch(slot));
  const hipError_t e = launch_arena(a, stream);
  const int rd = scratch_done(c, slot);
  if (e != hipSuccess) return hip_fail(e);
  return rd;
}

// ---- automatic choice between the arena and the sorted path (annety_crc32_batch_var) ----
// The arena path needs its extent on the host (grid, scratch) but the offsets are device data; reading them
// back would make every call synchronous. Instead every call launches the extent kernel (crc32_kernels.h
// launch_extent, ~5 us), which leaves the batch's extent in a pinned record per stream slot, and a call
// takes the arena path over [lo, hi) when the two latest completed records for the same (base, offsets,
// lengths, n) agree, are dense (payload bytes >= 2/3 of the span) and safe (sorted starts with gaps < 4 KiB, or
// in any order when the span lies inside one device allocation).
// The kernels then check this call's own extent against [lo, hi) on the device and, if it differs, read
// nothing outside the payloads (each is folded directly) - a stale record costs time, never correctness
// or a read of unmapped memory. Otherwise the sorted path runs. (Mode 0 of run_var_any.)
constexpr size_t kAutoMinPayloads = 1024;  // below this the extent kernel is not worth its launch
// Arena calls between two that record their extent. In between, the arena launches skip the extent kernel
// and the device check: the declared range is checked on the host to lie inside one device allocation
// (range_mapped), so the line pass reads only mapped memory, and the stitch folds any payload outside the
// range directly from its own bytes - the digests never depend on the record, which only steers the path.
constexpr uint64_t kAutoRefresh = 8;

// [lo, hi) lies inside one device allocation (hipMemGetAddressRange), so all of it is mapped.
bool range_mapped(uint64_t lo, uint64_t hi) {
  hipDeviceptr_t b = nullptr;
  size_t sz = 0;
  if (hipMemGetAddressRange(&b, &sz, reinterpret_cast<hipDeviceptr_t>(lo)) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  const uint64_t bb = (uint64_t)(uintptr_t)b;
  return lo >= bb && hi <= bb + sz && hi > lo;
}

// Reads the slot's pinned record; true if a new completed one for the current key arrived.
bool poll_hint(ScratchSlot* slot) {
  Scratch* s = &slot->data;
  ExtentHint h{};
  h.lo = __atomic_load_n(&s->hint->lo, __ATOMIC_RELAXED);
  h.hi = __atomic_load_n(&s->hint->hi, __ATOMIC_RELAXED);
  h.sum = __atomic_load_n(&s->hint->sum, __ATOMIC_RELAXED);
  h.bad = __atomic_load_n(&s->hint->bad, __ATOMIC_RELAXED);
  h.seq = __atomic_load_n(&s->hint->seq, __ATOMIC_RELAXED);
  h.chk = __atomic_load_n(&s->hint->chk, __ATOMIC_RELAXED);
  if ((h.lo ^ h.hi ^ h.sum ^ h.bad ^ h.seq ^ kExtentCheck) != h.chk) return false;  // torn: the next call reads it
  const uint64_t seq = h.seq;
  if (seq <= s->seen_seq || seq < s->key_since) return false;
  if (s->seen_seq >= s->key_since) {
    s->prev = s->seen;
    s->prev_seq = s->seen_seq;
  }
  s->seen = h;
  s->seen_seq = seq;
  return true;
}

// Whether a completed record allows the arena path: a dense span (payload bytes >= 2/3 of it, under 32 GiB) that is
// safe to read - sorted starts with gaps < 4 KiB, or (host check) inside one device allocation.
bool record_allows_arena(const ExtentHint& h, uint64_t b) {
  if (!(h.hi > h.lo && h.sum * 3 >= (h.hi - h.lo) * 2 && h.hi - h.lo < (32ull << 30))) return false;
  return !h.bad || range_mapped(b + h.lo, b + h.hi);
}

// The slot's latest completed record, whatever pointers it was for (false if none or torn).
bool latest_hint(const ScratchSlot* slot, ExtentHint* out) {
  const ExtentHint* p = slot->data.hint;
  ExtentHint h{};
  h.lo = __atomic_load_n(&p->lo, __ATOMIC_RELAXED);
  h.hi = __atomic_load_n(&p->hi, __ATOMIC_RELAXED);
  h.sum = __atomic_load_n(&p->sum, __ATOMIC_RELAXED);
  h.bad = __atomic_load_n(&p->bad, __ATOMIC_RELAXED);
  h.seq = __atomic_load_n(&p->seq, __ATOMIC_RELAXED);
  h.chk = __atomic_load_n(&p->chk, __ATOMIC_RELAXED);
  if (h.seq == 0 || (h.lo ^ h.hi ^ h.sum ^ h.bad ^ h.seq ^ kExtentCheck) != h.chk) return false;
  *out = h;
  return true;
}

int run_var_auto(DeviceCtx& c, const void* d_base, size_t n, const uint64_t* d_off, const uint32_t* d_len,
                 uint32_t* d_out, hipStream_t stream, bool update) {
  if (n < kAutoMinPayloads) return run_var_sorted(c, d_base, n, d_off, d_len, d_out, stream, update);
  std::lock_guard<std::mutex> lk(c.arena_mu);
  ScratchSlot* slot = nullptr;
  int rc = scratch_slot(c, stream, sorted_scratch_bytes(n), &slot);
  if (rc) return rc;
  if (!slot->data.hint) {
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&slot->data.hint), sizeof(ExtentHint), hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(slot->data.hint, 0, sizeof(ExtentHint));
  }
  const Scratch::Key key{d_base, d_off, d_len, n, update};
  if (!(key == slot->data.key)) {
    slot->data.key = key;
    slot->data.key_since = slot->data.calls + 1;
    slot->data.seen_seq = slot->data.prev_seq = 0;
    slot->data.since_extent = 0;
  }
  poll_hint(slot);
  {  // the arena scratch that the densest span recorded here needs (whatever pointers it was for), so that a device
     // choice on fresh pointers of a similar batch finds room for it (the span's alignment can add a superblock at
     // each end)
    ExtentHint lh{};
    if (latest_hint(slot, &lh) && lh.hi > lh.lo && lh.sum * 3 >= (lh.hi - lh.lo) * 2 && lh.hi - lh.lo < (32ull << 30))
      slot->data.arena_want = std::max<uint64_t>(
          slot->data.arena_want, arena_geom_of(((lh.hi - lh.lo) >> 13) + 2, grid_cus(c)).words * sizeof(uint32_t));
  }
  const ExtentHint& h = slot->data.seen;
  const uint64_t b = (uint64_t)(uintptr_t)d_base;
  const bool have1 = slot->data.seen_seq >= slot->data.key_since;                // a completed record for these pointers
  const bool have2 = have1 && slot->data.prev_seq >= slot->data.key_since;       // and the one before it
  const bool allow_h = have1 && record_allows_arena(h, b);
  bool arena = have2 && allow_h && h.lo == slot->data.prev.lo && h.hi == slot->data.prev.hi &&
               slot->data.prev.sum * 3 >= (h.hi - h.lo) * 2;
  // Safe: sorted starts with gaps < 4 KiB put every byte of the span on a page holding payload bytes; any
  // other order or gap qualifies when the span lies inside one device allocation (the arena's cost follows
  // the span, which the density bound above keeps within 1.5x the payload bytes, in any order).
  const bool any_order = arena && (h.bad || slot->data.prev.bad);
  ArenaLaunch a{};
  if ((rc = arena_powers(c, a))) return rc;
  if (arena) {
    arena_fill_range(c, d_base, b + h.lo, b + h.hi, a);
    a.off = d_off;
    a.len = d_len;
    a.n = n;
    a.out = d_out;
    a.update = update;
    a.check_lo = h.lo;
    a.check_hi = h.hi;
    a.check_any_order = any_order;
    if (a.nsb && (rc = scratch_slot(c, stream, arena_geom(a).words * sizeof(uint32_t), &slot))) return rc;
    if (++slot->data.since_extent < kAutoRefresh && range_mapped(b + h.lo, b + h.hi)) {
      // between two recording calls: the arena launches alone (kAutoRefresh above)
      c.auto_arena++;
      c.auto_unchecked++;
      a.scratch = reinterpret_cast<uint32_t*>(path_scratch(slot));
      const hipError_t e = launch_arena(a, stream);
      rc = e == hipSuccess ? ANNETY_CRC_OK : hip_fail(e);
      const int rd = scratch_done(c, slot);
      return rc ? rc : rd;
    }
    slot->data.since_extent = 0;
  }
  // No verdict from two records yet, and no record against the arena: the device chooses (AutoChoice) from this
  // call's own extent - so a caller that passes fresh offset/length arrays on every call (per-connection batches)
  // still reaches the arena path. A completed record for these pointers that rules the arena out
  // (sparse, or unsorted across allocations) sends the call to the sorted path directly.
  const bool device = !arena && !(have1 && !allow_h);
  if (device) {
    const size_t want = std::max<size_t>(sorted_scratch_bytes(n), (size_t)slot->data.arena_want);
    if ((rc = scratch_slot(c, stream, want, &slot))) return rc;
  }
  // this call's extent: the check the arena launches make, and the next calls' record (on the sorted
  // path the bucket count runs in the same launch, and the bucket place publishes the record)
  const uint64_t seq = ++slot->data.calls;
  (arena ? c.auto_arena : device ? c.auto_device : c.auto_sorted)++;
  if (arena) {
    uint32_t parts = 0;
    hipError_t e = launch_extent(d_off, d_len, n, slot->data.ptr, &parts, nullptr, stream);
    if (e == hipSuccess) {
      a.check = static_cast<const uint64_t*>(slot->data.ptr);
      a.check_parts = parts;
      a.record = slot->data.hint;
      a.record_seq = seq;
      a.scratch = reinterpret_cast<uint32_t*>(path_scratch(slot));
      e = launch_arena(a, stream);
    }
    rc = e == hipSuccess ? ANNETY_CRC_OK : hip_fail(e);
  } else if (device) {
    // extent partials, then both paths' launches; each runs only if the device's choice is its own, and the one that
    // runs publishes the record
    uint32_t parts = 0;
    hipError_t e = launch_extent(d_off, d_len, n, slot->data.ptr, &parts, nullptr, stream);
    AutoChoice ch{};
    ch.ws = static_cast<const uint64_t*>(slot->data.ptr);
    ch.parts = parts;
    ch.blocks = (uint32_t)grid_cus(c);
    ch.base = b;
    ch.cap_words = slot->data.bytes / sizeof(uint32_t);
    if (e == hipSuccess) {
      arena_fill_range(c, d_base, 0, 0, a);  // (images and grid; the span is the device's; a.pow8k set above)
      a.off = d_off;
      a.len = d_len;
      a.n = n;
      a.out = d_out;
      a.update = update;
      a.record = slot->data.hint;
      a.record_seq = seq;
      a.scratch = reinterpret_cast<uint32_t*>(path_scratch(slot));
      a.choice = ch;
      e = launch_arena(a, stream);
    }
    rc = e == hipSuccess ? run_var_sorted_in(c, slot, d_base, n, d_off, d_len, d_out, stream, update, slot->data.hint,
                                             seq, &ch)
                         : hip_fail(e);
  } else {
    rc = run_var_sorted_in(c, slot, d_base, n, d_off, d_len, d_out, stream, update, slot->data.hint, seq);
  }
  const int rd = scratch_done(c, slot);
  return rc ? rc : rd;
}

// The general variable path (annety_crc_set_var_path; initial value from ANNETY_CRC_VAR_PATH = auto / sorted,
// or ANNETY_CRC_VAR_AUTO=0 = sorted): 0 = automatic arena/sorted choice from recorded extents, 1 = the
// length-sorted path.
std::atomic<int> g_var_mode{[] {
  const char* e = std::getenv("ANNETY_CRC_VAR_PATH");
  if (e && std::strcmp(e, "sorted") == 0) return 1;
  if (e && std::strcmp(e, "auto") == 0) return 0;
  const char* a = std::getenv("ANNETY_CRC_VAR_AUTO");
  return a && a[0] == '0' ? 1 : 0;
}()};

int run_var_any(DeviceCtx& c, const void* d_base, size_t n, const uint64_t* d_off, const uint32_t* d_len,
                uint32_t* d_out, hipStream_t stream, bool update) {
  switch (g_var_mode.load(std::memory_order_relaxed)) {
    case 1: return run_var_sorted(c, d_base, n, d_off, d_len, d_out, stream, update);
    default: return run_var_auto(c, d_base, n, d_off, d_len, d_out, stream, update);
  }
}

bool fixed_fast_ok(const void* d_base, size_t len, size_t stride) {
  return ((uintptr_t)d_base % 16 == 0) && (stride % 16 == 0) && (len % 16 == 0) && len >= 16 &&
         len / 16 <= 0xFFFFFFFFull;
}

// ---- long payloads: end-aligned segments joined by the combine identity (see crc32_split_join) ----
constexpr uint64_t kSegBytes = 65536;  // 512 lines: 16 rounds of a 32-lane group
constexpr uint32_t kMaxSegs = 16384;
static_assert(kMaxSegs == kSplitMaxSegs, "the sorted path's split join uses this power table");

// Split policy (annety_crc_set_split; the environment's ANNETY_CRC_SPLIT / ANNETY_CRC_SEG give the initial
// values, read once): mode 0 never splits, 1 splits whenever the payload spans two segments, -1 = auto;
// min_segment = the smallest segment size (a power of two >= 4096). Atomics: no getenv per call, and a
// setter racing with a call is harmless (either policy gives the same digests).
std::atomic<int> g_split_mode{[] {
  const char* e = std::getenv("ANNETY_CRC_SPLIT");
  return e && *e ? std::atoi(e) : -1;
}()};
std::atomic<uint64_t> g_split_seg{[] {
  const char* e = std::getenv("ANNETY_CRC_SEG");
  const unsigned long long v = e && *e ? std::strtoull(e, nullptr, 10) : 0;
  return v >= 4096 && (v & (v - 1)) == 0 ? (uint64_t)v : kSegBytes;
}()};
int split_mode() { return g_split_mode.load(std::memory_order_relaxed); }
uint64_t split_min_segment() { return g_split_seg.load(std::memory_order_relaxed); }

// Segment size for a fixed-length batch, or 0 to run payloads whole.
uint64_t split_segment(size_t n, uint64_t len, int cus) {
  const int mode = split_mode();
  if (mode == 0) return 0;
  uint64_t seg = split_min_segment();
  while ((len + seg - 1) / seg > kMaxSegs) seg *= 2;
  if (len < 2 * seg) return 0;
  const uint64_t S = (len + seg - 1) / seg;
  if ((uint64_t)n * S > 0xFFFFFFFFull) return 0;  // descriptor indices are 32-bit
  if (mode == 1) return seg;                        // forced (tests, tuning)
  // auto: whole payloads leave 32-lane groups idle (or a long tail) when there are fewer than two
  // payloads per group; with more, whole payloads measured slightly faster.
  const size_t groups_chip = (size_t)cus * fixed_kernel_block() / 32;
  return n < 2 * groups_chip ? seg : 0;
}

// powers[(m-1)*32 + b] = shift_{m*seg}(1 << b) for m = 1..kMaxSegs-1, built once per segment size.
int split_powers(DeviceCtx& c, uint64_t seg, const uint32_t** out) {
  std::lock_guard<std::mutex> lk(c.pow_mu);
  for (auto& pw : c.powers)
    if (pw.first == seg) {
      *out = pw.second;
      return ANNETY_CRC_OK;
    }
  std::vector<uint32_t> host((size_t)(kMaxSegs - 1) * 32);
  const Gf2Mat step = shift_matrix(seg);
  Gf2Mat cur = step;
  for (uint32_t m = 1; m < kMaxSegs; m++) {
    std::memcpy(&host[(size_t)(m - 1) * 32], cur.col, sizeof cur.col);
    cur = gf2_mul(step, cur);
  }
  uint32_t* d = nullptr;
  HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d), host.size() * 4));
  hipError_t e = hipMemcpy(d, host.data(), host.size() * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    (void)hipFree(d);
    return hip_fail(e);
  }
  c.powers.emplace_back(seg, d);
  *out = d;
  return ANNETY_CRC_OK;
}

int run_split(DeviceCtx& c, const void* d_base, size_t n, uint64_t len, uint64_t stride, uint64_t seg,
              uint32_t* d_out, hipStream_t stream) {
  const uint32_t S = (uint32_t)((len + seg - 1) / seg);
  const size_t tasks = n * (size_t)S;
  const uint32_t* powers = nullptr;
  int rc = split_powers(c, seg, &powers);
  if (rc) return rc;
  const size_t crc_bytes = (tasks * 4 + 15) & ~(size_t)15;
  std::lock_guard<std::mutex> lk(c.arena_mu);
  ScratchSlot* slot = nullptr;
  if ((rc = scratch_slot(c, stream, 16 + crc_bytes + 16 * tasks, &slot))) return rc;
  char* scratch = path_scratch(slot);
  uint32_t* range = reinterpret_cast<uint32_t*>(scratch);
  uint32_t* seg_crc = reinterpret_cast<uint32_t*>(scratch + 16);
  void* desc = scratch + 16 + crc_bytes;
  if (stride == len && len % seg == 0 && fixed_fast_ok(d_base, seg, seg)) {
    // packed payloads whose length is a multiple of seg: the segments are one uniform fixed batch
    rc = run_fixed(c, d_base, tasks, seg, seg, seg_crc, false, stream);
  } else {
    hipError_t e = launch_split_desc(d_base, n, len, stride, seg, S, desc, range, stream);
    rc = e == hipSuccess ? run_var(c, d_base, tasks, 0, 0, 32, desc, range, seg_crc, stream) : hip_fail(e);
  }
  if (rc == ANNETY_CRC_OK) {
    hipError_t e = launch_split_join(seg_crc, n, S, powers, d_out, stream);
    if (e != hipSuccess) rc = hip_fail(e);
  }
  const int rd = scratch_done(c, slot);
  return rc ? rc : rd;
}

}  // namespace

// crc32_kernels.h: each launcher names the kernel it enqueues (consecutive repeats are kept once).
void annety_crc::note_kernel(const char* name) {
  const size_t n = std::strlen(name);
  if (t_kernels.size() >= n && t_kernels.compare(t_kernels.size() - n, n, name) == 0) return;
  if (!t_kernels.empty()) t_kernels += " + ";
  t_kernels += name;
}

extern "C" {

int annety_crc_init(int device) {
  if (device < 0 || device >= kMaxDev) return ANNETY_CRC_ENODEV;
  std::lock_guard<std::mutex> lk(g_init_mu);
  return init_device_locked(device);
}

int annety_crc_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) prev = 0;
  for (int d = 0; d < kMaxDev; d++) {
    DeviceCtx& c = g_dev[d];
    if (!c.ready) continue;
    (void)hipSetDevice(d);
    std::lock_guard<std::mutex> sl(c.stg_mu);
    for (int i = 0; i < 2; i++) {
      if (c.stg.stream[i]) (void)hipStreamDestroy(c.stg.stream[i]);
      if (c.stg.done[i]) (void)hipEventDestroy(c.stg.done[i]);
      if (c.stg.h_pinned[i]) (void)hipHostFree(c.stg.h_pinned[i]);
      if (c.stg.h_out[i]) (void)hipHostFree(c.stg.h_out[i]);
      if (c.stg.d_buf[i]) (void)hipFree(c.stg.d_buf[i]);
      if (c.stg.d_out[i]) (void)hipFree(c.stg.d_out[i]);
    }
    if (c.stg.d_stream) (void)hipFree(c.stg.d_stream);
    if (c.stg.d_meta) (void)hipFree(c.stg.d_meta);
    if (c.stg.h_meta) (void)hipHostFree(c.stg.h_meta);
    c.stg = Staging{};
    {
      std::lock_guard<std::mutex> pl(c.pow_mu);
      for (auto& pw : c.powers) (void)hipFree(pw.second);
      c.powers.clear();
    }
    {
      std::lock_guard<std::mutex> al(c.arena_mu);
      // the slots' last uses may carry no event: drain the device before their memory goes
      if (c.slots.size()) {
        (void)hipDeviceSynchronize();
        c.shutdown_syncs++;
      }
      HipSlotOps ops;
      c.slots.clear(ops, [](ScratchSlot& sl) {
        if (sl.data.ptr) (void)hipFree(sl.data.ptr);
        if (sl.data.hint) (void)hipHostFree(sl.data.hint);
      });
    }
    free_images(c);
    c.ready = false;
  }
  (void)hipSetDevice(prev);
  return ANNETY_CRC_OK;
}

int annety_crc_last_hip_error(void) { return t_last_hip; }

int annety_crc_reserve_cus(int n) {
  if (n < 0) return ANNETY_CRC_EINVAL;
  g_reserved_cus.store(n);
  return ANNETY_CRC_OK;
}

int annety_crc_set_split(int mode, uint64_t min_segment) {
  if (mode < -1 || mode > 1) return ANNETY_CRC_EINVAL;
  if (min_segment && (min_segment < 4096 || (min_segment & (min_segment - 1)))) return ANNETY_CRC_EINVAL;
  g_split_mode.store(mode);
  g_split_seg.store(min_segment ? min_segment : kSegBytes);
  return ANNETY_CRC_OK;
}

int annety_crc_set_split_cap(uint32_t extra_segments) {
  if (extra_segments > kSplitSegCap) return ANNETY_CRC_EINVAL;
  g_split_cap.store(extra_segments);
  return ANNETY_CRC_OK;
}

int annety_crc_scratch_stats(int device, uint64_t* slots, uint64_t* handoffs, uint64_t* device_syncs) {
  if (device < 0 || device >= kMaxDev) return ANNETY_CRC_ENODEV;
  DeviceCtx& c = g_dev[device];
  std::lock_guard<std::mutex> lk(c.arena_mu);
  if (slots) *slots = c.slots.size();
  if (handoffs) *handoffs = c.slots.handoffs();
  if (device_syncs) *device_syncs = c.slots.drains() + c.shutdown_syncs.load();
  return ANNETY_CRC_OK;
}

int annety_crc_set_var_path(int mode) {
  if (mode < 0 || mode > 1) return ANNETY_CRC_EINVAL;
  g_var_mode.store(mode);
  return ANNETY_CRC_OK;
}

int annety_crc_get_var_path(void) { return g_var_mode.load(); }

int annety_crc_var_path_stats(int device, uint64_t* arena, uint64_t* sorted, uint64_t* arena_unrecorded,
                              uint64_t* device_chosen) {
  if (device < 0 || device >= kMaxDev) return ANNETY_CRC_ENODEV;
  if (arena) *arena = g_dev[device].auto_arena.load();
  if (sorted) *sorted = g_dev[device].auto_sorted.load();
  if (arena_unrecorded) *arena_unrecorded = g_dev[device].auto_unchecked.load();
  if (device_chosen) *device_chosen = g_dev[device].auto_device.load();
  return ANNETY_CRC_OK;
}

int annety_crc_stream_release(void* stream) {
  hipStream_t s = static_cast<hipStream_t>(stream);
  DeviceCtx* c = nullptr;
  int rc = stream_ctx(s, &c);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(c->arena_mu);
  HipSlotOps ops;
  return c->slots.release(ops, s, s == hipStreamPerThread, [&](ScratchSlot& sl) -> int {
    // Every member is released even when a step fails (the slot leaves the table either way), and the first
    // failure is returned (an early return leaked the pinned record).
    int first = ANNETY_CRC_OK;
    auto note = [&](hipError_t e) {
      if (e != hipSuccess && first == ANNETY_CRC_OK) first = hip_fail(e);
    };
    // stream-ordered: the memory returns to the pool after the stream's queued work, nobody waits
    if (sl.data.ptr) note(hipFreeAsync(sl.data.ptr, s));
    sl.data.ptr = nullptr;
    if (sl.data.hint) {  // the stream's queued extent kernels may still write it: wait for them first
      const hipError_t e = hipStreamSynchronize(s);
      note(e);
      if (e != hipSuccess) (void)hipDeviceSynchronize();  // nothing may still write it when it goes
      (void)hipHostFree(sl.data.hint);
      sl.data.hint = nullptr;
    }
    return first;
  });
}

int annety_crc32_batch_fixed(const void* d_base, size_t n, size_t len, size_t stride, uint32_t* d_out,
                             void* stream) {
  if (n == 0) return ANNETY_CRC_OK;
  if (!d_out || (!d_base && len > 0) || (n > 1 && stride < len)) return ANNETY_CRC_EINVAL;
  DeviceCtx* c = nullptr;
  int rc = stream_ctx(static_cast<hipStream_t>(stream), &c);
  if (rc) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (len == 0) {
    HIP_TRY(hipMemsetAsync(d_out, 0, n * sizeof(uint32_t), s));  // crc of the empty string is 0
    return ANNETY_CRC_OK;
  }
  if (const uint64_t seg = split_segment(n, len, c->cus)) return run_split(*c, d_base, n, len, stride, seg, d_out, s);
  if (len > 0xFFFFFFFFull) return ANNETY_CRC_EINVAL;  // whole-payload kernels take 32-bit lengths
  if (fixed_fast_ok(d_base, len, stride)) return run_fixed(*c, d_base, n, len, stride, d_out, false, s);
  if (n > 0xFFFFFFFFull) return ANNETY_CRC_EINVAL;  // the general kernel's task descriptors hold 32-bit indices
  const uint64_t lines = (len + 255) / 128;
  return run_var(*c, d_base, n, stride, (uint32_t)len, pick_group(lines, n, c->cus), nullptr, nullptr, d_out, s);
}

int annety_crc32_batch_var(const void* d_base, const uint64_t* d_off, const uint32_t* d_len, size_t n,
                           uint32_t* d_out, void* stream) {
  if (n == 0) return ANNETY_CRC_OK;
  if (!d_base || !d_off || !d_len || !d_out) return ANNETY_CRC_EINVAL;
  DeviceCtx* c = nullptr;
  int rc = stream_ctx(static_cast<hipStream_t>(stream), &c);
  if (rc) return rc;
  if (n > 0xFFFFFFFFull) return ANNETY_CRC_EINVAL;  // order[] holds 32-bit payload indices
  return run_var_any(*c, d_base, n, d_off, d_len, d_out, static_cast<hipStream_t>(stream), false);
}

int annety_crc32_batch_var_arena(const void* d_arena, size_t arena_bytes, const uint64_t* d_off,
                                 const uint32_t* d_len, size_t n, uint32_t* d_out, void* stream) {
  if (n == 0) return ANNETY_CRC_OK;
  if (!d_arena || !d_off || !d_len || !d_out) return ANNETY_CRC_EINVAL;
  DeviceCtx* c = nullptr;
  int rc = stream_ctx(static_cast<hipStream_t>(stream), &c);
  if (rc) return rc;
  return run_arena(*c, d_arena, arena_bytes, d_off, d_len, n, d_out, static_cast<hipStream_t>(stream), false);
}

int annety_crc32_update_batch_var_arena(uint32_t* d_state, const void* d_arena, size_t arena_bytes,
                                        const uint64_t* d_off, const uint32_t* d_len, size_t n, void* stream) {
  if (n == 0) return ANNETY_CRC_OK;
  if (!d_state || !d_arena || !d_off || !d_len) return ANNETY_CRC_EINVAL;
  DeviceCtx* c = nullptr;
  int rc = stream_ctx(static_cast<hipStream_t>(stream), &c);
  if (rc) return rc;
  return run_arena(*c, d_arena, arena_bytes, d_off, d_len, n, d_state, static_cast<hipStream_t>(stream), true);
}

int annety_crc32_update_batch_fixed(uint32_t* d_state, const void* d_base, size_t n, size_t len, size_t stride,
                                    void* stream) {
  if (n == 0 || len == 0) return ANNETY_CRC_OK;  // no bytes: register unchanged
  if (!d_state || !d_base || (n > 1 && stride < len)) return ANNETY_CRC_EINVAL;
  if (len > 0xFFFFFFFFull) return ANNETY_CRC_EINVAL;
  DeviceCtx* c = nullptr;
  int rc = stream_ctx(static_cast<hipStream_t>(stream), &c);
  if (rc) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (fixed_fast_ok(d_base, len, stride)) return run_fixed(*c, d_base, n, len, stride, d_state, true, s);
  if (n > 0xFFFFFFFFull) return ANNETY_CRC_EINVAL;  // 32-bit task indices in the general kernel
  const uint64_t lines = (len + 255) / 128;  // odd shapes: the general kernel in update mode
  return run_var(*c, d_base, n, stride, (uint32_t)len, pick_group(lines, n, c->cus), nullptr, nullptr, d_state, s,
                 true);
}

int annety_crc32_update_batch_var(uint32_t* d_state, const void* d_base, const uint64_t* d_off, const uint32_t* d_len,
                                  size_t n, void* stream) {
  if (n == 0) return ANNETY_CRC_OK;
  if (!d_state || !d_base || !d_off || !d_len) return ANNETY_CRC_EINVAL;
  if (n > 0xFFFFFFFFull) return ANNETY_CRC_EINVAL;
  DeviceCtx* c = nullptr;
  int rc = stream_ctx(static_cast<hipStream_t>(stream), &c);
  if (rc) return rc;
  return run_var_any(*c, d_base, n, d_off, d_len, d_state, static_cast<hipStream_t>(stream), true);
}

// Staging ring of the current device's context, allocated for at least `need` bytes per slot.
static int ensure_ring(Staging& st, size_t need, size_t outs) {
  if (st.bytes >= need && st.outs >= outs) return ANNETY_CRC_OK;
  for (int i = 0; i < 2; i++) {
    if (st.h_pinned[i]) (void)hipHostFree(st.h_pinned[i]);
    if (st.d_buf[i]) (void)hipFree(st.d_buf[i]);
    if (st.d_out[i]) (void)hipFree(st.d_out[i]);
    if (st.h_out[i]) (void)hipHostFree(st.h_out[i]);
    st.h_pinned[i] = st.d_buf[i] = nullptr;
    st.d_out[i] = st.h_out[i] = nullptr;
    st.bytes = st.outs = 0;
    HIP_TRY(hipHostMalloc(&st.h_pinned[i], need, hipHostMallocDefault));
    HIP_TRY(hipMalloc(&st.d_buf[i], need));
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&st.d_out[i]), outs * 4));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&st.h_out[i]), outs * 4, hipHostMallocDefault));
    if (!st.stream[i]) HIP_TRY(hipStreamCreateWithFlags(&st.stream[i], hipStreamNonBlocking));
    if (!st.done[i]) HIP_TRY(hipEventCreateWithFlags(&st.done[i], hipEventDisableTiming));
  }
  st.bytes = need;
  st.outs = outs;
  return ANNETY_CRC_OK;
}

int annety_crc32_batch_fixed_host(const void* h_base, size_t n, size_t len, size_t stride, uint32_t* h_out) {
  if (n == 0) return ANNETY_CRC_OK;
  if (!h_out || (!h_base && len > 0) || (n > 1 && stride < len)) return ANNETY_CRC_EINVAL;
  if (len == 0) {
    std::memset(h_out, 0, n * sizeof(uint32_t));
    return ANNETY_CRC_OK;
  }
  DeviceCtx* c = nullptr;
  int rc = stream_ctx(nullptr, &c);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(c->stg_mu);
  Staging& st = c->stg;
  // Chunk of payloads per pipeline stage: ~64 MiB of packed payload bytes.
  const size_t plen = (len + 15) & ~(size_t)15;  // packed, 16-byte aligned stride on the device
  size_t per = std::max<size_t>(1, (64u << 20) / plen);
  per = std::min(per, n);
  const size_t need = per * plen;
  if ((rc = ensure_ring(st, need, per))) return rc;
  const char* src = static_cast<const char*>(h_base);
  // caller memory that is already pinned (hipHostRegister'ed NetBuffer arenas) is DMA'd in place when
  // the payloads are packed 16-byte multiples; otherwise it is packed into the pinned ring in parallel
  const bool direct = stride == plen && host_pinned(h_base, (n - 1) * stride + len);
  size_t pending_lo[2] = {0, 0}, pending_n[2] = {0, 0};
  auto drain = [&](int i) -> int {  // wait for slot i's batch and copy its digests out
    if (!pending_n[i]) return ANNETY_CRC_OK;
    const hipError_t e = hipEventSynchronize(st.done[i]);
    if (e == hipSuccess) std::memcpy(h_out + pending_lo[i], st.h_out[i], pending_n[i] * 4);
    pending_n[i] = 0;
    return e == hipSuccess ? ANNETY_CRC_OK : hip_fail(e);
  };
  auto fail = [&](int status) {  // leave no copy in flight on the shared staging buffers
    (void)hipStreamSynchronize(st.stream[0]);
    (void)hipStreamSynchronize(st.stream[1]);
    return status;
  };
  int slot = 0;
  for (size_t lo = 0; lo < n; lo += per, slot ^= 1) {
    const size_t cnt = std::min(per, n - lo);
    if ((rc = drain(slot))) return fail(rc);  // the previous use of this slot
    const char* from = src + lo * stride;
    if (!direct) {  // pack payloads into the pinned slot (the host side of a NetBuffer -> device hand-off)
      char* dst = static_cast<char*>(st.h_pinned[slot]);
      parallel_pack(dst, plen, from, stride, cnt, len);
      from = dst;
    }
    hipError_t e = hipMemcpyAsync(st.d_buf[slot], from, cnt * plen - (plen - len), hipMemcpyHostToDevice, st.stream[slot]);
    if (e != hipSuccess) return fail(hip_fail(e));
    rc = annety_crc32_batch_fixed(st.d_buf[slot], cnt, len, plen, st.d_out[slot], st.stream[slot]);
    if (rc) return fail(rc);
    e = hipMemcpyAsync(st.h_out[slot], st.d_out[slot], cnt * 4, hipMemcpyDeviceToHost, st.stream[slot]);
    if (e == hipSuccess) e = hipEventRecord(st.done[slot], st.stream[slot]);
    if (e != hipSuccess) return fail(hip_fail(e));
    pending_lo[slot] = lo;
    pending_n[slot] = cnt;
  }
  for (int i = 0; i < 2; i++)
    if ((rc = drain(i))) return fail(rc);
  return ANNETY_CRC_OK;
}

// Pins [h_ptr, h_ptr + bytes) for in-place DMA. The library records the range (crc32_host.h HostRegistry) and
// refuses a pointer that is not page-aligned or a range that shares a page with one it already pinned: the
// runtime pins whole pages, and two registrations sharing a page leave it a lookup it can resolve to either.
int annety_crc_host_register(void* h_ptr, size_t bytes) {
  if (!host::host_registry().add(h_ptr, bytes)) return ANNETY_CRC_EINVAL;
  const hipError_t e = hipHostRegister(h_ptr, bytes, hipHostRegisterDefault);
  if (e != hipSuccess) {
    host::host_registry().drop(h_ptr);
    return hip_fail(e);
  }
  return ANNETY_CRC_OK;
}

int annety_crc_host_unregister(void* h_ptr) {
  if (!h_ptr || !host::host_registry().drop(h_ptr)) return ANNETY_CRC_EINVAL;  // not a range pinned here
  HIP_TRY(hipHostUnregister(h_ptr));
  return ANNETY_CRC_OK;
}

const char* annety_crc_last_error_stage(void) { return t_fail_stage; }

const char* annety_crc_last_kernels(void) { return t_kernels.c_str(); }

static int lhc_verify(const void* d_stream, size_t stream_bytes, bool arena, const uint64_t* d_payload_off,
                      const uint32_t* d_payload_len, size_t n, uint8_t* d_ok, uint32_t* d_digest, void* stream) {
  if (n == 0) return ANNETY_CRC_OK;
  if (!d_stream || !d_payload_off || !d_payload_len || !d_ok) return ANNETY_CRC_EINVAL;
  DeviceCtx* c = nullptr;
  int rc = stream_ctx(static_cast<hipStream_t>(stream), &c);
  if (rc) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // arena: the stitch compares the trailers itself (crc32_arena.hip Stitcher VER), digests only if asked for
  if (arena) return run_arena(*c, d_stream, stream_bytes, d_payload_off, d_payload_len, n, d_digest, s, false, d_ok);
  uint32_t* dig = d_digest;
  if (!dig) HIP_TRY(hipMallocAsync(reinterpret_cast<void**>(&dig), n * sizeof(uint32_t), s));
  rc = annety_crc32_batch_var(d_stream, d_payload_off, d_payload_len, n, dig, stream);
  if (rc == ANNETY_CRC_OK) {
    hipError_t e = launch_lhc_compare(d_stream, d_payload_off, d_payload_len, n, dig, d_ok, s);
    if (e != hipSuccess) rc = hip_fail(e);
  }
  if (!d_digest) {
    hipError_t e = hipFreeAsync(dig, s);
    if (rc == ANNETY_CRC_OK && e != hipSuccess) rc = hip_fail(e);
  }
  return rc;
}

int annety_lhc_verify_batch(const void* d_stream, const uint64_t* d_payload_off, const uint32_t* d_payload_len,
                            size_t n, uint8_t* d_ok, uint32_t* d_digest, void* stream) {
  return lhc_verify(d_stream, 0, false, d_payload_off, d_payload_len, n, d_ok, d_digest, stream);
}

int annety_lhc_verify_stream(const void* d_stream, size_t stream_bytes, const uint64_t* d_payload_off,
                             const uint32_t* d_payload_len, size_t n, uint8_t* d_ok, uint32_t* d_digest,
                             void* stream) {
  return lhc_verify(d_stream, stream_bytes, true, d_payload_off, d_payload_len, n, d_ok, d_digest, stream);
}

static int encode_batch(const FrameRules& r, const void* d_src, const uint64_t* d_src_off, const uint32_t* d_len,
                        size_t n, void* d_dst, const uint64_t* d_frame_off, void* stream) {
  if (n == 0) return ANNETY_CRC_OK;
  if (!lhc_type_ok(r.T) || !d_src || !d_src_off || !d_len || !d_dst || !d_frame_off) return ANNETY_CRC_EINVAL;
  if (n > 0xFFFFFFFFull) return ANNETY_CRC_EINVAL;  // the long frames' entries hold 32-bit frame indices
  DeviceCtx* c = nullptr;
  int rc = stream_ctx(static_cast<hipStream_t>(stream), &c);
  if (rc) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  SortedSplit split{};  // the long frames' segment power tables (built once per device)
  rc = split_powers(*c, kSplitSeg, &split.powers);
  if (rc == ANNETY_CRC_OK) rc = split_powers(*c, kSplitSegBig, &split.powers_big);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(c->arena_mu);
  ScratchSlot* slot = nullptr;
  if ((rc = scratch_slot(*c, s, kEncLongScratchBytes, &slot))) return rc;
  Scratch& d = slot->data;
  char* ctrs = static_cast<char*>(d.ptr) + kEncCtrOff;
  if (!d.enc_clean) {  // both counter sets
    const hipError_t z = hipMemsetAsync(ctrs, 0, 32, s);
    if (z != hipSuccess) return hip_fail(z);
    d.enc_clean = true;
  }
  const uint32_t set = (uint32_t)(d.encodes & 1);
  EncLong lg{};
  lg.ctr = reinterpret_cast<unsigned long long*>(ctrs + 16 * set + 8);
  lg.ctr_next = reinterpret_cast<unsigned long long*>(ctrs + 16 * (set ^ 1) + 8);
  char* scratch = path_scratch(slot);
  lg.digest = reinterpret_cast<uint32_t*>(scratch);
  lg.entry = lg.digest + kEncLongCap;
  lg.desc = scratch + 8 * kEncLongCap;
  lg.seg_dst = reinterpret_cast<uint64_t*>(scratch + 8 * kEncLongCap + 16 * kEncLongSegCap);
  // one pass: each payload read once, its frame (header, copy, CRC trailer) written once (crc32_frames.hip); the
  // long frames it hands over: their digests on the sorted kernel (segments), then their copy, headers and trailers
  // (lanes per frame: 4 when most frames fit one 4-line round - 408-byte chat frames: 0.594 -> 0.427 ms for 2M - else
  // 8 - frames of 16 B - 1 KiB: 0.646 ms against 0.83 with 4; the two instances choose on the device, crc32_frames.hip)
  hipError_t e = launch_lhc_encode_fused(d_src, d_src_off, d_len, n, r.T, r.enc_min, r.enc_max, d_dst, d_frame_off,
                                         c->d_zero, c->d_slice, c->d_w8, lg, grid_cus(*c), s);
  if (e == hipSuccess) {
    VarLaunch a{};
    a.base = d_src;
    a.n = kEncLongCap;
    a.desc = lg.desc;
    a.range = reinterpret_cast<const uint32_t*>(lg.ctr) - 1;  // {0, segments}
    a.img_slice = c->d_slice;
    a.img_unshift = c->d_unshift;
    a.out = lg.digest;
    a.max_blocks = grid_cus(*c);
    e = launch_var_sorted(a, c->d_w8, split, s);
  }
  if (e == hipSuccess) e = launch_lhc_encode_long(d_len, r.T, d_dst, d_frame_off, lg, grid_cus(*c), s);
  if (e != hipSuccess) {
    d.enc_clean = false;  // the next call zeroes both sets first
    (void)scratch_done(*c, slot);
    return hip_fail(e);
  }
  d.encodes++;
  return scratch_done(*c, slot);
}

int annety_lhc_encode_batch(const void* d_src, const uint64_t* d_src_off, const uint32_t* d_len, size_t n,
                            int length_type, int64_t max_payload, void* d_dst, const uint64_t* d_frame_off,
                            void* stream) {
  return encode_batch(lhc_rules(length_type, max_payload), d_src, d_src_off, d_len, n, d_dst, d_frame_off, stream);
}

int annety_pbc_encode_batch(const void* d_src, const uint64_t* d_src_off, const uint32_t* d_len, size_t n,
                            void* d_dst, const uint64_t* d_frame_off, void* stream) {
  return encode_batch(kPbcRules, d_src, d_src_off, d_len, n, d_dst, d_frame_off, stream);
}

// Codec::recv over K host receive buffers at once (include/codec/Codec.h:52-76 + LengthHeaderCodec::decode
// :71-137), one per connection (src/TcpConnection.cc:438-461: each TcpConnection owns its input NetBuffer).
// The buffers are concatenated on the device (one stream, one arena verify). On the host each buffer's
// header walk - a dependent chain of one header read per frame, ~140-170 ns a frame from DRAM - runs on
// its own walker thread (connections are independent), while the buffers are packed into pinned memory
// and uploaded (pinned buffers, e.g. annety_crc_host_register'ed NetBuffer arenas, are DMA'd in place).
// Pageable frame buffers: packed into the library's pinned ring by the pack threads (default), or uploaded by
// the runtime's own pageable copy (annety_crc_set_frames_pack(0); initial value from ANNETY_CRC_FRAMES_PACK).
// The pack never hands a user page to the DMA engine, so the runtime's pinning of user memory (which keys on
// pages that neighbouring buffers and earlier registrations may share) stays out of this path.
static std::atomic<int> g_frames_pack{[] {
  const char* e = std::getenv("ANNETY_CRC_FRAMES_PACK");
  return (e && e[0] == '0') ? 0 : 1;
}()};

// ANNETY_CRC_SYNC_STAGES=1: finish the stage's queued work now, so a failure is charged to it.
static int stage_sync(hipStream_t s) {
  if (!sync_stages()) return ANNETY_CRC_OK;
  const hipError_t e = hipStreamSynchronize(s);
  return e == hipSuccess ? ANNETY_CRC_OK : hip_fail(e);
}

static int verify_host_iov(const FrameRules& r, const void* const* h_bufs, const size_t* sizes, size_t k,
                           uint64_t* h_payload_off, uint32_t* h_payload_len, uint8_t* h_ok, size_t max_frames,
                           size_t* conn_frames, size_t* conn_consumed, int* conn_rt) {
  if (!lhc_type_ok(r.T) || (k && (!h_bufs || !sizes || !conn_frames || !conn_consumed || !conn_rt)) ||
      (max_frames && (!h_payload_off || !h_payload_len || !h_ok)))
    return ANNETY_CRC_EINVAL;
  std::vector<uint64_t> base(k + 1, 0);
  for (size_t c = 0; c < k; c++) {
    if (!h_bufs[c] && sizes[c]) return ANNETY_CRC_EINVAL;
    base[c + 1] = base[c] + sizes[c];
    conn_frames[c] = conn_consumed[c] = 0;
    conn_rt[c] = 0;
  }
  const uint64_t total = base[k];
  if (total == 0 || max_frames == 0) return ANNETY_CRC_OK;
  // the walks (connections, and segments of large buffers, side by side: FrameWalks) run on their own
  // threads while the bytes are packed and uploaded
  FrameWalks fw(r, h_bufs, sizes, k, max_frames);
  fw.start();
  auto join_walkers = [&] { fw.join(); };
  DeviceCtx* c = nullptr;
  int rc = stream_ctx(nullptr, &c);
  if (rc) {
    join_walkers();
    return rc;
  }
  std::unique_lock<std::mutex> lk(c->stg_mu);
  Staging& st = c->stg;
  set_stage("staging buffers");
  auto fail = [&](int status) {
    join_walkers();
    if (st.stream[0]) (void)hipStreamSynchronize(st.stream[0]);
    if (st.stream[1]) (void)hipStreamSynchronize(st.stream[1]);
    return status;
  };
  if ((rc = ensure_ring(st, std::max<size_t>(st.bytes, 64u << 20), std::max<size_t>(st.outs, 1)))) return fail(rc);
  if (st.stream_cap < total) {
    if (st.d_stream) (void)hipFree(st.d_stream);
    st.d_stream = nullptr;
    st.stream_cap = 0;
    const hipError_t e = hipMalloc(reinterpret_cast<void**>(&st.d_stream), total);
    if (e != hipSuccess) return fail(hip_fail(e));
    st.stream_cap = total;
  }
  hipStream_t s = st.stream[0];
  bool pinned = true;
  for (size_t i = 0; i < k && pinned; i++) pinned = !sizes[i] || host_pinned(h_bufs[i], sizes[i]);
  set_stage(pinned ? "upload (pinned, in place)" : g_frames_pack.load() ? "upload (packed)" : "upload (pageable)");
  if (pinned || !g_frames_pack.load()) {
    for (size_t i = 0; i < k; i++) {
      if (!sizes[i]) continue;
      const hipError_t e = hipMemcpyAsync(st.d_stream + base[i], h_bufs[i], sizes[i], hipMemcpyHostToDevice, s);
      if (e != hipSuccess) return fail(hip_fail(e));
    }
  } else {
    const size_t chunk = st.bytes;
    size_t src = 0;  // buffer holding the chunk's first byte
    for (uint64_t lo = 0, i = 0; lo < total; lo += chunk, i++) {
      const int slot = (int)(i & 1);
      const uint64_t hi = std::min<uint64_t>(total, lo + chunk);
      if (i >= 2) {  // the slot's previous upload has finished reading it
        const hipError_t e = hipEventSynchronize(st.done[slot]);
        if (e != hipSuccess) return fail(hip_fail(e));
      }
      // gather [lo, hi) of the concatenation from the buffers it spans, in parallel pieces
      char* dst = static_cast<char*>(st.h_pinned[slot]);
      while (src < k && base[src + 1] <= lo) src++;
      for (size_t b = src; b < k && base[b] < hi; b++) {
        const uint64_t a = std::max<uint64_t>(lo, base[b]), e = std::min<uint64_t>(hi, base[b + 1]);
        if (e > a)
          parallel_pack(dst + (a - lo), e - a, static_cast<const char*>(h_bufs[b]) + (a - base[b]), e - a, 1, e - a);
      }
      hipError_t e = hipMemcpyAsync(st.d_stream + lo, dst, hi - lo, hipMemcpyHostToDevice, s);
      if (e == hipSuccess) e = hipEventRecord(st.done[slot], s);
      if (e != hipSuccess) return fail(hip_fail(e));
    }
  }
  if ((rc = stage_sync(s))) return fail(rc);
  set_stage("walk join");
  join_walkers();
  std::vector<ConnWalk>& walks = fw.walks();
  // frames in connection order, the output bound applied in that order (Codec::recv's per-connection
  // results; a connection cut by the bound stops as annety_lhc_parse does at max_frames: rt 0)
  size_t nf = 0;
  int prc = 0;
  for (size_t i = 0; i < k; i++) {
    ConnWalk& w = walks[i];
    size_t m = w.off.size();
    if (nf + m > max_frames) {
      m = max_frames - nf;
      w.rt = 0;
      w.consumed = m ? w.off[m - 1] + w.len[m - 1] + 4 : 0;
    }
    for (size_t f = 0; f < m; f++) {
      h_payload_off[nf + f] = w.off[f];
      h_payload_len[nf + f] = w.len[f];
    }
    conn_frames[i] = m;
    conn_consumed[i] = w.consumed;
    conn_rt[i] = w.rt;
    if (w.rt < 0) prc = w.rt;
    nf += m;
  }
  if (prc < 0) {
    (void)hipStreamSynchronize(s);
    return prc;
  }
  if (nf) {
    set_stage("metadata buffers");
    if (st.meta_cap < nf) {
      if (st.d_meta) (void)hipFree(st.d_meta);
      st.d_meta = nullptr;
      st.meta_cap = 0;
      const hipError_t e = hipMalloc(reinterpret_cast<void**>(&st.d_meta), nf * 17);
      if (e != hipSuccess) return fail(hip_fail(e));
      st.meta_cap = nf;
    }
    if (st.h_meta_cap < nf) {
      if (st.h_meta) (void)hipHostFree(st.h_meta);
      st.h_meta = nullptr;
      st.h_meta_cap = 0;
      const hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&st.h_meta), nf * 13, hipHostMallocDefault);
      if (e != hipSuccess) return fail(hip_fail(e));
      st.h_meta_cap = nf;
    }
    // device offsets are into the concatenation; the host outputs stay relative to each buffer
    uint64_t* m_off = reinterpret_cast<uint64_t*>(st.h_meta);
    for (size_t i = 0, f = 0; i < k; i++)
      for (size_t q = 0; q < conn_frames[i]; q++, f++) m_off[f] = h_payload_off[f] + base[i];
    std::memcpy(st.h_meta + nf * 8, h_payload_len, nf * 4);
    uint64_t* d_off = reinterpret_cast<uint64_t*>(st.d_meta);
    uint32_t* d_len = reinterpret_cast<uint32_t*>(st.d_meta + nf * 8);
    uint32_t* d_dig = d_len + nf;
    uint8_t* d_ok = reinterpret_cast<uint8_t*>(d_dig + nf);
    set_stage("metadata upload");
    hipError_t e = hipMemcpyAsync(d_off, st.h_meta, nf * 12, hipMemcpyHostToDevice, s);  // off then len
    if (e != hipSuccess) return fail(hip_fail(e));
    if ((rc = stage_sync(s))) return fail(rc);
    set_stage("arena verify");  // (the stitch compares the trailers: no digests kept)
    rc = run_arena(*c, st.d_stream, total, d_off, d_len, nf, nullptr, s, false, d_ok);
    if (rc == ANNETY_CRC_OK) rc = stage_sync(s);
    if (rc == ANNETY_CRC_OK) {
      set_stage("verdict download");
      e = hipMemcpyAsync(st.h_meta + nf * 12, d_ok, nf, hipMemcpyDeviceToHost, s);
      if (e != hipSuccess) rc = hip_fail(e);
    }
  }
  set_stage("final sync");
  const hipError_t e = hipStreamSynchronize(s);
  if (rc == ANNETY_CRC_OK && e != hipSuccess) rc = hip_fail(e);
  if (rc == ANNETY_CRC_OK && nf) std::memcpy(h_ok, st.h_meta + nf * 12, nf);
  return rc;
}

int annety_crc_set_frames_pack(int pack) {
  if (pack != 0 && pack != 1) return ANNETY_CRC_EINVAL;
  g_frames_pack.store(pack);
  return ANNETY_CRC_OK;
}

// One receive buffer: the K = 1 case of verify_host_iov.
static int verify_host(const FrameRules& r, const void* h_stream, size_t size, uint64_t* h_payload_off,
                       uint32_t* h_payload_len, uint8_t* h_ok, size_t max_frames, size_t* n_frames, size_t* consumed) {
  if (!n_frames || !consumed || !lhc_type_ok(r.T) || (!h_stream && size) ||
      (max_frames && (!h_payload_off || !h_payload_len || !h_ok)))
    return ANNETY_CRC_EINVAL;
  int crt = 0;
  const int rc = verify_host_iov(r, &h_stream, &size, 1, h_payload_off, h_payload_len, h_ok, max_frames, n_frames,
                                 consumed, &crt);
  return rc ? rc : crt;
}

int annety_lhc_verify_host(const void* h_stream, size_t size, int length_type, int64_t max_payload,
                           uint64_t* h_payload_off, uint32_t* h_payload_len, uint8_t* h_ok, size_t max_frames,
                           size_t* n_frames, size_t* consumed) {
  return verify_host(lhc_rules(length_type, max_payload), h_stream, size, h_payload_off, h_payload_len, h_ok,
                     max_frames, n_frames, consumed);
}

int annety_pbc_verify_host(const void* h_stream, size_t size, uint64_t* h_payload_off, uint32_t* h_payload_len,
                           uint8_t* h_ok, size_t max_frames, size_t* n_frames, size_t* consumed) {
  return verify_host(kPbcRules, h_stream, size, h_payload_off, h_payload_len, h_ok, max_frames, n_frames, consumed);
}

int annety_lhc_verify_host_iov(const void* const* h_bufs, const size_t* sizes, size_t k, int length_type,
                               int64_t max_payload, uint64_t* h_payload_off, uint32_t* h_payload_len, uint8_t* h_ok,
                               size_t max_frames, size_t* conn_frames, size_t* conn_consumed, int* conn_rt) {
  return verify_host_iov(lhc_rules(length_type, max_payload), h_bufs, sizes, k, h_payload_off, h_payload_len, h_ok,
                         max_frames, conn_frames, conn_consumed, conn_rt);
}

int annety_pbc_verify_host_iov(const void* const* h_bufs, const size_t* sizes, size_t k, uint64_t* h_payload_off,
                               uint32_t* h_payload_len, uint8_t* h_ok, size_t max_frames, size_t* conn_frames,
                               size_t* conn_consumed, int* conn_rt) {
  return verify_host_iov(kPbcRules, h_bufs, sizes, k, h_payload_off, h_payload_len, h_ok, max_frames, conn_frames,
                         conn_consumed, conn_rt);
}

}  // extern "C"
