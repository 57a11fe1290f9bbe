// Host-only parts of libannety_crc.so (crc32_host.h): worker pools, frame walks, encode plans, host
// registrations, shard plans, and the host scalar replacements of annety::Crc32c. No HIP: g++ builds this
// file alone for the sanitizer self-test (annety_amd/csrc/Makefile `sanitize`).
#include "crc32_host.h"

#include <unistd.h>

#include <atomic>
#include <cstdlib>
#include <cstring>

#include "annety_crc.h"
#include "crc32_math.h"

namespace annety_crc {
namespace host {

// ---------------- WorkPool ----------------
WorkPool::WorkPool(int workers) {
  for (int i = 0; i < workers; i++) workers_.emplace_back([this] { loop(); });
}

WorkPool::~WorkPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& w : workers_) w.join();
}

std::unique_ptr<WorkPool::Job> WorkPool::submit(size_t n, std::function<void(size_t)> fn) {
  auto job = std::make_unique<Job>();
  job->fn = std::move(fn);
  job->total = job->left = n;
  if (n) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      jobs_.push_back(job.get());
    }
    cv_.notify_all();
  }
  return job;
}

void WorkPool::wait(Job& job) {
  for (;;) {
    size_t i;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (job.next >= job.total) break;
      i = job.next++;
    }
    job.fn(i);
    finish(job);
  }
  std::unique_lock<std::mutex> lk(mu_);
  job.done_cv.wait(lk, [&] { return job.left == 0; });
  const auto it = std::find(jobs_.begin(), jobs_.end(), &job);
  if (it != jobs_.end()) jobs_.erase(it);
}

void WorkPool::finish(Job& job) {
  std::lock_guard<std::mutex> lk(mu_);
  if (--job.left == 0) job.done_cv.notify_all();
}

void WorkPool::loop() {
  for (;;) {
    Job* job = nullptr;
    size_t i = 0;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] {
        if (stop_) return true;
        for (Job* j : jobs_)
          if (j->next < j->total) return true;
        return false;
      });
      if (stop_) return;
      for (Job* j : jobs_)
        if (j->next < j->total) {
          job = j;
          break;
        }
      i = job->next++;
    }
    job->fn(i);
    finish(*job);
  }
}

namespace {
int pool_threads(const char* env, int dflt) {
  int t = dflt;
  if (const char* e = std::getenv(env)) t = std::max(1, std::min(64, std::atoi(e)));
  return t;
}
int default_threads() { return (int)std::min<unsigned>(8, std::max<unsigned>(1, std::thread::hardware_concurrency())); }
}  // namespace

WorkPool& pack_pool() {
  static WorkPool pool(pool_threads("ANNETY_CRC_PACK_THREADS", default_threads()) - 1);
  return pool;
}

WorkPool& walk_pool() {
  static WorkPool pool(pool_threads("ANNETY_CRC_WALK_THREADS", default_threads()));
  return pool;
}

void parallel_pack(char* dst, size_t dstride, const char* src, size_t sstride, size_t cnt, size_t len) {
  if (dstride == sstride && dstride == len) {  // one contiguous block
    const size_t bytes = cnt * len, piece = std::max<size_t>(1 << 20, bytes / (4 * pack_pool().threads()) + 1);
    pack_pool().run((bytes + piece - 1) / piece, [&](size_t i) {
      const size_t lo = i * piece, hi = std::min(bytes, lo + piece);
      std::memcpy(dst + lo, src + lo, hi - lo);
    });
    return;
  }
  const size_t per = std::max<size_t>(1, (1 << 20) / std::max<size_t>(len, 1));
  pack_pool().run((cnt + per - 1) / per, [&](size_t i) {
    const size_t lo = i * per, hi = std::min(cnt, lo + per);
    for (size_t k = lo; k < hi; k++) std::memcpy(dst + k * dstride, src + k * sstride, len);
  });
}

// ---------------- frame walks ----------------
// A dependent chain of one header read per frame (~140-170 ns a frame from DRAM).
namespace {
enum class Step { kFrame, kInvalid, kIncomplete, kTooBig };

// The frame whose header starts at `pos`; *length = its length field (payload + 4 checksum bytes).
inline Step frame_at(const FrameRules& r, const unsigned char* p, size_t size, size_t pos, int64_t* length) {
  const size_t T = (size_t)r.T;
  if (pos > size || size - pos < T) return Step::kIncomplete;
  uint64_t u = 0;
  for (size_t b = 0; b < T; b++) u = (u << 8) | p[pos + b];
  switch (T) {  // sign-extend like peek_int8/16/32/64
    case 1: *length = (int8_t)u; break;
    case 2: *length = (int16_t)u; break;
    case 4: *length = (int32_t)u; break;
    default: *length = (int64_t)u; break;
  }
  if (*length < r.dec_min || (r.dec_max > 0 && *length > r.dec_max)) return Step::kInvalid;  // decode: -1
  if (size - pos - T < (uint64_t)*length) return Step::kIncomplete;                           // decode: 0
  if (*length - 4 > 0xFFFFFFFFll) return Step::kTooBig;  // valid for the codec, beyond 32-bit lengths
  return Step::kFrame;
}
inline int step_rt(Step s) { return s == Step::kInvalid ? 1 : s == Step::kTooBig ? ANNETY_CRC_EINVAL : 0; }

// Frames from header position `pos` while pos < stop_at, at most `cap` of them in w.
void walk_range(const FrameRules& r, const unsigned char* p, size_t size, size_t pos, size_t stop_at, size_t cap,
                ConnWalk& w) {
  const size_t T = (size_t)r.T;
  while (pos < stop_at && w.off.size() < cap) {
    int64_t L = 0;
    const Step st = frame_at(r, p, size, pos, &L);
    if (st != Step::kFrame) {
      w.ended = true;
      w.rt = step_rt(st);
      break;
    }
    w.off.push_back(pos + T);
    w.len.push_back((uint32_t)(L - 4));
    pos += T + (size_t)L;
  }
  w.consumed = pos;
}

constexpr uint64_t kDefaultWalkSeg = 64ull << 20;
std::atomic<uint64_t> g_walk_seg{kDefaultWalkSeg};
constexpr size_t kWalkMaxSegs = 64;
constexpr size_t kSpecProbe = 1u << 20;

// Segment [lo, hi) of a buffer (not the first): a speculative entry, then the walk from it up to hi.
void walk_segment(const FrameRules& r, const unsigned char* p, size_t size, size_t lo, size_t hi, size_t cap,
                  ConnWalk& w) {
  const size_t T = (size_t)r.T;
  const int hops = T == 1 ? 32 : T == 2 ? 16 : 8;  // short length fields parse by chance more often
  const size_t end = std::min(size, lo + kSpecProbe);
  for (size_t q = lo; q < end; q++) {
    size_t pos = q;
    int h = 0;
    int64_t L = 0;
    for (; h < hops && frame_at(r, p, size, pos, &L) == Step::kFrame; h++) pos += T + (size_t)L;
    if (h == hops) {
      walk_range(r, p, size, q, hi, cap, w);
      return;
    }
  }
  w.consumed = SIZE_MAX;  // no entry found: the join walks this segment itself
}
}  // namespace

void set_walk_segment(uint64_t bytes) { g_walk_seg.store(bytes ? bytes : kDefaultWalkSeg); }
uint64_t walk_segment_bytes() { return g_walk_seg.load(); }

FrameWalks::FrameWalks(const FrameRules& r, const void* const* bufs, const size_t* sizes, size_t k, size_t cap)
    : r_(r), bufs_(bufs), sizes_(sizes), cap_(cap), bounds_(k), segs_(k), walks_(k) {
  const size_t seg = (size_t)g_walk_seg.load();
  for (size_t c = 0; c < k; c++) {
    const size_t m = std::max<size_t>(1, std::min<size_t>(kWalkMaxSegs, sizes[c] / seg));
    bounds_[c].resize(m + 1);
    for (size_t i = 0; i < m; i++) bounds_[c][i] = sizes[c] / m * i;
    bounds_[c][m] = SIZE_MAX;  // the last segment walks to the stream's end
    segs_[c].resize(m);
    for (size_t i = 0; i < m; i++) tasks_.push_back({c, i});
  }
}

FrameWalks::~FrameWalks() { join_threads(); }

void FrameWalks::start() { job_ = walk_pool().submit(tasks_.size(), [this](size_t i) { run(tasks_[i]); }); }

void FrameWalks::join() {
  join_threads();
  if (joined_) return;
  joined_ = true;
  for (size_t c = 0; c < walks_.size(); c++) splice(c);
}

void FrameWalks::run(const Task& t) {
  const size_t lo = bounds_[t.c][t.i], hi = bounds_[t.c][t.i + 1];
  if (t.i == 0)
    walk_range(r_, buf(t.c), sizes_[t.c], 0, hi, cap_, segs_[t.c][0]);
  else
    walk_segment(r_, buf(t.c), sizes_[t.c], lo, hi, cap_, segs_[t.c][t.i]);
}

void FrameWalks::join_threads() {
  if (job_) walk_pool().wait(*job_);
  job_.reset();
}

void FrameWalks::splice(size_t c) {
  std::vector<ConnWalk>& segs = segs_[c];
  ConnWalk& out = walks_[c];
  out = std::move(segs[0]);
  const unsigned char* p = buf(c);
  const size_t size = sizes_[c], T = (size_t)r_.T;
  size_t pos = out.consumed;
  for (size_t i = 1; i < segs.size() && !out.ended && out.off.size() < cap_; i++) {
    ConnWalk& s = segs[i];
    const size_t hi = bounds_[c][i + 1];
    while (!out.ended && out.off.size() < cap_ && pos < hi) {
      const auto it = std::lower_bound(s.off.begin(), s.off.end(), (uint64_t)pos + T);
      if (it != s.off.end() && *it == pos + T) {  // the true walk reached a header of the segment's walk
        const size_t j = (size_t)(it - s.off.begin());
        const size_t take = std::min(s.off.size() - j, cap_ - out.off.size());
        out.off.insert(out.off.end(), s.off.begin() + j, s.off.begin() + j + take);
        out.len.insert(out.len.end(), s.len.begin() + j, s.len.begin() + j + take);
        if (j + take < s.off.size()) {  // cut by the frame cap
          pos = out.off.back() + out.len.back() + 4;
          break;
        }
        pos = s.consumed;  // the segment's end, its own cap (go on frame by frame) or the stream's end
        if (s.ended) {
          out.ended = true;
          out.rt = s.rt;
        }
        continue;
      }
      int64_t L = 0;
      const Step st = frame_at(r_, p, size, pos, &L);
      if (st != Step::kFrame) {
        out.ended = true;
        out.rt = step_rt(st);
        break;
      }
      out.off.push_back(pos + T);
      out.len.push_back((uint32_t)(L - 4));
      pos += T + (size_t)L;
    }
  }
  out.consumed = pos;
  segs.clear();
}

int parse_frames(const FrameRules& r, const void* h_stream, size_t size, uint64_t* payload_off, uint32_t* payload_len,
                 size_t max_frames, size_t* n_frames, size_t* consumed) {
  if (!n_frames || !consumed || !lhc_type_ok(r.T) || (!h_stream && size) || (max_frames && (!payload_off || !payload_len)))
    return ANNETY_CRC_EINVAL;
  FrameWalks fw(r, &h_stream, &size, 1, max_frames);
  fw.start();
  fw.join();
  const ConnWalk& w = fw.walks()[0];
  std::copy(w.off.begin(), w.off.end(), payload_off);
  std::copy(w.len.begin(), w.len.end(), payload_len);
  *n_frames = w.off.size();
  *consumed = w.consumed;
  return w.rt;
}

// encode()'s per-payload decision (LengthHeaderCodec :169-176, ProtobufCodec :225-233): rt 0 for an empty
// payload, -1 outside [enc_min, enc_max], else 1 with a frame of T + len + 4 bytes. Rejected payloads get zero
// bytes, so the frames of the accepted ones are packed back to back as consecutive encode calls on one
// NetBuffer would leave them.
int encode_plan(const FrameRules& r, const uint32_t* h_len, size_t n, uint64_t* h_frame_off, int8_t* h_rt,
                uint64_t* total) {
  if (!lhc_type_ok(r.T) || !total || (n && (!h_len || !h_frame_off))) return ANNETY_CRC_EINVAL;
  uint64_t pos = 0;
  for (size_t i = 0; i < n; i++) {
    const int64_t L = h_len[i];
    const int8_t rt = L == 0 ? 0 : (L < r.enc_min || (r.enc_max > 0 && L > r.enc_max)) ? -1 : 1;
    if (h_rt) h_rt[i] = rt;
    h_frame_off[i] = pos;
    if (rt == 1) pos += (uint64_t)r.T + (uint64_t)L + 4;
  }
  *total = pos;
  return ANNETY_CRC_OK;
}

// ---------------- host registrations ----------------
size_t HostRegistry::page_size() {
  static const size_t pg = [] {
    const long v = sysconf(_SC_PAGESIZE);
    return v > 0 ? (size_t)v : (size_t)4096;
  }();
  return pg;
}

bool HostRegistry::add(const void* p, size_t bytes) {
  const size_t pg = page_size();
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
  if (!p || !bytes || lo % pg || bytes > UINTPTR_MAX - lo - pg) return false;
  const uintptr_t hi = lo + bytes, hi_pg = (hi + pg - 1) / pg * pg;
  std::lock_guard<std::mutex> lk(mu_);
  for (const Range& x : r_) {
    const uintptr_t x_hi_pg = (x.hi + pg - 1) / pg * pg;
    if (lo < x_hi_pg && x.lo < hi_pg) return false;  // the two share a page
  }
  r_.push_back({lo, hi});
  return true;
}

bool HostRegistry::drop(const void* p) {
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
  std::lock_guard<std::mutex> lk(mu_);
  for (size_t i = 0; i < r_.size(); i++)
    if (r_[i].lo == lo) {
      r_.erase(r_.begin() + (long)i);
      return true;
    }
  return false;
}

bool HostRegistry::covers(const void* p, size_t bytes) const {
  const uintptr_t lo = reinterpret_cast<uintptr_t>(p);
  if (!p || bytes > UINTPTR_MAX - lo) return false;
  const uintptr_t hi = lo + bytes;
  std::lock_guard<std::mutex> lk(mu_);
  for (const Range& x : r_)
    if (lo >= x.lo && hi <= x.hi) return true;
  return false;
}

size_t HostRegistry::size() const {
  std::lock_guard<std::mutex> lk(mu_);
  return r_.size();
}

HostRegistry& host_registry() {
  static HostRegistry reg;
  return reg;
}

}  // namespace host
}  // namespace annety_crc

// ---------------- host scalar replacements (drop-in for include/Crc32c.h) ----------------
namespace annety {
namespace internal {
// src/Crc32c.cc:20-92 — same symbols, same contents, generated from the polynomial at compile time.
#define ANNETY_T256(i) annety_crc::table256_entry(i)
#define ANNETY_R4(b) ANNETY_T256(b), ANNETY_T256(b + 1), ANNETY_T256(b + 2), ANNETY_T256(b + 3)
#define ANNETY_R16(b) ANNETY_R4(b), ANNETY_R4(b + 4), ANNETY_R4(b + 8), ANNETY_R4(b + 12)
#define ANNETY_R64(b) ANNETY_R16(b), ANNETY_R16(b + 16), ANNETY_R16(b + 32), ANNETY_R16(b + 48)
uint32_t crc32_table256[256] = {ANNETY_R64(0u), ANNETY_R64(64u), ANNETY_R64(128u), ANNETY_R64(192u)};
#define ANNETY_T16(i) annety_crc::table256_entry(16u * (i))
uint32_t crc32_table16[16] = {ANNETY_T16(0u),  ANNETY_T16(1u),  ANNETY_T16(2u),  ANNETY_T16(3u),
                              ANNETY_T16(4u),  ANNETY_T16(5u),  ANNETY_T16(6u),  ANNETY_T16(7u),
                              ANNETY_T16(8u),  ANNETY_T16(9u),  ANNETY_T16(10u), ANNETY_T16(11u),
                              ANNETY_T16(12u), ANNETY_T16(13u), ANNETY_T16(14u), ANNETY_T16(15u)};
}  // namespace internal
}  // namespace annety

using annety_crc::host::FrameRules;
using annety_crc::host::kPbcRules;
using annety_crc::host::lhc_rules;

extern "C" {

int annety_crc_abi_version(void) { return ANNETY_CRC_ABI_VERSION; }

const char* annety_crc_strerror(int status) {
  switch (status) {
    case ANNETY_CRC_OK: return "ok";
    case ANNETY_CRC_EINVAL: return "invalid argument";
    case ANNETY_CRC_EHIP: return "HIP runtime error";
    case ANNETY_CRC_ENOMEM: return "out of memory";
    case ANNETY_CRC_ENODEV: return "no usable gfx950 device";
    case ANNETY_CRC_ERCCL: return "collective failure";
    default: return "unknown status";
  }
}

// include/Crc32c.h:58-69
uint32_t annety_crc32_long(const char* buff, size_t len) {
  const unsigned char* p = reinterpret_cast<const unsigned char*>(buff);
  uint32_t crc = annety_crc::kInit;
  while (len--) crc = annety::internal::crc32_table256[(crc ^ *p++) & 0xff] ^ (crc >> 8);
  return crc ^ annety_crc::kXorOut;
}

// include/Crc32c.h:41-55
uint32_t annety_crc32_short(const char* buff, size_t len) {
  const unsigned char* p = reinterpret_cast<const unsigned char*>(buff);
  uint32_t crc = annety_crc::kInit;
  while (len--) {
    const unsigned c = *p++;
    crc = annety::internal::crc32_table16[(crc ^ (c & 0xf)) & 0xf] ^ (crc >> 4);
    crc = annety::internal::crc32_table16[(crc ^ (c >> 4)) & 0xf] ^ (crc >> 4);
  }
  return crc ^ annety_crc::kXorOut;
}

// include/Crc32c.h:71-82
void annety_crc32_update(uint32_t* crc, const char* buff, size_t len) {
  if (!crc) return;
  const unsigned char* p = reinterpret_cast<const unsigned char*>(buff);
  uint32_t c = *crc;
  while (len--) c = annety::internal::crc32_table256[(c ^ *p++) & 0xff] ^ (c >> 8);
  *crc = c;
}

uint32_t annety_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) {
  return annety_crc::combine(crc_a, crc_b, len_b);
}

const uint32_t* annety_crc32_table16(void) { return annety::internal::crc32_table16; }
const uint32_t* annety_crc32_table256(void) { return annety::internal::crc32_table256; }

int annety_crc_set_walk_segment(uint64_t bytes) {
  if (bytes && bytes < 4096) return ANNETY_CRC_EINVAL;
  annety_crc::host::set_walk_segment(bytes);
  return ANNETY_CRC_OK;
}

// include/codec/LengthHeaderCodec.h:71-137 without the CRC: signed big-endian length (peek_int*),
// min_payload = checksum_length = 4, max_payload check, completeness check.
int annety_lhc_parse(const void* h_stream, size_t size, int length_type, int64_t max_payload, uint64_t* payload_off,
                     uint32_t* payload_len, size_t max_frames, size_t* n_frames, size_t* consumed) {
  return annety_crc::host::parse_frames(lhc_rules(length_type, max_payload), h_stream, size, payload_off, payload_len,
                                        max_frames, n_frames, consumed);
}

int annety_pbc_parse(const void* h_stream, size_t size, uint64_t* payload_off, uint32_t* payload_len,
                     size_t max_frames, size_t* n_frames, size_t* consumed) {
  return annety_crc::host::parse_frames(kPbcRules, h_stream, size, payload_off, payload_len, max_frames, n_frames,
                                        consumed);
}

int annety_lhc_encode_plan(const uint32_t* h_len, size_t n, int length_type, int64_t max_payload,
                           uint64_t* h_frame_off, int8_t* h_rt, uint64_t* total) {
  return annety_crc::host::encode_plan(lhc_rules(length_type, max_payload), h_len, n, h_frame_off, h_rt, total);
}

int annety_pbc_encode_plan(const uint32_t* h_len, size_t n, uint64_t* h_frame_off, int8_t* h_rt, uint64_t* total) {
  return annety_crc::host::encode_plan(kPbcRules, h_len, n, h_frame_off, h_rt, total);
}

// Contiguous block shards, balanced to within one payload.
int annety_crc_shard_plan(size_t n, int nshards, size_t* first, size_t* count) {
  if (nshards <= 0 || !first || !count) return ANNETY_CRC_EINVAL;
  for (int k = 0; k < nshards; k++) {
    const size_t lo = (size_t)((unsigned __int128)n * (unsigned)k / (unsigned)nshards);
    const size_t hi = (size_t)((unsigned __int128)n * (unsigned)(k + 1) / (unsigned)nshards);
    first[k] = lo;
    count[k] = hi - lo;
  }
  return ANNETY_CRC_OK;
}

// The device group's transfer schedule (crc32_group.cpp): shard k in `chunks` near-equal pieces.
int annety_crc_group_schedule(const size_t* n_shard, int nd, size_t chunks, size_t* plan) {
  if (!n_shard || nd <= 0 || chunks == 0 || !plan) return ANNETY_CRC_EINVAL;
  size_t base = 0;
  for (int k = 0; k < nd; k++) {
    for (size_t c = 0; c < chunks; c++) {
      const size_t lo = n_shard[k] * c / chunks, hi = n_shard[k] * (c + 1) / chunks;
      size_t* e = plan + (c * (size_t)nd + (size_t)k) * 3;
      e[0] = lo;         // first payload of the piece, within shard k
      e[1] = hi - lo;    // payloads in the piece (0: nothing to compute or move)
      e[2] = base + lo;  // where its digests land in the root's output
    }
    base += n_shard[k];
  }
  return ANNETY_CRC_OK;
}

}  // extern "C"
