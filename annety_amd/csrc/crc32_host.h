// Host-only engine parts of libannety_crc.so: no HIP in this header or in crc32_host.cpp, so that g++
// builds them alone under AddressSanitizer/UBSan and ThreadSanitizer (`make -C annety_amd/csrc sanitize`,
// tests/native/host_selftest.cpp). crc32_capi.cpp drives the device with them.
//
//  * WorkPool: the persistent host thread pools (staging packs, frame walks).
//  * FrameWalks / parse_frames: LengthHeaderCodec::decode's framing over host buffers
//    (include/codec/LengthHeaderCodec.h:71-137), segmented and speculative, exact.
//  * encode_plan: LengthHeaderCodec::encode's per-payload decision (:146-201).
//  * HostRegistry: the library's own record of hipHostRegister'ed ranges (page-aligned, disjoint).
//  * SlotTable: per-stream device scratch bookkeeping, templated on the runtime operations it needs
//    (fence create/record/wait, device drain), so a fake runtime can drive it in the self-test.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace annety_crc {
namespace host {

// ---------------- persistent worker pools ----------------
// Several callers may run jobs at once (the device group's per-device threads, concurrent host batches):
// each job sits in a shared list, the workers take pieces of any job, and a caller that waits also works on
// its own job until it is done, so concurrent jobs share the workers instead of queueing behind one another.
class WorkPool {
 public:
  struct Job {
    std::function<void(size_t)> fn;
    size_t next = 0, total = 0, left = 0;
    std::condition_variable done_cv;
  };
  explicit WorkPool(int workers);
  ~WorkPool();
  WorkPool(const WorkPool&) = delete;
  WorkPool& operator=(const WorkPool&) = delete;
  int threads() const { return (int)workers_.size() + 1; }
  // Queues fn(i) for i in [0, n) to the workers; wait() on the returned job.
  std::unique_ptr<Job> submit(size_t n, std::function<void(size_t)> fn);
  // The caller works on what is left of the job, then waits until the workers' pieces are done.
  void wait(Job& job);
  // Runs fn(i) for i in [0, n) on the pool and the calling thread; returns when all are done.
  template <class F>
  void run(size_t n, F&& fn) {
    if (n == 0) return;
    if (workers_.empty() || n == 1) {
      for (size_t i = 0; i < n; i++) fn(i);
      return;
    }
    auto job = submit(n, std::function<void(size_t)>(std::ref(fn)));
    wait(*job);
  }

 private:
  void finish(Job& job);
  void loop();
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Job*> jobs_;  // jobs with pieces left or still being finished (owned by their callers)
  bool stop_ = false;
};

WorkPool& pack_pool();  // ANNETY_CRC_PACK_THREADS (default min(8, cores)); the caller is one of the threads
WorkPool& walk_pool();  // ANNETY_CRC_WALK_THREADS (default min(8, cores)); submitted jobs start on the workers

// dst[i*dstride, +len) = src[i*sstride, +len) for i < cnt, in parallel pieces of >= 1 MiB.
void parallel_pack(char* dst, size_t dstride, const char* src, size_t sstride, size_t cnt, size_t len);

// ---------------- LengthHeaderCodec / ProtobufCodec framing ----------------
// Framing rules of annety's two CRC codecs (same wire layout [len T BE][payload][crc BE]):
//   decode: length (payload + 4) outside [dec_min, dec_max] is invalid (decode -1); dec_max <= 0: no limit
//   encode: payload length 0 -> rt 0; outside [enc_min, enc_max] -> rt -1; enc_max <= 0: no limit
struct FrameRules {
  int T;
  int64_t dec_min, dec_max, enc_min, enc_max;
};
inline bool lhc_type_ok(int t) { return t == 1 || t == 2 || t == 4 || t == 8; }
// LengthHeaderCodec (include/codec/LengthHeaderCodec.h): min_payload() = checksum_length() = 4 (:214-217),
// max_payload checked only when > 0 (:102, :174), decode :71-137, encode :146-201.
inline FrameRules lhc_rules(int T, int64_t max_payload) { return {T, 4, max_payload, 1, max_payload}; }
// ProtobufCodec (include/protobuf/ProtobufCodec.h): T = kLengthType32 (:260-263), min_payload() =
// header_length() 4 + 2 + checksum_length() 4 = 10 (:279-283), max_payload() = 64 MiB unconditional
// (:273-277); decode rejects length < 10 or > 64 MiB (:149-153), encode rejects payload < 10 - 4 = 6 or
// > 64 MiB (:229-233).
constexpr FrameRules kPbcRules = {4, 10, 64ll << 20, 6, 64ll << 20};

// One connection's walk: payload offsets (relative to its buffer) and lengths, where it stopped, and why.
struct ConnWalk {
  std::vector<uint64_t> off;
  std::vector<uint32_t> len;
  size_t consumed = 0;  // where the walk stopped
  int rt = 0;           // 0, 1 (invalid length) or -1 = ANNETY_CRC_EINVAL (a frame beyond 32-bit lengths)
  bool ended = false;   // stopped by the stream itself, not by its stop position or the frame cap
};

// Segment size of the walks (annety_crc_set_walk_segment; 0 restores the default 64 MiB).
void set_walk_segment(uint64_t bytes);
uint64_t walk_segment_bytes();

// The walks of k buffers, on walk_pool()'s workers: a buffer of at least two walk segments is walked in
// segments side by side; segment 0 from offset 0 as the codec does, every later one from a speculative entry
// (the first position in its first MiB from which several frames in a row parse). join() splices them in
// order: the true walk continues frame by frame until it lands on a header a segment's walk recorded, from
// where both are the same chain; a segment whose entry was wrong is walked again by the join. Speculation
// costs time, never a different result. walks()[c] = buffer c's walk from offset 0 after join().
class FrameWalks {
 public:
  FrameWalks(const FrameRules& r, const void* const* bufs, const size_t* sizes, size_t k, size_t cap);
  ~FrameWalks();
  FrameWalks(const FrameWalks&) = delete;
  FrameWalks& operator=(const FrameWalks&) = delete;
  void start();  // the walks start on walk_pool()'s workers
  void join();   // idempotent; the caller takes any walks still queued
  std::vector<ConnWalk>& walks() { return walks_; }

 private:
  struct Task {
    size_t c, i;
  };
  const unsigned char* buf(size_t c) const { return static_cast<const unsigned char*>(bufs_[c]); }
  void run(const Task& t);
  void join_threads();
  void splice(size_t c);

  const FrameRules r_;
  const void* const* bufs_;
  const size_t* sizes_;
  const size_t cap_;
  std::vector<std::vector<size_t>> bounds_;
  std::vector<std::vector<ConnWalk>> segs_;
  std::vector<ConnWalk> walks_;
  std::vector<Task> tasks_;
  std::unique_ptr<WorkPool::Job> job_;
  bool joined_ = false;
};

// annety_lhc_parse / annety_pbc_parse: one buffer's walk into caller arrays (status as the C-ABI's).
int parse_frames(const FrameRules& r, const void* h_stream, size_t size, uint64_t* payload_off, uint32_t* payload_len,
                 size_t max_frames, size_t* n_frames, size_t* consumed);
// annety_lhc_encode_plan / annety_pbc_encode_plan.
int encode_plan(const FrameRules& r, const uint32_t* h_len, size_t n, uint64_t* h_frame_off, int8_t* h_rt,
                uint64_t* total);

// ---------------- host registrations ----------------
// The ranges annety_crc_host_register pinned. The library DMAs a caller buffer in place only when the whole
// buffer lies inside one of them: the runtime's own view of pinned memory cannot tell a stale or partly
// overlapping registration from a live one, so nothing else counts as pinned.
class HostRegistry {
 public:
  static size_t page_size();
  // Refuses (false) a pointer that is not page-aligned, zero bytes, or a page range overlapping one already
  // recorded. Records [p, p + bytes) on success; the caller pins it afterwards (and calls drop() if that fails).
  bool add(const void* p, size_t bytes);
  // Removes the range that starts at p; false if p starts none.
  bool drop(const void* p);
  // [p, p + bytes) lies inside one recorded range.
  bool covers(const void* p, size_t bytes) const;
  size_t size() const;

 private:
  struct Range {
    uintptr_t lo, hi;
  };
  mutable std::mutex mu_;
  std::vector<Range> r_;
};
HostRegistry& host_registry();

// ---------------- per-stream scratch slots ----------------
// Device scratch of the arena, split and sorted paths, one slot per stream, reused in stream order with no
// per-call event while the table has room (an event after every call costs 2-4 us of GPU time per call).
// Slots are keyed by stream handle, and for the per-thread handle also by calling thread. When the table is
// full, a new stream takes the least recently used slot over:
//   * its last call was made while the table was full, or on a per-thread handle: a fence was recorded on
//     the owner's stream right after that call (while the caller had it alive), and the new stream waits
//     for the fence;
//   * otherwise (its last call predates the table filling up): the device is drained once, which leaves
//     every slot clean, since nothing queued before the drain can still run.
// So no event is ever recorded on a stream other than the calling one: a stream destroyed without
// annety_crc_stream_release costs at most one drain, never a use of a dead handle.
//
// Ops (the runtime; a fake in tests/native/host_selftest.cpp) provides
//   int make_fence(void** ev); void destroy_fence(void* ev);
//   int record(void* ev, const void* stream);      // on the calling thread's stream
//   int wait(const void* stream, void* ev);        // stream waits for ev
//   int drain();                                   // every stream of the device has finished
// each returning 0 or a negative status. The caller serialises calls into one table (the device's mutex).
enum class SlotState : uint8_t {
  kClean,   // nothing queued that uses the slot may still run (fresh, or drained)
  kFenced,  // `fence` was recorded right after the latest call
  kOpen,    // the latest call carries no fence
};

template <class P>
struct Slot {
  const void* owner = nullptr;  // stream handle of the latest call
  bool per_thread = false;      // owner is the per-thread handle: `tid` tells its stream apart
  std::thread::id tid{};
  uint64_t tick = 0;            // latest use, for the LRU hand-over
  void* fence = nullptr;
  SlotState state = SlotState::kClean;
  P data{};                     // the path's scratch (pointer, size, extent record, ...)
};

template <class P>
class SlotTable {
 public:
  explicit SlotTable(size_t cap) : cap_(cap ? cap : 1) {}
  size_t cap() const { return cap_; }
  size_t size() const { return slots_.size(); }
  uint64_t handoffs() const { return handoffs_; }
  uint64_t drains() const { return drains_; }
  bool full() const { return slots_.size() >= cap_; }

  // The slot for a call on `owner` from this thread (fresh, its own, or handed over), ready to be used in
  // stream order on owner. *out is null on failure.
  template <class Ops>
  int acquire(Ops& ops, const void* owner, bool per_thread, Slot<P>** out) {
    *out = nullptr;
    const std::thread::id me = std::this_thread::get_id();
    Slot<P>* s = find(owner, per_thread, me);
    if (s) {
      // a per-thread handle names the stream of whichever thread holds this id now: a thread that reuses
      // an exited thread's id must still wait for the old stream's last call
      if (per_thread && s->state == SlotState::kFenced) {
        const int rc = ops.wait(owner, s->fence);
        if (rc) return rc;
      }
    } else if (slots_.size() < cap_) {
      auto fresh = std::make_unique<Slot<P>>();
      const int rc = ops.make_fence(&fresh->fence);
      if (rc) return rc;
      s = fresh.get();
      slots_.push_back(std::move(fresh));
    } else {
      s = slots_.front().get();
      for (auto& x : slots_)
        if (x->tick < s->tick) s = x.get();
      if (s->state == SlotState::kFenced) {
        const int rc = ops.wait(owner, s->fence);
        if (rc) return rc;
      } else if (s->state == SlotState::kOpen) {
        const int rc = ops.drain();
        if (rc) return rc;
        drains_++;
        for (auto& x : slots_) x->state = SlotState::kClean;
      }
      handoffs_++;
    }
    s->owner = owner;
    s->per_thread = per_thread;
    s->tid = me;
    s->tick = ++tick_;
    *out = s;
    return 0;
  }

  // After the call's work on `owner` is enqueued: fence it when a later hand-over may need the fence
  // (the table is full, or the handle is per-thread), else leave it open.
  template <class Ops>
  int done(Ops& ops, Slot<P>* s) {
    if (s->per_thread || full()) {
      const int rc = ops.record(s->fence, s->owner);
      s->state = rc ? SlotState::kOpen : SlotState::kFenced;
      return rc;
    }
    s->state = SlotState::kOpen;
    return 0;
  }

  // Drops owner's slot (this thread's, for the per-thread handle): free(slot) releases its payload in
  // owner's stream order. Returns free's status; 0 if owner holds no slot.
  template <class Ops, class Free>
  int release(Ops& ops, const void* owner, bool per_thread, Free&& free) {
    const std::thread::id me = std::this_thread::get_id();
    for (size_t i = 0; i < slots_.size(); i++) {
      Slot<P>& s = *slots_[i];
      if (!owns(s, owner, per_thread, me)) continue;
      const int rc = free(s);
      ops.destroy_fence(s.fence);
      slots_.erase(slots_.begin() + (long)i);
      return rc;
    }
    return 0;
  }

  // Every slot (shutdown, after a drain): free(slot), then the table is empty.
  template <class Ops, class Free>
  void clear(Ops& ops, Free&& free) {
    for (auto& s : slots_) {
      free(*s);
      ops.destroy_fence(s->fence);
    }
    slots_.clear();
  }

 private:
  static bool owns(const Slot<P>& s, const void* owner, bool per_thread, std::thread::id me) {
    return s.owner == owner && s.per_thread == per_thread && (!per_thread || s.tid == me);
  }
  Slot<P>* find(const void* owner, bool per_thread, std::thread::id me) {
    for (auto& s : slots_)
      if (owns(*s, owner, per_thread, me)) return s.get();
    return nullptr;
  }
  size_t cap_;
  std::vector<std::unique_ptr<Slot<P>>> slots_;
  uint64_t tick_ = 0, handoffs_ = 0, drains_ = 0;
};

}  // namespace host
}  // namespace annety_crc
