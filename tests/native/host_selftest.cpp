// Self-test of the engine's host-only parts (annety_amd/csrc/crc32_host.{h,cpp}), built by
// `make -C annety_amd/csrc sanitize` twice: under AddressSanitizer + UBSan and under ThreadSanitizer
// (the reference relies on -Wthread-safety, CMakeLists.txt:34, and runtime thread checks,
// src/EventLoop.cc:215-221; this engine has more host concurrency than the reference's pure functions).
// Every part runs from several threads at once:
//   1. WorkPool: concurrent run()/submit()+wait() callers on one pool; parallel_pack on the shared pool.
//   2. Frame walks: parse_frames and multi-buffer FrameWalks against a plain sequential walk of
//      LengthHeaderCodec::decode's framing (include/codec/LengthHeaderCodec.h:71-137), with 4 KiB walk
//      segments so every buffer is walked from speculative entries and joined; header-like payloads, invalid
//      lengths, incomplete tails, frame caps.
//   3. encode_plan against consecutive LengthHeaderCodec::encode decisions (:146-201).
//   4. Shard plans and the device group's transfer schedule.
//   5. HostRegistry: page alignment, no shared pages, coverage, concurrent add/drop/covers.
//   6. SlotTable over a fake runtime: a hand-over of a slot from stream A to stream B always follows either
//      a drain after A's last use or B's wait on a fence A recorded after its last use; no event is ever
//      recorded on a stream other than the calling one or on a destroyed stream.
// Exit status 0 and no sanitizer report = pass (tests/test_sanitize.py).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <set>
#include <thread>
#include <vector>

#include "annety_crc.h"
#include "crc32_host.h"

using namespace annety_crc::host;

#define CHECK(c)                                                                 \
  do {                                                                           \
    if (!(c)) {                                                                  \
      std::fprintf(stderr, "CHECK failed at %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::abort();                                                              \
    }                                                                            \
  } while (0)

template <class F>
void on_threads(int n, F&& f) {
  std::vector<std::thread> th;
  for (int t = 0; t < n; t++) th.emplace_back([&f, t] { f(t); });
  for (auto& x : th) x.join();
}

// ---------------- 1. worker pools ----------------
void test_workpool() {
  WorkPool pool(3);
  on_threads(6, [&](int t) {
    std::mt19937_64 rng(100 + t);
    for (int it = 0; it < 150; it++) {
      const size_t n = rng() % 64;
      std::vector<std::atomic<int>> hits(n);
      pool.run(n, [&](size_t i) { hits[i].fetch_add(1, std::memory_order_relaxed); });
      for (auto& h : hits) CHECK(h.load() == 1);
      std::vector<std::atomic<int>> h2(n);
      auto job = pool.submit(n, [&](size_t i) { h2[i].fetch_add(1, std::memory_order_relaxed); });
      if (rng() & 1) std::this_thread::yield();
      pool.wait(*job);
      for (auto& h : h2) CHECK(h.load() == 1);
    }
  });
  // the library's shared pack pool, from several callers at once
  on_threads(4, [&](int t) {
    std::mt19937_64 rng(200 + t);
    for (int it = 0; it < 20; it++) {
      const size_t cnt = 1 + rng() % 3000, len = 1 + rng() % 700, ss = len + rng() % 40, ds = len + rng() % 40;
      std::vector<char> src(cnt * ss), dst(cnt * ds, 0);
      for (auto& c : src) c = (char)rng();
      parallel_pack(dst.data(), ds, src.data(), ss, cnt, len);
      for (size_t k = 0; k < cnt; k++) CHECK(std::memcmp(dst.data() + k * ds, src.data() + k * ss, len) == 0);
      std::vector<char> a(cnt * len), b(cnt * len);
      for (auto& c : a) c = (char)rng();
      parallel_pack(b.data(), len, a.data(), len, cnt, len);  // one contiguous block
      CHECK(a == b);
    }
  });
  std::printf("workpool ok\n");
}

// ---------------- 2. frame walks ----------------
struct RefWalk {
  std::vector<uint64_t> off;
  std::vector<uint32_t> len;
  size_t consumed = 0;
  int rt = 0;
};

// Codec::recv's loop over LengthHeaderCodec::decode's framing, one frame after another.
RefWalk ref_walk(const FrameRules& r, const std::vector<unsigned char>& b, size_t cap) {
  RefWalk w;
  size_t pos = 0;
  const size_t T = (size_t)r.T;
  while (w.off.size() < cap && b.size() - pos >= T) {
    uint64_t u = 0;
    for (size_t i = 0; i < T; i++) u = (u << 8) | b[pos + i];
    int64_t L = T == 1 ? (int8_t)u : T == 2 ? (int16_t)u : T == 4 ? (int32_t)u : (int64_t)u;
    if (L < r.dec_min || (r.dec_max > 0 && L > r.dec_max)) {
      w.rt = 1;
      break;
    }
    if (b.size() - pos - T < (uint64_t)L) break;
    w.off.push_back(pos + T);
    w.len.push_back((uint32_t)(L - 4));
    pos += T + (size_t)L;
  }
  w.consumed = pos;
  return w;
}

std::vector<unsigned char> make_stream(std::mt19937_64& rng, int T, size_t frames, size_t maxlen, int flavour) {
  std::vector<unsigned char> s;
  const int64_t tmax = T == 1 ? 127 : T == 2 ? 32767 : (int64_t)1 << 40;
  for (size_t f = 0; f < frames; f++) {
    int64_t L = (int64_t)(rng() % (maxlen + 1)) + 4;
    if (L > tmax) L = tmax;
    for (int i = T - 1; i >= 0; i--) s.push_back((unsigned char)((uint64_t)L >> (8 * i)));
    for (int64_t i = 0; i < L; i++) {
      unsigned char c = (unsigned char)rng();
      if (flavour == 1) c = (unsigned char)(i % T == T - 1 ? (rng() % 8) + 4 : 0);  // payload bytes look like headers
      s.push_back(c);
    }
  }
  if (flavour == 2 && s.size() > 64) {  // an invalid length somewhere later
    const size_t at = s.size() / 2 + rng() % (s.size() / 4);
    for (int i = 0; i < T; i++) s[at + i] = 0xFF;
  }
  const size_t tail = rng() % 20;  // an incomplete next frame
  for (size_t i = 0; i < tail; i++) s.push_back((unsigned char)rng());
  return s;
}

void test_walks() {
  set_walk_segment(4096);  // every buffer here spans several segments: speculative entries + join
  CHECK(walk_segment_bytes() == 4096);
  on_threads(4, [&](int t) {
    std::mt19937_64 rng(300 + t);
    for (int it = 0; it < 40; it++) {
      const int T = 1 << (rng() % 4);
      const int flavour = (int)(rng() % 3);
      const FrameRules r = (rng() % 5 == 0) ? kPbcRules : lhc_rules(T, (rng() & 1) ? 0 : 2000);
      const int Tr = r.T;
      auto s = make_stream(rng, Tr, 50 + rng() % 400, Tr == 1 ? 100 : 3000, flavour);
      const size_t cap = (rng() % 4 == 0) ? 1 + rng() % 100 : s.size();
      const RefWalk want = ref_walk(r, s, cap);
      std::vector<uint64_t> off(cap + 1);
      std::vector<uint32_t> len(cap + 1);
      size_t nf = 0, used = 0;
      const int rc = parse_frames(r, s.data(), s.size(), off.data(), len.data(), cap, &nf, &used);
      CHECK(rc == want.rt);
      CHECK(nf == want.off.size() && used == want.consumed);
      for (size_t i = 0; i < nf; i++) CHECK(off[i] == want.off[i] && len[i] == want.len[i]);
      // several buffers in one FrameWalks (the K-connection verify)
      const size_t k = 1 + rng() % 5;
      std::vector<std::vector<unsigned char>> bufs;
      for (size_t c = 0; c < k; c++) bufs.push_back(make_stream(rng, Tr, rng() % 300, Tr == 1 ? 100 : 2000, (int)(rng() % 3)));
      std::vector<const void*> ptrs;
      std::vector<size_t> sizes;
      for (auto& b : bufs) {
        ptrs.push_back(b.empty() ? nullptr : b.data());
        sizes.push_back(b.size());
      }
      const size_t kcap = 1 << 20;
      FrameWalks fw(r, ptrs.data(), sizes.data(), k, kcap);
      fw.start();
      if (rng() & 1) fw.join();  // join is idempotent
      fw.join();
      for (size_t c = 0; c < k; c++) {
        const RefWalk wc = ref_walk(r, bufs[c], kcap);
        const ConnWalk& g = fw.walks()[c];
        CHECK(g.off == wc.off && g.len == wc.len && g.consumed == wc.consumed && g.rt == wc.rt);
      }
    }
  });
  // a FrameWalks destroyed before join (an early error return) waits for its walks
  {
    std::mt19937_64 rng(399);
    auto s = make_stream(rng, 4, 3000, 3000, 0);
    const void* p = s.data();
    size_t sz = s.size();
    FrameWalks fw(lhc_rules(4, 0), &p, &sz, 1, 1 << 20);
    fw.start();
  }
  set_walk_segment(0);
  CHECK(walk_segment_bytes() == 64ull << 20);
  std::printf("walks ok\n");
}

// ---------------- 3. encode plans ----------------
void test_encode_plan() {
  std::mt19937_64 rng(500);
  for (int it = 0; it < 200; it++) {
    const int T = 1 << (rng() % 4);
    const int64_t maxp = (rng() % 3 == 0) ? 0 : (int64_t)(rng() % 5000);
    const FrameRules r = (rng() % 4 == 0) ? kPbcRules : lhc_rules(T, maxp);
    const size_t n = rng() % 60;
    std::vector<uint32_t> lens(n);
    for (auto& l : lens) l = (rng() % 7 == 0) ? 0 : (uint32_t)(rng() % 6000);
    std::vector<uint64_t> off(n + 1);
    std::vector<int8_t> rt(n + 1);
    uint64_t total = 0;
    CHECK(encode_plan(r, lens.data(), n, off.data(), rt.data(), &total) == ANNETY_CRC_OK);
    uint64_t pos = 0;
    for (size_t i = 0; i < n; i++) {
      const int64_t L = lens[i];
      const int want = L == 0 ? 0 : (L < r.enc_min || (r.enc_max > 0 && L > r.enc_max)) ? -1 : 1;
      CHECK(rt[i] == want && off[i] == pos);
      if (want == 1) pos += (uint64_t)r.T + (uint64_t)L + 4;
    }
    CHECK(total == pos);
  }
  uint64_t total = 0;
  CHECK(encode_plan(lhc_rules(3, 0), nullptr, 0, nullptr, nullptr, &total) == ANNETY_CRC_EINVAL);
  std::printf("encode plan ok\n");
}

// ---------------- 4. shard plans and schedules ----------------
void test_plans() {
  std::mt19937_64 rng(600);
  for (int it = 0; it < 300; it++) {
    const size_t n = (it < 10) ? (size_t)it : rng() % 100000000;
    const int nd = 1 + (int)(rng() % 8);
    std::vector<size_t> first(nd), count(nd);
    CHECK(annety_crc_shard_plan(n, nd, first.data(), count.data()) == ANNETY_CRC_OK);
    size_t sum = 0, mn = SIZE_MAX, mx = 0;
    for (int k = 0; k < nd; k++) {
      CHECK(first[k] == sum);
      sum += count[k];
      mn = std::min(mn, count[k]);
      mx = std::max(mx, count[k]);
    }
    CHECK(sum == n && mx - mn <= 1);
    const size_t chunks = 1 + rng() % 6;
    std::vector<size_t> plan(chunks * nd * 3);
    CHECK(annety_crc_group_schedule(count.data(), nd, chunks, plan.data()) == ANNETY_CRC_OK);
    for (int k = 0; k < nd; k++) {
      size_t next = 0;
      for (size_t c = 0; c < chunks; c++) {
        const size_t* e = &plan[(c * nd + k) * 3];
        CHECK(e[0] == next && e[2] == first[k] + e[0]);
        next += e[1];
      }
      CHECK(next == count[k]);
    }
  }
  CHECK(annety_crc_shard_plan(5, 0, nullptr, nullptr) == ANNETY_CRC_EINVAL);
  std::printf("plans ok\n");
}

// ---------------- 5. host registrations ----------------
void test_registry() {
  HostRegistry reg;
  const size_t pg = HostRegistry::page_size();
  const uintptr_t base = (uintptr_t)1 << 40;  // addresses only: the registry never touches the memory
  auto P = [&](uintptr_t off) { return reinterpret_cast<const void*>(base + off); };
  CHECK(!reg.add(P(8), 100));        // not page-aligned
  CHECK(!reg.add(P(0), 0));          // empty
  CHECK(!reg.add(nullptr, 100));
  CHECK(reg.add(P(0), 2 * pg + 100));  // pages 0..2
  CHECK(!reg.add(P(2 * pg), pg));      // shares page 2
  CHECK(!reg.add(P(pg), 10));          // inside
  CHECK(reg.add(P(3 * pg), pg));       // page 3: adjacent, no page shared
  CHECK(reg.covers(P(10), 2 * pg));
  CHECK(reg.covers(P(0), 2 * pg + 100));
  CHECK(!reg.covers(P(0), 2 * pg + 101));      // past the registered bytes
  CHECK(!reg.covers(P(2 * pg), pg + 10));      // spans two registrations
  CHECK(reg.covers(P(3 * pg + 5), pg - 5));
  CHECK(!reg.drop(P(pg)));
  CHECK(reg.drop(P(0)));
  CHECK(!reg.covers(P(10), 10));
  CHECK(reg.add(P(pg), pg));  // page 1 is free again
  CHECK(reg.drop(P(pg)) && reg.drop(P(3 * pg)) && reg.size() == 0);
  // concurrent: each thread owns its own pages, and probes the others'
  on_threads(6, [&](int t) {
    std::mt19937_64 rng(700 + t);
    for (int it = 0; it < 500; it++) {
      const uintptr_t off = ((uintptr_t)t * 1000 + rng() % 1000) * pg;
      const size_t bytes = 1 + rng() % pg;
      if (reg.add(P(off), bytes)) {
        CHECK(reg.covers(P(off), bytes));
        CHECK(!reg.add(P(off), 1));
        (void)reg.covers(P(((uintptr_t)(rng() % 6) * 1000 + rng() % 1000) * pg), 1);
        CHECK(reg.drop(P(off)));
      }
    }
  });
  CHECK(reg.size() == 0);
  std::printf("registry ok\n");
}

// ---------------- 6. scratch slot table ----------------
struct FakeRuntime {
  uint64_t clock = 0;
  struct Ev {
    const void* stream = nullptr;
    std::thread::id tid{};
    uint64_t t = 0;
    bool recorded = false;
  };
  std::vector<std::unique_ptr<Ev>> evs;
  std::set<const void*> dead;
  uint64_t last_drain = 0, drains = 0, waits_total = 0;
  std::vector<Ev> waits;  // the current acquire's waits
};
thread_local const void* t_current = nullptr;

struct FakeOps {
  FakeRuntime* rt;
  int make_fence(void** ev) {
    rt->evs.push_back(std::make_unique<FakeRuntime::Ev>());
    *ev = rt->evs.back().get();
    return 0;
  }
  void destroy_fence(void* ev) { CHECK(ev != nullptr); }
  int record(void* ev, const void* stream) {
    CHECK(stream == t_current);          // only ever on the calling stream
    CHECK(!rt->dead.count(stream));      // never on a destroyed one
    auto* e = static_cast<FakeRuntime::Ev*>(ev);
    e->stream = stream;
    e->tid = std::this_thread::get_id();
    e->t = ++rt->clock;
    e->recorded = true;
    return 0;
  }
  int wait(const void* stream, void* ev) {
    CHECK(stream == t_current);
    rt->waits.push_back(*static_cast<FakeRuntime::Ev*>(ev));
    rt->waits_total++;
    return 0;
  }
  int drain() {
    rt->last_drain = ++rt->clock;
    rt->drains++;
    return 0;
  }
};

struct Use {
  const void* owner = nullptr;
  bool per_thread = false;
  std::thread::id tid{};
  uint64_t t = 0;
};
struct Payload {
  int bytes = 0;
  Use last;  // the latest use of this slot's memory
};

void test_slots() {
  const void* const kPerThread = reinterpret_cast<const void*>(2);
  for (size_t cap : {1, 3, 4, 16}) {
    SlotTable<Payload> table(cap);
    FakeRuntime rt;
    std::mutex mu;  // the device's arena_mu
    std::atomic<uint64_t> next_stream{0x1000};
    uint64_t calls = 0, handovers_checked = 0;
    on_threads(4, [&](int t) {
      std::mt19937_64 rng(800 + t * 31 + cap);
      std::vector<const void*> mine;
      for (int it = 0; it < 2000; it++) {
        const unsigned op = (unsigned)(rng() % 100);
        if (mine.empty() || op < 8) {  // a new stream (handle values are never reused here)
          mine.push_back(reinterpret_cast<const void*>((uintptr_t)next_stream.fetch_add(0x100)));
          continue;
        }
        const bool per_thread = op < 15;
        const void* s = per_thread ? kPerThread : mine[rng() % mine.size()];
        std::lock_guard<std::mutex> lk(mu);
        t_current = s;
        FakeOps ops{&rt};
        if (!per_thread && op < 20) {  // destroyed: with or without release
          if (op < 17) {
            int freed = 0;
            CHECK(table.release(ops, s, false, [&](Slot<Payload>& sl) {
              CHECK(sl.owner == s);
              freed++;
              return 0;
            }) == 0);
            CHECK(freed <= 1);
          }
          rt.dead.insert(s);
          mine.erase(std::find(mine.begin(), mine.end(), s));
          continue;
        }
        rt.waits.clear();
        Slot<Payload>* sl = nullptr;
        CHECK(table.acquire(ops, s, per_thread, &sl) == 0 && sl);
        CHECK(sl->owner == s && sl->per_thread == per_thread && sl->tid == std::this_thread::get_id());
        CHECK(table.size() <= cap);
        const Use& prev = sl->data.last;
        const bool other = prev.owner && (prev.owner != s || prev.per_thread != per_thread ||
                                          (per_thread && prev.tid != std::this_thread::get_id()));
        if (other) {  // handed over: ordered after prev's last use
          bool ordered = rt.last_drain > prev.t;
          for (const auto& w : rt.waits)
            ordered |= w.recorded && w.stream == prev.owner && w.t > prev.t &&
                       (!prev.per_thread || w.tid == prev.tid);
          CHECK(ordered);
          handovers_checked++;
        }
        sl->data.last = Use{s, per_thread, std::this_thread::get_id(), ++rt.clock};  // the call's work
        if (rng() % 4 == 0) sl->data.bytes = std::max(sl->data.bytes, (int)(rng() % 1000));
        CHECK(table.done(ops, sl) == 0);
        CHECK(sl->state == ((per_thread || table.full()) ? SlotState::kFenced : SlotState::kOpen));
        calls++;
      }
    });
    CHECK(table.drains() == rt.drains && table.handoffs() == handovers_checked);
    FakeOps ops{&rt};
    size_t n = 0;
    table.clear(ops, [&](Slot<Payload>&) { n++; });
    CHECK(table.size() == 0);
    std::printf("slots cap %zu ok: %llu calls, %llu hand-overs checked, %llu drains, %llu fence waits\n", cap,
                (unsigned long long)calls, (unsigned long long)handovers_checked, (unsigned long long)rt.drains,
                (unsigned long long)rt.waits_total);
  }
}

int main() {
  test_workpool();
  test_walks();
  test_encode_plan();
  test_plans();
  test_registry();
  test_slots();
  std::printf("host self-test passed\n");
  return 0;
}
