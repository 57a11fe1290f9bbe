// TEST INFRASTRUCTURE ONLY — exposes the UNMODIFIED reference checksum (compiled from
// /root/reference/include/Crc32c.h + /root/reference/src/Crc32c.cc, never copied) behind a C ABI so
// the golden-fixture generator and bench.py's cpu_baseline can call it. Built into oracle/_ref/ by
// oracle/Makefile; oracle/_ref/ is git-ignored and only exists where /root/reference was present.
#include "Crc32c.h"

#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

extern "C" {

uint32_t ref_crc32_long(const char* buf, size_t len) { return annety::Crc32c::crc32_long(buf, len); }

uint32_t ref_crc32_short(const char* buf, size_t len) { return annety::Crc32c::crc32_short(buf, len); }

void ref_crc32_update(uint32_t* crc, const char* buf, size_t len) { annety::Crc32c::crc32_update(crc, buf, len); }

void ref_tables(uint32_t* t256, uint32_t* t16) {
  for (int i = 0; i < 256; i++) t256[i] = annety::internal::crc32_table256[i];
  for (int i = 0; i < 16; i++) t16[i] = annety::internal::crc32_table16[i];
}

// The codecs pick crc32_long for payloads > 60 bytes and crc32_short otherwise
// (include/codec/LengthHeaderCodec.h:115-119); this mirrors that choice for a batch.
void ref_crc32_batch_fixed(const char* base, size_t n, size_t len, size_t stride, uint32_t* out) {
  for (size_t i = 0; i < n; i++)
    out[i] = len > 60 ? annety::Crc32c::crc32_long(base + i * stride, len)
                      : annety::Crc32c::crc32_short(base + i * stride, len);
}

struct RefJob {
  const char* base;
  size_t lo, hi, len, stride;
  uint32_t* out;
};

static void* ref_worker(void* p) {
  RefJob* j = static_cast<RefJob*>(p);
  ref_crc32_batch_fixed(j->base + j->lo * j->stride, j->hi - j->lo, j->len, j->stride, j->out + j->lo);
  return nullptr;
}

// Payload-parallel over T threads: one worker per core, like annety's one event loop per thread
// (src/EventLoopPool.cc:55-66).
int ref_crc32_batch_fixed_mt(const char* base, size_t n, size_t len, size_t stride, uint32_t* out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  RefJob jobs[256];
  for (int t = 0; t < threads; t++) {
    jobs[t] = RefJob{base, n * static_cast<size_t>(t) / threads, n * static_cast<size_t>(t + 1) / threads, len,
                     stride, out};
    if (pthread_create(&tid[t], nullptr, ref_worker, &jobs[t]) != 0) return -1;
  }
  for (int t = 0; t < threads; t++) pthread_join(tid[t], nullptr);
  return 0;
}

// Variable-length batch (BASELINE config 3): payload i = [base + off[i], + len[i]), with the codecs'
// long/short choice per payload (include/codec/LengthHeaderCodec.h:115-119).
void ref_crc32_batch_var(const char* base, const uint64_t* off, const uint32_t* len, size_t n, uint32_t* out) {
  for (size_t i = 0; i < n; i++)
    out[i] = len[i] > 60 ? annety::Crc32c::crc32_long(base + off[i], len[i])
                         : annety::Crc32c::crc32_short(base + off[i], len[i]);
}

struct RefVarJob {
  const char* base;
  const uint64_t* off;
  const uint32_t* len;
  size_t lo, hi;
  uint32_t* out;
};

static void* ref_var_worker(void* p) {
  RefVarJob* j = static_cast<RefVarJob*>(p);
  ref_crc32_batch_var(j->base, j->off + j->lo, j->len + j->lo, j->hi - j->lo, j->out + j->lo);
  return nullptr;
}

// Payload-parallel over T threads, contiguous index ranges balanced by BYTES (Zipf lengths would leave
// an index-balanced split with one long-tailed thread).
int ref_crc32_batch_var_mt(const char* base, const uint64_t* off, const uint32_t* len, size_t n, uint32_t* out,
                           int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  uint64_t total = 0;
  for (size_t i = 0; i < n; i++) total += len[i];
  pthread_t tid[256];
  RefVarJob jobs[256];
  size_t lo = 0;
  uint64_t acc = 0;
  for (int t = 0; t < threads; t++) {
    const uint64_t goal = total * static_cast<uint64_t>(t + 1) / static_cast<uint64_t>(threads);
    size_t hi = lo;
    while (hi < n && (acc < goal || t == threads - 1)) acc += len[hi++];
    jobs[t] = RefVarJob{base, off, len, lo, hi, out};
    lo = hi;
  }
  for (int t = 0; t < threads; t++)
    if (pthread_create(&tid[t], nullptr, ref_var_worker, &jobs[t]) != 0) return -1;
  for (int t = 0; t < threads; t++) pthread_join(tid[t], nullptr);
  return 0;
}

}  // extern "C"
