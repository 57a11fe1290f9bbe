// Multi-GPU entry points of the C-ABI (include/annety_crc.h, "device groups"): one process drives a
// group of gfx950 devices, the way one annety process runs N event loops (src/EventLoopPool.cc:55-66)
// but with the batch sharded over GPUs instead of threads.
//
//  * annety_crc_shard_plan (host only, crc32_host.cpp): contiguous block shards, balanced to within one payload.
//  * annety_crc32_group_batch_fixed: device-resident shards; each device checksums its shard chunk by
//    chunk on its own stream, and chunk c's digests travel to the root device over RCCL (xGMI) on a
//    communication stream while chunk c+1 is computed. The communicator is ncclCommInitAll over the
//    group's devices (single process); send/recv pairs are fused in ncclGroupStart/End. The pieces and
//    their destinations come from annety_crc_group_schedule (host only, CPU-tested for 8 devices).
//    UNVERIFIED ON HARDWARE: with one device nothing is sent (the root computes in place), so the
//    send/recv branch runs only on a multi-GPU box, which the test pool does not provide.
//  * annety_crc32_group_batch_fixed_host: a host batch split over the devices, each share staged over
//    its own device's PCIe link by one host thread (annety_crc32_batch_fixed_host per device).
// Built on the single-device entry points; every call restores the caller's current device.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "annety_crc.h"

struct annety_crc_group {
  std::vector<int> dev;
  std::vector<ncclComm_t> comm;
  std::vector<hipStream_t> compute, comms;
  std::vector<hipEvent_t> ready;          // per device: chunk digests written
  std::vector<uint32_t*> scratch;         // per non-root device: its shard's digests
  std::vector<size_t> scratch_cap;
  std::mutex mu;                          // one batch at a time per group
};

namespace {

int hip_status(hipError_t e) { return e == hipSuccess ? ANNETY_CRC_OK : (e == hipErrorOutOfMemory ? ANNETY_CRC_ENOMEM : ANNETY_CRC_EHIP); }

#define GHIP(expr)                                   \
  do {                                               \
    const hipError_t e_ = (expr);                    \
    if (e_ != hipSuccess) return hip_status(e_);     \
  } while (0)
#define GNCCL(expr)                                  \
  do {                                               \
    if ((expr) != ncclSuccess) return ANNETY_CRC_ERCCL; \
  } while (0)

struct DeviceGuard {  // restores the caller's current device
  int prev = 0;
  DeviceGuard() { (void)hipGetDevice(&prev); }
  ~DeviceGuard() { (void)hipSetDevice(prev); }
};

void release(annety_crc_group* g) {
  for (size_t k = 0; k < g->dev.size(); k++) {
    (void)hipSetDevice(g->dev[k]);
    if (k < g->comm.size() && g->comm[k]) (void)ncclCommDestroy(g->comm[k]);
    if (k < g->compute.size() && g->compute[k]) {
      // the split path may hold a scratch slot keyed on this stream: drop it while the stream is alive
      (void)annety_crc_stream_release(g->compute[k]);
      (void)hipStreamDestroy(g->compute[k]);
    }
    if (k < g->comms.size() && g->comms[k]) (void)hipStreamDestroy(g->comms[k]);
    if (k < g->ready.size() && g->ready[k]) (void)hipEventDestroy(g->ready[k]);
    if (k < g->scratch.size() && g->scratch[k]) (void)hipFree(g->scratch[k]);
  }
}

}  // namespace

extern "C" {

// annety_crc_shard_plan and annety_crc_group_schedule are host-only: crc32_host.cpp.

int annety_crc_group_create(const int* devices, int ndev, annety_crc_group** out) {
  if (!devices || ndev <= 0 || !out) return ANNETY_CRC_EINVAL;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return ANNETY_CRC_ENODEV;
  for (int k = 0; k < ndev; k++) {
    if (devices[k] < 0 || devices[k] >= count) return ANNETY_CRC_ENODEV;
    for (int q = 0; q < k; q++)
      if (devices[q] == devices[k]) return ANNETY_CRC_EINVAL;  // one rank per device
  }
  DeviceGuard guard;
  for (int k = 0; k < ndev; k++) {
    const int rc = annety_crc_init(devices[k]);  // table images, gfx950 check
    if (rc) return rc;
  }
  auto* g = new annety_crc_group();
  g->dev.assign(devices, devices + ndev);
  g->comm.assign(ndev, nullptr);
  g->compute.assign(ndev, nullptr);
  g->comms.assign(ndev, nullptr);
  g->ready.assign(ndev, nullptr);
  g->scratch.assign(ndev, nullptr);
  g->scratch_cap.assign(ndev, 0);
  int rc = ANNETY_CRC_OK;
  if (ncclCommInitAll(g->comm.data(), ndev, g->dev.data()) != ncclSuccess) rc = ANNETY_CRC_ERCCL;
  for (int k = 0; k < ndev && rc == ANNETY_CRC_OK; k++) {
    hipError_t e = hipSetDevice(g->dev[k]);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->compute[k], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&g->comms[k], hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&g->ready[k], hipEventDisableTiming);
    if (e != hipSuccess) rc = hip_status(e);
  }
  if (rc != ANNETY_CRC_OK) {
    release(g);
    delete g;
    return rc;
  }
  *out = g;
  return ANNETY_CRC_OK;
}

int annety_crc_group_destroy(annety_crc_group* g) {
  if (!g) return ANNETY_CRC_OK;
  DeviceGuard guard;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    release(g);
  }
  delete g;
  return ANNETY_CRC_OK;
}

int annety_crc_group_size(const annety_crc_group* g) { return g ? (int)g->dev.size() : 0; }

int annety_crc32_group_batch_fixed(annety_crc_group* g, const void* const* d_shard, const size_t* n_shard, size_t len,
                                   size_t stride, uint32_t* d_root_out, size_t chunks) {
  if (!g || !d_shard || !n_shard || !d_root_out) return ANNETY_CRC_EINVAL;
  const int nd = (int)g->dev.size();
  size_t total = 0;
  for (int k = 0; k < nd; k++) {
    if (n_shard[k] && !d_shard[k]) return ANNETY_CRC_EINVAL;
    if (n_shard[k] > 1 && stride < len) return ANNETY_CRC_EINVAL;
    total += n_shard[k];
  }
  if (total == 0) return ANNETY_CRC_OK;
  chunks = std::max<size_t>(1, std::min(chunks, total));
  std::vector<size_t> plan(chunks * (size_t)nd * 3);
  (void)annety_crc_group_schedule(n_shard, nd, chunks, plan.data());
  std::lock_guard<std::mutex> lk(g->mu);
  DeviceGuard guard;
  // digests of device k land at d_root_out + base[k] (root) or in its scratch (others), then move to root
  for (int k = 1; k < nd; k++) {
    if (g->scratch_cap[k] < n_shard[k]) {
      GHIP(hipSetDevice(g->dev[k]));
      if (g->scratch[k]) GHIP(hipFree(g->scratch[k]));
      g->scratch[k] = nullptr;
      g->scratch_cap[k] = 0;
      GHIP(hipMalloc(reinterpret_cast<void**>(&g->scratch[k]), std::max<size_t>(n_shard[k], 1) * sizeof(uint32_t)));
      g->scratch_cap[k] = n_shard[k];
    }
  }
  // Everything is enqueued here; on any failure part of it may already be queued (kernels writing the
  // scratch, sends reading it), so every stream of the group is drained before the mutex is released and
  // the next call may reuse the scratch.
  auto enqueue = [&]() -> int {
    for (size_t c = 0; c < chunks; c++) {
      // compute piece c of every shard
      for (int k = 0; k < nd; k++) {
        const size_t* e = &plan[(c * (size_t)nd + (size_t)k) * 3];
        if (!e[1]) continue;
        GHIP(hipSetDevice(g->dev[k]));
        uint32_t* dst = k == 0 ? d_root_out + e[2] : g->scratch[k] + e[0];
        const int rc = annety_crc32_batch_fixed(static_cast<const char*>(d_shard[k]) + e[0] * stride, e[1], len, stride,
                                                dst, g->compute[k]);
        if (rc) return rc;
        if (k == 0) continue;  // the root's digests are already in place
        GHIP(hipEventRecord(g->ready[k], g->compute[k]));
        GHIP(hipStreamWaitEvent(g->comms[k], g->ready[k], 0));  // the send waits for its piece's kernel
      }
      // move piece c of every other shard to the root while piece c+1 computes: one send/recv pair per
      // device (rank k of the communicator -> rank 0), fused in one group so the root's receives from all
      // peers progress together; the root never sends to itself
      if (nd > 1) {
        GNCCL(ncclGroupStart());
        int bad = 0;
        for (int k = 1; k < nd && !bad; k++) {
          const size_t* e = &plan[(c * (size_t)nd + (size_t)k) * 3];
          if (!e[1]) continue;
          bad = ncclSend(g->scratch[k] + e[0], e[1], ncclUint32, 0, g->comm[k], g->comms[k]) != ncclSuccess ||
                ncclRecv(d_root_out + e[2], e[1], ncclUint32, k, g->comm[0], g->comms[0]) != ncclSuccess;
        }
        if (ncclGroupEnd() != ncclSuccess || bad) return ANNETY_CRC_ERCCL;
      }
    }
    return ANNETY_CRC_OK;
  };
  int rc = enqueue();
  for (int k = 0; k < nd; k++) {  // drain every stream, also after a failure
    if (hipSetDevice(g->dev[k]) != hipSuccess) {
      if (!rc) rc = ANNETY_CRC_EHIP;
      continue;
    }
    const hipError_t e1 = hipStreamSynchronize(g->compute[k]);
    const hipError_t e2 = hipStreamSynchronize(g->comms[k]);
    if (!rc && (e1 != hipSuccess || e2 != hipSuccess)) rc = hip_status(e1 != hipSuccess ? e1 : e2);
    ncclResult_t async = ncclSuccess;
    if (!rc && (ncclCommGetAsyncError(g->comm[k], &async) != ncclSuccess || async != ncclSuccess)) rc = ANNETY_CRC_ERCCL;
  }
  return rc;
}

int annety_crc32_group_batch_fixed_host(annety_crc_group* g, const void* h_base, size_t n, size_t len, size_t stride,
                                        uint32_t* h_out) {
  if (!g) return ANNETY_CRC_EINVAL;
  if (n == 0) return ANNETY_CRC_OK;
  if (!h_out || (!h_base && len > 0) || (n > 1 && stride < len)) return ANNETY_CRC_EINVAL;
  const int nd = (int)g->dev.size();
  std::vector<size_t> first(nd), count(nd);
  (void)annety_crc_shard_plan(n, nd, first.data(), count.data());
  std::atomic<int> status{ANNETY_CRC_OK};
  std::vector<std::thread> th;
  for (int k = 0; k < nd; k++) {
    if (!count[k]) continue;
    th.emplace_back([&, k] {
      // hipSetDevice is per host thread: each worker drives its own device's staging ring
      if (hipSetDevice(g->dev[k]) != hipSuccess) {
        status = ANNETY_CRC_EHIP;
        return;
      }
      const int rc = annety_crc32_batch_fixed_host(static_cast<const char*>(h_base) + first[k] * stride, count[k], len,
                                                   stride, h_out + first[k]);
      if (rc) status = rc;
    });
  }
  for (auto& t : th) t.join();
  return status.load();
}

}  // extern "C"
