"""Multi-GPU sharding of a payload batch: one process per GPU, torch.distributed over
RCCL ("nccl" backend on ROCm) or gloo (CPU tests).

The path shards trivially: payloads are independent, so each rank checksums its own contiguous block
of the batch with no data-path collective. The only exchanges are the ones the caller asks for:
  * PipelinedGather - the per-shard digests to one rank chunk by chunk, overlapped with the compute of
                      the next chunk (BASELINE config 4: 8 x 32 MiB of digests over xGMI);
  * gather_digests  - the per-shard uint32 digests to one rank (4 B per payload, one RCCL gather);
  * stream_crc      - the CRC of ONE logical stream split across ranks, joined from per-rank
                      (crc, length) pairs with the GF(2) combine (8 B per rank exchanged).
"""
from __future__ import annotations

import zlib
from typing import Callable, List, Optional, Sequence

import numpy as np
import torch
import torch.distributed as dist

from .crc32c import crc32_batch, crc32_combine


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block of payload indices [lo, hi) owned by `rank` (balanced to within one)."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return lo, hi


def crc32_batch_shard(data_local, n_local: int, length: int, stride: Optional[int] = None, out=None, stream=None):
    """Checksum this rank's shard (device-resident). Identical to crc32_batch; named for symmetry."""
    return crc32_batch(data_local, n_local, length, stride, out, stream)


def gather_digests(local: torch.Tensor, counts: Sequence[int], dst: int = 0, group=None) -> Optional[torch.Tensor]:
    """Gather every rank's digests (int32 tensor, `counts[r]` entries on rank r) to `dst` in rank order.
    Shards may differ in size by one payload; they are padded to the largest for the collective."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if len(counts) != world or local.numel() != counts[rank]:
        raise ValueError("counts must list every rank's shard size")
    m = max(counts)
    buf = local
    if local.numel() < m:
        buf = torch.zeros(m, dtype=local.dtype, device=local.device)
        buf[: local.numel()] = local
    parts = [torch.empty(m, dtype=local.dtype, device=local.device) for _ in range(world)] if rank == dst else None
    dist.gather(buf, parts, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([p[:c] for p, c in zip(parts, counts)])


def chunk_bounds(n: int, chunks: int, taper: int = 0) -> List[tuple]:
    """[lo, hi) of `chunks` near-equal consecutive pieces of n payloads (empty pieces dropped). With
    `taper` t > 0 the last piece is cut again into t pieces of 1/2, 1/4, ..., 1/2^(t-1), 1/2^(t-1) of it:
    in a pipelined gather only the last piece's transfer is not hidden behind compute."""
    chunks = max(1, min(chunks, n)) if n else 1
    b = [(n * k // chunks, n * (k + 1) // chunks) for k in range(chunks) if n * (k + 1) // chunks > n * k // chunks]
    if taper > 1 and b:
        lo, hi = b.pop()
        for _ in range(taper - 1):
            if hi - lo < 2:
                break
            mid = hi - (hi - lo) // 2
            b.append((lo, mid))
            lo = mid
        b.append((lo, hi))
    return b


class PipelinedGather:
    """the shard is checksummed chunk by chunk, and chunk k's digests travel to `dst`
    (RCCL gather over xGMI on a GPU run) while chunk k+1 is computed. Every rank holds `n_local`
    payloads; on `dst` the result is `recv[r]` = rank r's digests.

    torch.distributed issues each collective on its communication stream after the work already queued
    on the current stream, so `produce` (a kernel launch) and the gathers overlap with no extra sync."""

    def __init__(self, n_local: int, chunks: int, dst: int = 0, group=None, device=None, dtype=torch.int32,
                 taper: int = 0, buffers: int = 1):
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.dst, self.group = dst, group
        self.bounds = chunk_bounds(n_local, chunks, taper)
        # one receive buffer per digest buffer (run_steps): gathers in flight together never share one, so
        # the result does not depend on the backend running them in order (gloo runs them on a thread pool)
        self.buffers = max(1, buffers)
        self.recvs = ([torch.empty((self.world, n_local), dtype=dtype, device=device) for _ in range(self.buffers)]
                      if self.rank == dst else None)
        self.last = 0  # the receive buffer of the latest step

    @property
    def recv(self) -> Optional[torch.Tensor]:
        """On `dst`: recv[r] = rank r's digests of the latest step; None elsewhere."""
        return self.recvs[self.last] if self.recvs is not None else None

    def run(self, produce: Callable[[int, int], torch.Tensor], gather: bool = True, buf: int = 0):
        """produce(lo, hi) -> this rank's digests of payloads [lo, hi) (a view of its output). Returns
        the list of async work handles (empty when gather is False); call wait() on them."""
        handles = []
        self.last = buf % (len(self.recvs) if self.recvs is not None else 1)
        for lo, hi in self.bounds:
            out = produce(lo, hi)
            if gather:
                parts = [self.recv[r, lo:hi] for r in range(self.world)] if self.rank == self.dst else None
                handles.append(dist.gather(out, parts, dst=self.dst, group=self.group, async_op=True))
        return handles

    @staticmethod
    def wait(handles) -> None:
        for h in handles:
            h.wait()

    def run_steps(self, produce: Callable[[int, int, int], torch.Tensor], steps: int, buffers: Optional[int] = None,
                  gather: bool = True) -> None:
        """`steps` consecutive steps; produce(s, lo, hi) writes step s's digests of [lo, hi) into buffer
        s % buffers and returns that view. Step s's handles are waited (on a GPU: the compute stream waits
        for step s's gathers, no host block) only after step s + buffers - 1 is launched, just before step
        s + buffers reuses the buffer: with two buffers step s+1 computes while step s's last gathers still
        read the other one. Everything is waited before returning. `buffers` defaults to the receive buffers
        allocated at construction; more would put two steps' gathers in flight into one receive buffer."""
        from collections import deque

        buffers = self.buffers if buffers is None else max(1, buffers)
        if buffers > self.buffers:
            raise ValueError(f"run_steps with {buffers} buffers, but the gather was built with {self.buffers} "
                             "receive buffers (PipelinedGather(buffers=...))")
        pending = deque()
        for s in range(steps):
            pending.append(self.run(lambda lo, hi, s=s: produce(s, lo, hi), gather=gather, buf=s % buffers))
            if len(pending) >= buffers:  # step s+1 reuses the buffer of step s+1-buffers
                self.wait(pending.popleft())
        while pending:
            self.wait(pending.popleft())


def digest_checksum(t: torch.Tensor) -> int:
    """CRC-32 of a digest array's bytes (a checksum of checksums, computed on the host)."""
    return zlib.crc32(np.ascontiguousarray(t.detach().cpu().numpy()).tobytes())


def verify_gather(recv: Optional[torch.Tensor], local: torch.Tensor, group=None, dst: int = 0) -> bool:
    """Every rank sends the checksum of its own digests; `dst` checks each received row against it.
    Returns the verdict on every rank (broadcast), True on success."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = local.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    mine = torch.tensor([digest_checksum(local)], dtype=torch.int64, device=dev)
    allv = [torch.empty(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(allv, mine, group=group)
    ok = torch.ones(1, dtype=torch.int64, device=dev)
    if rank == dst:
        good = all(digest_checksum(recv[r]) == int(allv[r].item()) for r in range(world))
        ok.fill_(1 if good else 0)
    dist.broadcast(ok, src=dst, group=group)
    return bool(ok.item())


def stream_crc(local_crc: int, local_len: int, group=None, device=None) -> int:
    """CRC of the concatenation of every rank's slice (rank order) from per-rank (crc, len).
    All ranks return the joined value; 16 bytes per rank cross the fabric."""
    world = dist.get_world_size(group)
    dev = device if device is not None else torch.device("cpu")
    mine = torch.tensor([local_crc & 0xFFFFFFFF, local_len], dtype=torch.int64, device=dev)
    allv = [torch.empty(2, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(allv, mine, group=group)
    crc = 0
    for i, v in enumerate(allv):
        c, ln = int(v[0]), int(v[1])
        crc = c if i == 0 else crc32_combine(crc, c, ln)
    return crc


# ---- single-process device groups over the C-ABI (annety_crc_group_*, RCCL ncclCommInitAll) ----
def shard_plan(n: int, nshards: int) -> list:
    """annety_crc_shard_plan: [(first, count)] of n payloads over nshards (the C-ABI's own arithmetic)."""
    import ctypes

    from . import _lib

    first = (ctypes.c_size_t * nshards)()
    count = (ctypes.c_size_t * nshards)()
    _lib.check(_lib.get().annety_crc_shard_plan(n, nshards, first, count), "annety_crc_shard_plan")
    return [(int(first[k]), int(count[k])) for k in range(nshards)]


def group_schedule(n_shard, chunks: int) -> list:
    """annety_crc_group_schedule: for piece c of shard k, plan[c][k] = (first payload within the shard,
    payload count, index of its first digest in the root's output) - what annety_crc32_group_batch_fixed
    computes and sends."""
    import ctypes

    from . import _lib

    nd = len(n_shard)
    ns = (ctypes.c_size_t * nd)(*n_shard)
    plan = (ctypes.c_size_t * (chunks * nd * 3))()
    _lib.check(_lib.get().annety_crc_group_schedule(ns, nd, chunks, plan), "annety_crc_group_schedule")
    return [[tuple(int(plan[(c * nd + k) * 3 + i]) for i in range(3)) for k in range(nd)] for c in range(chunks)]


class DeviceGroup:
    """One process driving several devices (annety_crc_group): device-resident shards with the digests
    gathered to devices[0] over RCCL, or a host batch staged over every device's PCIe link."""

    def __init__(self, devices):
        import ctypes

        from . import _lib

        self.devices = list(devices)
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        _lib.check(_lib.get().annety_crc_group_create(arr, len(self.devices), ctypes.byref(h)),
                   "annety_crc_group_create")
        self._h = h

    def close(self):
        from . import _lib

        if self._h:
            _lib.get().annety_crc_group_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def batch_fixed(self, shards, length: int, stride: int | None = None, chunks: int = 8, out=None):
        """shards[k]: uint8 tensor on devices[k] holding a whole number of payloads. Returns the int32
        digests of all shards in order, on devices[0]."""
        import ctypes

        from . import _lib

        stride = length if stride is None else stride
        if len(shards) != len(self.devices):
            raise ValueError("one shard per device")
        counts = [(s.numel() - length) // stride + 1 if s.numel() >= length else 0 for s in shards]
        for s, d in zip(shards, self.devices):
            if s.device != torch.device("cuda", d):
                raise ValueError(f"shard on {s.device}, expected cuda:{d}")
        total = sum(counts)
        if out is None:
            out = torch.empty(total, dtype=torch.int32, device=torch.device("cuda", self.devices[0]))
        ptrs = (ctypes.c_void_p * len(shards))(*[s.data_ptr() for s in shards])
        ns = (ctypes.c_size_t * len(shards))(*counts)
        for d in self.devices:  # the group's streams run after the work already queued on torch's
            torch.cuda.synchronize(d)
        _lib.check(_lib.get().annety_crc32_group_batch_fixed(self._h, ptrs, ns, length, stride, out.data_ptr(), chunks),
                   "annety_crc32_group_batch_fixed")
        return out

    def batch_fixed_host(self, buf, n: int, length: int, stride: int | None = None) -> np.ndarray:
        from . import _lib
        from .crc32c import _host_view

        stride = length if stride is None else stride
        addr, size, keep = _host_view(buf)
        if n > 0 and (n - 1) * stride + length > size:
            raise ValueError("batch extends past the end of `buf`")
        out = np.zeros(n, dtype=np.uint32)
        _lib.check(_lib.get().annety_crc32_group_batch_fixed_host(self._h, addr, n, length, stride, out.ctypes.data),
                   "annety_crc32_group_batch_fixed_host")
        return out
