"""Multi-GPU sharding of a payload batch: one process per GPU, torch.distributed over
RCCL ("nccl" backend on ROCm) or gloo (CPU tests).

The path shards trivially: payloads are independent, so each rank checksums its own contiguous block
of the batch with no data-path collective. The only exchanges are the optional ones the caller asks
for after the compute:
  * gather_digests  - the per-shard uint32 digests to one rank (4 B per payload, one RCCL gather);
  * stream_crc      - the CRC of ONE logical stream split across ranks, joined from per-rank
                      (crc, length) pairs with the GF(2) combine (8 B per rank exchanged).
"""
from __future__ import annotations

from typing import Optional, Sequence

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
