"""Multi-process (world_size 2, gloo on CPU) coverage of the sharding path: shard ranges, the digest
gather to rank 0 and the combine-joined stream CRC. The per-shard compute is the GPU kernel on a
real run; here each rank uses the CPU oracle as the stand-in producer of its shard's digests, so the
test checks the distributed plumbing, not the kernel."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, L, q):
    import torch.distributed as dist

    from annety_amd import sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        arena = oracle.lcg_bytes(n * L, 4242)
        lo, hi = sharded.shard_range(n, rank, world)
        local = oracle.batch_fixed(arena[lo * L:hi * L], hi - lo, L)
        counts = [sharded.shard_range(n, r, world)[1] - sharded.shard_range(n, r, world)[0] for r in range(world)]
        got = sharded.gather_digests(torch.from_numpy(local.view(np.int32).copy()), counts, dst=0)
        # one logical stream = the whole arena, split at the shard boundary
        part = arena[lo * L:hi * L]
        joined = sharded.stream_crc(oracle.crc32_long(part), part.size)
        if rank == 0:
            q.put(("digests", got.numpy().view(np.uint32).tolist()))
        q.put(("stream", rank, joined))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [1000, 1001])
def test_gloo_world2_shard_gather_and_stream(n):
    L = 256
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, L, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    msgs = [q.get(timeout=5) for _ in range(3)]
    arena = oracle.lcg_bytes(n * L, 4242)
    want = oracle.batch_fixed(arena, n, L).tolist()
    dig = [m for m in msgs if m[0] == "digests"][0][1]
    assert dig == want
    full = oracle.crc32_long(arena)
    streams = [m for m in msgs if m[0] == "stream"]
    assert len(streams) == 2 and all(s[2] == full for s in streams)


def test_shard_range_covers():
    from annety_amd import sharded

    for n in [0, 1, 7, 1 << 20, (64 << 20)]:
        for w in [1, 2, 3, 8]:
            rs = [sharded.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1
