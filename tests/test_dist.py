"""Multi-process (world_size 2, gloo on CPU) coverage of the sharding path bench.py runs at N > 1:
shard ranges, the chunked digest gather to rank 0 (sharded.PipelinedGather, async collectives),
the checksum-of-checksums verification, the one-shot gather and the combine-joined stream CRC, and
bench.py's own rank spawner. The per-shard compute is the GPU kernel on a real run; here each rank
uses the CPU oracle as the stand-in producer of its chunk's digests, so these tests check the
distributed plumbing, not the kernel (the kernel's parity is tests/test_gpu_*.py)."""
import os
import socket
import subprocess
import time
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


def _pipe_worker(rank, world, port, n_local, L, chunks, q, corrupt):
    """bench.py's N > 1 step: each rank produces its shard's digests chunk by chunk; every chunk is
    gathered to rank 0 asynchronously while the next one is produced; then verify_gather."""
    import torch.distributed as dist

    from annety_amd import sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        arena = oracle.lcg_bytes(n_local * L, 1000 + rank)  # each rank's own shard (weak scaling)
        out = torch.zeros(n_local, dtype=torch.int32)
        pipe = sharded.PipelinedGather(n_local, chunks, dst=0)

        def produce(lo, hi):
            d = oracle.batch_fixed(arena[lo * L:hi * L], hi - lo, L)
            out[lo:hi] = torch.from_numpy(d.view(np.int32).copy())
            return out[lo:hi]

        handles = pipe.run(produce)
        sharded.PipelinedGather.wait(handles)
        if corrupt and rank == 0:
            pipe.recv[1, 3] ^= 1
        ok = sharded.verify_gather(pipe.recv, out)
        q.put(("ok", rank, ok, len(pipe.bounds)))
        if rank == 0:
            q.put(("recv", pipe.recv.numpy().view(np.uint32).tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("corrupt", [False, True])
def test_gloo_world2_pipelined_gather(corrupt):
    n_local, L, chunks = 1000, 128, 7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, 2, port, n_local, L, chunks, q, corrupt)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    msgs = [q.get(timeout=5) for _ in range(3)]
    oks = [m for m in msgs if m[0] == "ok"]
    assert all(m[2] == (not corrupt) for m in oks) and all(m[3] == chunks for m in oks)
    recv = [m for m in msgs if m[0] == "recv"][0][1]
    for r in range(2):
        want = oracle.batch_fixed(oracle.lcg_bytes(n_local * L, 1000 + r), n_local, L).tolist()
        if corrupt and r == 1:
            want[3] ^= 1
        assert recv[r] == want


def _steps_worker(rank, world, port, n_local, L, chunks, steps, buffers, q):
    """bench.py's timed loop at N > 1 (PipelinedGather.run_steps): every step's digests differ (a
    different shard per step), written into buffer s % buffers; rank 0 logs what it received after each
    step's gathers are waited, which with two buffers is one step later."""
    import torch.distributed as dist

    from annety_amd import sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        outs = [torch.zeros(n_local, dtype=torch.int32) for _ in range(buffers)]
        pipe = sharded.PipelinedGather(n_local, chunks, dst=0, buffers=buffers)

        def produce(s, lo, hi):
            arena = oracle.lcg_bytes(n_local * L, 100 * s + rank)
            out = outs[s % buffers]
            out[lo:hi] = torch.from_numpy(oracle.batch_fixed(arena[lo * L:hi * L], hi - lo, L).view(np.int32).copy())
            return out[lo:hi]

        pipe.run_steps(produce, steps)  # defaults to the receive buffers built (never more)
        if rank == 0:
            q.put(("recv", pipe.recv.numpy().view(np.uint32).tolist()))
        try:  # more digest buffers than receive buffers would share one receive buffer between steps
            pipe.run_steps(produce, 1, buffers=buffers + 1)
            q.put(("raise", rank, False))
        except ValueError:
            q.put(("raise", rank, True))
        # every buffer still holds its last step's digests (no step overwrote a buffer under a gather)
        for b in range(buffers):
            s = max(x for x in range(steps) if x % buffers == b)
            want = oracle.batch_fixed(oracle.lcg_bytes(n_local * L, 100 * s + rank), n_local, L)
            q.put(("buf", rank, b, bool(np.array_equal(outs[b].numpy().view(np.uint32), want))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("buffers", [1, 2, 3])
def test_gloo_world2_run_steps(buffers):
    n_local, L, chunks, steps = 600, 128, 3, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_steps_worker, args=(r, 2, port, n_local, L, chunks, steps, buffers, q))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    msgs = [q.get(timeout=5) for _ in range(3 + 2 * buffers)]
    assert all(m[3] for m in msgs if m[0] == "buf")
    assert [m[2] for m in msgs if m[0] == "raise"] == [True, True]
    recv = [m for m in msgs if m[0] == "recv"][0][1]
    for r in range(2):  # rank 0 ends holding the last step's digests of every rank
        want = oracle.batch_fixed(oracle.lcg_bytes(n_local * L, 100 * (steps - 1) + r), n_local, L).tolist()
        assert recv[r] == want


def test_bench_spawns_ranks(tmp_path):
    """bench.py --gpus N without a launcher starts N ranks with the torchrun environment."""
    sys.path.insert(0, ROOT)
    import bench

    script = tmp_path / "rank.py"
    script.write_text("import os\nprint(os.environ['RANK'], os.environ['LOCAL_RANK'], os.environ['WORLD_SIZE'], "
                      "os.environ['MASTER_ADDR'])\n")
    out = subprocess.run([sys.executable, "-c", f"import sys; sys.path.insert(0, {ROOT!r}); import bench; "
                          f"sys.exit(bench.spawn(3, [{str(script)!r}]))"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0
    assert out.stdout.split() == ["0", "0", "3", "127.0.0.1"]  # rank 0's stdout only
    assert bench.spawn(2, ["-c", "import sys; sys.exit(3)"]) == 3
    # a rank that dies ends the run: the survivor (blocked as in a collective) is terminated
    t0 = time.time()
    rc = bench.spawn(2, ["-c", "import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(5)\ntime.sleep(600)"])
    assert rc != 0 and time.time() - t0 < 60


def test_shard_range_covers():
    from annety_amd import sharded

    for n in [0, 1, 7, 1 << 20, (64 << 20)]:
        for w in [1, 2, 3, 8]:
            rs = [sharded.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1
    assert sharded.chunk_bounds(10, 3) == [(0, 3), (3, 6), (6, 10)]
    assert sharded.chunk_bounds(2, 8) == [(0, 1), (1, 2)]
    # tapered tail: the last of 8 pieces cut into 1/2, 1/4, 1/4
    b = sharded.chunk_bounds(8192, 8, taper=3)
    assert b[:7] == [(1024 * k, 1024 * (k + 1)) for k in range(7)]
    assert b[7:] == [(7168, 7680), (7680, 7936), (7936, 8192)]
    for n, c, t in [(1, 8, 3), (5, 2, 4), (1000, 7, 3), (10 ** 6 + 3, 8, 5)]:
        b = sharded.chunk_bounds(n, c, taper=t)
        assert b[0][0] == 0 and b[-1][1] == n and all(lo < hi for lo, hi in b)
        assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
