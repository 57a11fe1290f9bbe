"""Per-call scratch across streams (crc32_host.h SlotTable: arena, sorted and split paths): each stream
keeps its own scratch slot, fenced by stream order; past the slot cap (ANNETY_CRC_STREAM_SLOTS, default 64)
the least recently used slot is handed over - by the event its last call recorded on its own stream while
the table was full, or after one device-wide synchronise for a slot last used before the table filled up
(annety_crc_scratch_stats counts both). No event is ever recorded on a stream other than the caller's, so
streams destroyed without annety_crc_stream_release are harmless. Streams interleave arena batches of
different sizes, several rounds each, and every digest is compared with the oracle. Batches are packed
Zipf-like lengths at unaligned starts, so every call runs the line pass and the stitch (the path of
BASELINE config 3). hipStreamPerThread, one handle naming a different stream per thread, gets a slot
per calling thread."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _batch(seed: int, total: int):
    rng = np.random.default_rng(seed)
    lens = []
    s = 0
    while s < total:
        L = int(min(65536, 64 * min(int(rng.zipf(1.6)), 1 << 20) + rng.integers(0, 64)))
        lens.append(L)
        s += L
    lens = np.array(lens, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    data = rng.integers(0, 256, int(offs[-1] + lens[-1]), dtype=np.uint8)
    return data, offs, lens


def test_arena_more_streams_than_slots(gpu):
    import torch

    import annety_amd

    nstreams, rounds = 11, 3
    streams = [torch.cuda.Stream(gpu) for _ in range(nstreams)]
    jobs = []
    for i in range(nstreams):
        data, offs, lens = _batch(1000 + i, (1 << 20) * (1 + i % 4) + 12345 * i)  # different sizes: slots grow
        want = oracle.batch_var(data, offs.astype(np.uint64), lens.astype(np.uint32))
        d = torch.from_numpy(data).to(gpu)
        o = torch.from_numpy(offs).to(gpu)
        ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
        outs = [torch.empty(len(lens), dtype=torch.int32, device=gpu) for _ in range(rounds)]
        jobs.append((d, o, ln, outs, want, len(data)))
    torch.cuda.synchronize()
    for r in range(rounds):
        for i, (d, o, ln, outs, want, nbytes) in enumerate(jobs):
            with torch.cuda.stream(streams[i]):
                for t in (d, o, ln, outs[r]):
                    t.record_stream(streams[i])
                annety_amd.crc32_batch_var(d, o, ln, out=outs[r], stream=streams[i], arena=nbytes)
    torch.cuda.synchronize()
    for i, (d, o, ln, outs, want, nbytes) in enumerate(jobs):
        for r in range(rounds):
            got = outs[r].cpu().numpy().view(np.uint32)
            assert np.array_equal(got, want), f"stream {i} round {r}: {int((got != want).sum())} digests differ"


def test_sorted_and_split_paths_across_streams(gpu):
    """The sorted variable path and the long-payload split path draw their scratch from the same
    per-stream slots: eleven streams alternate between the two, three rounds, every digest checked."""
    import torch

    import annety_amd

    nstreams, rounds = 11, 3
    streams = [torch.cuda.Stream(gpu) for _ in range(nstreams)]
    jobs = []
    for i in range(nstreams):
        if i % 2 == 0:  # sorted path: payloads scattered in a larger buffer
            data, offs, lens = _batch(2000 + i, (1 << 19) * (1 + i % 3))
            offs = offs + np.arange(len(offs), dtype=np.int64) * 8  # gaps between payloads
            buf = np.random.default_rng(i).integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
            want = oracle.batch_var(buf, offs.astype(np.uint64), lens.astype(np.uint32))
            args = (torch.from_numpy(buf).to(gpu), torch.from_numpy(offs).to(gpu),
                    torch.from_numpy(lens.astype(np.int32)).to(gpu))
            jobs.append(("var", args, len(lens), want))
        else:  # split path: a few long payloads (fewer than two per lane group)
            n, L = 3, (1 << 20) * (1 + i % 3) + 4096
            buf = np.random.default_rng(i).integers(0, 256, n * L, dtype=np.uint8)
            want = oracle.batch_fixed(buf, n, L)
            jobs.append(("fixed", (torch.from_numpy(buf).to(gpu), n, L), n, want))
    outs = [[torch.empty(j[2], dtype=torch.int32, device=gpu) for _ in range(rounds)] for j in jobs]
    torch.cuda.synchronize()
    for r in range(rounds):
        for i, (kind, args, n, want) in enumerate(jobs):
            with torch.cuda.stream(streams[i]):
                if kind == "var":
                    for t in list(args) + [outs[i][r]]:
                        t.record_stream(streams[i])
                    annety_amd.crc32_batch_var(*args, out=outs[i][r], stream=streams[i])
                else:
                    args[0].record_stream(streams[i])
                    outs[i][r].record_stream(streams[i])
                    annety_amd.crc32_batch(args[0], args[1], args[2], out=outs[i][r], stream=streams[i])
    torch.cuda.synchronize()
    for i, (kind, args, n, want) in enumerate(jobs):
        for r in range(rounds):
            got = outs[i][r].cpu().numpy().view(np.uint32)
            assert np.array_equal(got, want), f"{kind} stream {i} round {r}: {int((got != want).sum())} differ"


def _arena_job(gpu, seed, total):
    import torch

    data, offs, lens = _batch(seed, total)
    want = oracle.batch_var(data, offs.astype(np.uint64), lens.astype(np.uint32))
    return (torch.from_numpy(data).to(gpu), torch.from_numpy(offs).to(gpu),
            torch.from_numpy(lens.astype(np.int32)).to(gpu), want, len(data))


def test_sixteen_streams_in_rotation_no_device_sync(gpu):
    """16 streams in rotation (annety's >8 IO loops on one device): each keeps its own slot, no slot is
    handed over and no device-wide synchronise happens; per-call cost is timed against one stream."""
    import time

    import torch

    import annety_amd

    before = annety_amd.scratch_stats(0)
    streams = [torch.cuda.Stream(gpu) for _ in range(16)]
    d, o, ln, want, nbytes = _arena_job(gpu, 4242, 1 << 20)
    outs = [torch.empty(ln.numel(), dtype=torch.int32, device=gpu) for _ in streams]
    torch.cuda.synchronize()

    def rotate(ss, rounds):
        for _ in range(rounds):
            for i, st in enumerate(ss):
                annety_amd.crc32_batch_var(d, o, ln, out=outs[i], stream=st, arena=nbytes)
        torch.cuda.synchronize()

    rotate(streams, 2)  # every stream takes its slot
    for i in range(16):
        assert np.array_equal(outs[i].cpu().numpy().view(np.uint32), want), i
    after = annety_amd.scratch_stats(0)
    assert after["device_syncs"] == before["device_syncs"] == 0
    assert after["handoffs"] == before["handoffs"]
    assert after["slots"] >= 16
    # per-call time: the 16 streams in rotation against the same calls on one stream
    t0 = time.perf_counter()
    rotate(streams, 8)
    t16 = (time.perf_counter() - t0) / 128
    t0 = time.perf_counter()
    rotate([streams[0]] * 16, 8)
    t1 = (time.perf_counter() - t0) / 128
    print(f"per call: 16 streams {t16 * 1e6:.1f} us, 1 stream {t1 * 1e6:.1f} us")
    assert t16 < 3 * t1 + 100e-6
    assert annety_amd.scratch_stats(0)["device_syncs"] == 0
    for st in streams:
        annety_amd.stream_release(st)
    assert annety_amd.scratch_stats(0)["slots"] == after["slots"] - 16


HANDOFF_SCRIPT = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, {root!r})
sys.path.insert(0, {tests!r})
import annety_amd
import test_gpu_arena_streams as t
gpu = torch.device("cuda", 0)
streams = [torch.cuda.Stream(gpu) for _ in range(11)]
jobs = [t._arena_job(gpu, 500 + i, (1 << 19) * (1 + i % 3) + 777 * i) for i in range(11)]
outs = [[torch.empty(j[2].numel(), dtype=torch.int32, device=gpu) for _ in range(3)] for j in jobs]
torch.cuda.synchronize()
for r in range(3):
    for i, (d, o, ln, want, nb) in enumerate(jobs):
        with torch.cuda.stream(streams[i]):
            for x in (d, o, ln, outs[i][r]):
                x.record_stream(streams[i])
            annety_amd.crc32_batch_var(d, o, ln, out=outs[i][r], stream=streams[i], arena=nb)
torch.cuda.synchronize()
bad = sum(int((outs[i][r].cpu().numpy().view(np.uint32) != jobs[i][3]).sum()) for i in range(11) for r in range(3))
s = annety_amd.scratch_stats(0)
print("RESULT", bad, s["slots"], s["handoffs"], s["device_syncs"])
"""


def test_slot_handoff_past_the_cap(gpu, tmp_path):
    """With the cap at 4 slots, 11 streams x 3 rounds take slots over from each other: every digest is
    right, hand-overs happen, and only the first one (of a slot last used before the table was full)
    synchronises the device."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    script = tmp_path / "handoff.py"
    script.write_text(HANDOFF_SCRIPT.format(root=os.path.dirname(here), tests=here))
    env = dict(os.environ, ANNETY_CRC_STREAM_SLOTS="4")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    bad, slots, handoffs, syncs = map(int, [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")][0].split()[1:])
    assert bad == 0 and slots == 4 and handoffs > 0 and syncs == 1


DEAD_STREAMS_SCRIPT = r"""
import ctypes
import sys
import numpy as np
import torch
sys.path.insert(0, {root!r})
sys.path.insert(0, {tests!r})
import annety_amd
import oracle
import test_gpu_arena_streams as t
from annety_amd import sharded
hip = ctypes.CDLL("libamdhip64.so")
gpu = torch.device("cuda", 0)
d, o, ln, want, nb = t._arena_job(gpu, 77, (1 << 20) + 4321)
n, L = 3, (1 << 20) + 4096  # a few long payloads: the split path (a scratch slot too)
lb = np.random.default_rng(5).integers(0, 256, n * L, dtype=np.uint8)
lwant = oracle.batch_fixed(lb, n, L)
ld = torch.from_numpy(lb).to(gpu)
torch.cuda.synchronize()
bad = 0
# 12 raw HIP streams alive at once (distinct handles), each used by the arena and the split path, then all
# destroyed WITHOUT annety_crc_stream_release: the slot table (cap 4) hands slots over among them and must
# never touch a dead handle afterwards
raw = []
for i in range(12):
    s = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(s)) == 0
    raw.append(s)
for rnd in range(2):
    for s in raw:
        out = torch.empty(ln.numel(), dtype=torch.int32, device=gpu)
        lout = torch.empty(n, dtype=torch.int32, device=gpu)
        annety_amd.crc32_batch_var(d, o, ln, out=out, stream=s.value, arena=nb)
        annety_amd.crc32_batch(ld, n, L, out=lout, stream=s.value)
        assert hip.hipStreamSynchronize(s) == 0
        bad += int((out.cpu().numpy().view(np.uint32) != want).sum()) + int((lout.cpu().numpy().view(np.uint32) != lwant).sum())
for s in raw:
    assert hip.hipStreamDestroy(s) == 0
# new streams after the old ones died (HIP may hand out the dead handles' values again: hipStreamDestroy has
# finished their work, so a reused value takes its slot over in stream order)
for i in range(6):
    s = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(s)) == 0
    out = torch.empty(ln.numel(), dtype=torch.int32, device=gpu)
    annety_amd.crc32_batch_var(d, o, ln, out=out, stream=s.value, arena=nb)
    assert hip.hipStreamSynchronize(s) == 0
    bad += int((out.cpu().numpy().view(np.uint32) != want).sum())
    assert hip.hipStreamDestroy(s) == 0
# device groups created and destroyed past the cap (their compute streams run the split path)
for i in range(6):
    with sharded.DeviceGroup([0]) as g:
        out = g.batch_fixed([ld], L, chunks=1)
        torch.cuda.synchronize()
        bad += int((out.cpu().numpy().view(np.uint32) != lwant).sum())
# then a call on a fresh stream
s2 = torch.cuda.Stream(gpu)
out = torch.empty(ln.numel(), dtype=torch.int32, device=gpu)
annety_amd.crc32_batch_var(d, o, ln, out=out, stream=s2, arena=nb)
torch.cuda.synchronize()
bad += int((out.cpu().numpy().view(np.uint32) != want).sum())
st = annety_amd.scratch_stats(0)
print("RESULT", bad, st["slots"], st["handoffs"], st["device_syncs"])
"""


def test_destroyed_streams_past_the_cap(gpu, tmp_path):
    """Streams destroyed without annety_crc_stream_release, more of them than slots (cap 4), and device
    groups created and destroyed past the cap: every digest is right, the process ends cleanly (no event
    recorded on a dead stream), the groups released their streams' slots (the table stays at the cap), and
    the dead streams' slots are taken over with at most one device synchronise per table fill."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    script = tmp_path / "dead_streams.py"
    script.write_text(DEAD_STREAMS_SCRIPT.format(root=os.path.dirname(here), tests=here))
    env = dict(os.environ, ANNETY_CRC_STREAM_SLOTS="4")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    bad, slots, handoffs, syncs = map(int, [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT")][0].split()[1:])
    assert bad == 0 and slots <= 4 and handoffs > 0 and syncs <= 2


def test_per_thread_stream_handle_two_threads(gpu):
    """Two host threads pass the same hipStreamPerThread handle (2), which HIP resolves to each thread's
    own stream: they get separate scratch slots, so their line passes and stitches cannot overwrite each
    other's S/SB; every digest of every call is checked."""
    import threading

    import torch

    import annety_amd

    PER_THREAD = 2  # hipStreamPerThread
    jobs = [_arena_job(gpu, 900 + k, (1 << 20) + 999 * k) for k in range(2)]
    torch.cuda.synchronize()
    errors = []

    def worker(k):
        try:
            torch.cuda.set_device(gpu)
            d, o, ln, want, nb = jobs[k]
            for r in range(20):
                out = torch.empty(ln.numel(), dtype=torch.int32, device=gpu)
                annety_amd.crc32_batch_var(d, o, ln, out=out, stream=PER_THREAD, arena=nb)
                torch.cuda.synchronize()  # the per-thread stream is not torch's; wait for the device
                got = out.cpu().numpy().view(np.uint32)
                if not np.array_equal(got, want):
                    errors.append((k, r, int((got != want).sum())))
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(100)
    assert not errors, errors
    assert annety_amd.scratch_stats(0)["device_syncs"] == 0
