"""Per-call scratch across streams (crc32_capi.cpp scratch_slot: arena, sorted and split paths): each
stream keeps its own scratch slot, fenced by stream order; a ninth stream takes a slot over after a
device synchronise. Eleven streams
(more than the 8 slots) interleave arena batches of different sizes, several rounds each, and every
digest is compared with the oracle. Batches are packed Zipf-like lengths at unaligned starts, so every
call runs the line pass and the stitch (the path of BASELINE config 3)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _batch(seed: int, total: int):
    rng = np.random.default_rng(seed)
    lens = []
    s = 0
    while s < total:
        L = int(min(65536, 64 * rng.zipf(1.6) + rng.integers(0, 64)))
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
