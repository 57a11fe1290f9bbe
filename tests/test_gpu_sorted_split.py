"""Long payloads on the length-sorted path (crc32_kernels.h kSplitSeg): a payload of more than 128 KiB runs as
end-aligned 16 KiB segments (1 MiB past 256 MiB; the first takes the remainder), each a task of the sorted list,
whose group xors shift_{m seg}(its raw register) into the payload's digest. Digests against the oracle at the
edges: lengths just above the split threshold (a first segment of 1 byte), whole multiples of the segment, every
start offset class, payloads of several MiB and one past 256 MiB, long payloads mixed with many short ones, update
mode (the register moved aside for the first segment, the segments' xor as the new register), and the descriptor
cap (annety_crc_set_split_cap): payloads past it run whole, before and after it split."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

SEG = 16384
MIN = 131072  # kSplitMin


def _run(gpu, lens, seed, path="sorted", gap=9000):
    import torch

    import annety_amd

    rng = np.random.default_rng(seed)
    lens = np.asarray(lens, dtype=np.int64)
    starts = rng.integers(0, 128, lens.size)
    offs = np.concatenate([[0], np.cumsum(lens + gap)[:-1]]).astype(np.int64) + starts
    data = oracle.lcg_bytes(int(offs[-1] + lens[-1]) + 256, seed)
    d = torch.from_numpy(data.copy()).to(gpu)
    o = torch.from_numpy(offs).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    out = torch.full((lens.size,), 7, dtype=torch.int32, device=gpu)
    annety_amd.set_var_path(path)
    try:
        annety_amd.crc32_batch_var(d, o, ln, out=out)
        torch.cuda.synchronize()
    finally:
        annety_amd.set_var_path("auto")
    want = oracle.batch_var_mt(data, offs.astype(np.uint64), lens.astype(np.uint32), threads=8)
    got = out.cpu().numpy().view(np.uint32)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (bad[:8], lens[bad[:8]])
    return annety_amd.last_kernels()


def test_split_edges(gpu):
    lens = [MIN + 1, MIN, MIN + 15, MIN + SEG, MIN + SEG + 16, 12 * SEG - 1, 13 * SEG + 129, 200000,
            (1 << 20) + 3, 3 * (1 << 20) + 13, 4096, 1, 0, 127, 128, 129, SEG, 65536]
    kernels = _run(gpu, lens, 1)
    assert "crc32_var_sorted_kernel" in kernels


def test_split_many_long_among_short(gpu):
    rng = np.random.default_rng(2)
    lens = np.concatenate([rng.integers(0, 5000, 3000), rng.integers(MIN + 1, 50 * SEG, 60),
                           np.full(4, 16 << 20)])
    _run(gpu, rng.permutation(lens), 3)


def test_split_every_remainder_and_alignment(gpu):
    # the first segment's length runs through 1..128 and every start offset class of a line
    lens = [MIN + r for r in range(1, 129)] + [MIN + 2 * SEG + 64 * r + 1 for r in range(0, 32)]
    _run(gpu, lens, 4, gap=4100)


def test_split_big_segments(gpu):
    # past kSplitSeg * (kSplitMaxSegs - 1) bytes the segments are 1 MiB
    _run(gpu, [300 * (1 << 20) + 77, 5000, (1 << 20) + 1], 7, gap=5000)


def test_split_through_the_automatic_path(gpu):
    # under 1024 payloads the automatic entry takes the sorted path
    lens = [(1 << 20) + 17 * k for k in range(40)]
    _run(gpu, lens, 5, path="auto")


def test_update_mode_long_payloads(gpu):
    """crc32_update registers over long fragments (split like digests), carried over two calls."""
    import torch

    import annety_amd

    rng = np.random.default_rng(6)
    lens = np.concatenate([rng.integers(MIN + 1, 24 * SEG, 12), rng.integers(0, 3000, 200)]).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens + 5000)[:-1]]).astype(np.int64)
    data = oracle.lcg_bytes(int(offs[-1] + lens[-1]) + 256, 6)
    d = torch.from_numpy(data.copy()).to(gpu)
    o = torch.from_numpy(offs).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    state = torch.full((lens.size,), -1, dtype=torch.int32, device=gpu)
    want = np.full(lens.size, 0xFFFFFFFF, dtype=np.uint32)
    annety_amd.set_var_path("sorted")
    try:
        for _ in range(2):
            annety_amd.crc32_update_batch_var(state, d, o, ln)
            want = oracle.batch_var_mt(data, offs.astype(np.uint64), lens.astype(np.uint32), threads=8, states=want)
        torch.cuda.synchronize()
    finally:
        annety_amd.set_var_path("auto")
    assert np.array_equal(state.cpu().numpy().view(np.uint32), want)


def _update_run(gpu, lens, seed, gap=5000, calls=2, timing=False):
    """crc32_update over fragments `lens` (registers carried over `calls` calls) against the oracle; with timing,
    also the device time of one more call (ms, HIP events)."""
    import torch

    import annety_amd

    lens = np.asarray(lens, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens + gap)[:-1]]).astype(np.int64) + (seed % 61)
    total = int(offs[-1] + lens[-1]) + 256
    g = torch.Generator(device=gpu)
    g.manual_seed(seed)
    d = torch.randint(0, 256, (total,), dtype=torch.uint8, device=gpu, generator=g)
    data = d.cpu().numpy()
    o = torch.from_numpy(offs).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    rng = np.random.default_rng(seed)
    want = rng.integers(0, 1 << 32, lens.size, dtype=np.uint64).astype(np.uint32)
    state = torch.from_numpy(want.view(np.int32).copy()).to(gpu)
    ms = None
    annety_amd.set_var_path("sorted")
    try:
        for _ in range(calls):
            annety_amd.crc32_update_batch_var(state, d, o, ln)
            want = oracle.batch_var_mt(data, offs.astype(np.uint64), lens.astype(np.uint32), threads=16, states=want)
        torch.cuda.synchronize()
        got = state.cpu().numpy().view(np.uint32)
        if timing:
            s0 = state.clone()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            annety_amd.crc32_update_batch_var(s0, d, o, ln)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
    finally:
        annety_amd.set_var_path("auto")
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (bad[:8], lens[bad[:8]])
    return ms, annety_amd.last_kernels()


def test_update_mode_split_16x64mib(gpu):
    """16 update fragments of 64 MiB (the codec's largest frame, LengthHeaderCodec.h:51) run as
    segments: bit-exact registers over two calls, and one call in well under a millisecond (one lane group per
    fragment took ~145 ms)."""
    lens = [(64 << 20) - 13 * k for k in range(16)]
    ms, kernels = _update_run(gpu, lens, 11, calls=2, timing=True)
    print(f"16 x 64 MiB update fragments: {ms:.3f} ms per call ({kernels})")
    assert "crc32_var_sorted_kernel" in kernels
    assert ms < 5.0, ms


def test_update_mode_split_edges(gpu):
    """Update-mode splits at the edges: first segments of 1..128 bytes, big segments, registers of every kind."""
    lens = ([MIN + r for r in range(1, 40)] + [MIN, MIN + SEG, 300 * (1 << 20) + 77, 0, 1, 3, 4, 5000]
            + [MIN + 2 * SEG + 64 * r + 1 for r in range(0, 16)])
    _update_run(gpu, lens, 12, gap=4100)


@pytest.mark.parametrize("update", [False, True])
def test_split_cap_exhausted(gpu, update):
    """with the descriptor cap lowered, the payloads that find no room run whole (no preset, no moved
    register) and those before them split; every digest / register stays exact."""
    import annety_amd

    rng = np.random.default_rng(13)
    # 24 payloads of 20-40 segments each, cap 300: some split, the rest run whole
    lens = [int(x) for x in rng.integers(20 * SEG, 40 * SEG, 24)] + [int(x) for x in rng.integers(0, 3000, 100)]
    lens = [int(x) for x in rng.permutation(lens)]
    annety_amd.set_split_cap(300)
    try:
        if update:
            _update_run(gpu, lens, 14, calls=2)
        else:
            _run(gpu, lens, 15)
        annety_amd.set_split_cap(0)  # never split
        if update:
            _update_run(gpu, lens, 16, calls=1)
        else:
            _run(gpu, lens, 17)
    finally:
        annety_amd.set_split_cap(1 << 18)
