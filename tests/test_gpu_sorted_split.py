"""Long payloads on the length-sorted path (crc32_kernels.h kSplitSeg): a payload of more than 128 KiB runs as
end-aligned 16 KiB segments (1 MiB past 256 MiB; the first takes the remainder), each a task of the sorted list,
whose group xors shift_{m seg}(its raw register) into the payload's digest. Digests against the oracle at the
edges: lengths just above the split threshold (a first segment of 1 byte), whole multiples of the segment, every
start offset class, payloads of several MiB and one past 256 MiB, long payloads mixed with many short ones, and
update mode (never split)."""
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
    """crc32_update registers over long fragments (update mode does not split), carried over two calls."""
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
