"""The length-sorted variable path (annety_crc_set_var_path("sorted"): counting sort by line count, then the
length classes) on every layout and edge case, against the oracle.

Every batch runs through annety_crc32_batch_var / annety_crc32_update_batch_var with the path forced to
"sorted", so batches of any size take it (the automatic entry would move dense batches to the arena path).
Edge cases after the reference's own (empty payloads, lengths 1-3 at line ends, payloads of exactly one line,
the init's four bytes spilling into the next line), layouts from the fuzz families (packed, gapped, shuffled,
overlapping, repeated), long payloads among short ones, update registers, and repeated calls of changing sizes
on one stream (the counting sort's alternating cursor sets) and on several streams. (Round 4 ran these against
the line-stream path, which was removed in round 5: it never beat the sorted path)"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture
def sorted_path(gpu):
    import annety_amd

    prev = annety_amd.set_var_path("sorted")
    yield gpu
    annety_amd.set_var_path(prev)


def _run(dev, host, offs, lens, states=None, out=None):
    import torch

    import annety_amd

    d = torch.from_numpy(host).to(dev)
    o = torch.from_numpy(np.asarray(offs, dtype=np.int64)).to(dev)
    ln = torch.from_numpy(np.asarray(lens, dtype=np.int64).astype(np.int32)).to(dev)
    if states is not None:
        st = torch.from_numpy(np.asarray(states, dtype=np.uint32).view(np.int32).copy()).to(dev)
        annety_amd.crc32_update_batch_var(st, d, o, ln)
        res = st
    else:
        res = annety_amd.crc32_batch_var(d, o, ln, out=out)
    torch.cuda.synchronize()
    assert annety_amd.last_kernels().startswith("crc32_extent_kernel<count>"), annety_amd.last_kernels()
    return res.cpu().numpy().view(np.uint32)


def _check(dev, host, offs, lens, ctx="", states=None):
    got = _run(dev, host, offs, lens, states=states)
    want = oracle.batch_var_mt(host, np.asarray(offs, dtype=np.uint64), np.asarray(lens, dtype=np.uint32), threads=8,
                               states=None if states is None else np.asarray(states, dtype=np.uint32))
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (ctx, bad.size, bad[:8].tolist(), np.asarray(lens)[bad[:8]].tolist())


def test_golden_fixtures(sorted_path, golden):
    """The compiled reference's recorded digests: every length 0..300 and a sweep to 64 KiB at 12 start
    alignments, and the Zipf batch; then packed batches of 1..1000 payloads against the oracle."""
    import annety_amd
    import torch

    dev = sorted_path
    g = golden("lengths.json")
    arena = torch.from_numpy(oracle.lcg_bytes(g["arena_bytes"], g["seed"])).to(dev)
    lens = torch.tensor(g["lengths"], dtype=torch.int32, device=dev)
    for row in g["rows"]:
        offs = torch.full((len(g["lengths"]),), row["start"], dtype=torch.int64, device=dev)
        out = annety_amd.crc32_batch_var(arena, offs, lens)
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        want = np.array([int(x, 16) for x in row["crc"]], dtype=np.uint32)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"start {row['start']}: lengths {[g['lengths'][i] for i in bad[:10]]}"
    z = golden("zipf.json")
    got = _run(dev, oracle.lcg_bytes(z["total_bytes"], z["seed_bytes"]), z["offsets"], z["lengths"])
    assert [int(x) for x in got] == [int(x, 16) for x in z["digests"]]
    rng = np.random.default_rng(11)
    for n in (1, 2, 63, 64, 65, 1000):
        lens = rng.integers(0, 3000, n)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]) + 5
        host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 300, dtype=np.uint8)
        _check(dev, host, offs, lens, ctx=n)


def test_every_short_length_at_every_line_offset(sorted_path):
    # lengths 0..300 starting at every offset of a 128-byte line (the init spill, 1-3 byte payloads at line
    # ends, exactly-one-line payloads), each as its own payload in one batch over one buffer
    rng = np.random.default_rng(12)
    host = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    lens, offs = [], []
    for L in range(0, 301):
        for a in (0, 1, 60, 64, 124, 125, 126, 127):
            lens.append(L)
            offs.append(1024 + 128 * ((L * 7 + a) % 300) + a)
    _check(sorted_path, host, offs, lens, ctx="short")
    _check(sorted_path, host, offs, lens, ctx="short-upd",
           states=rng.integers(0, 2 ** 32, len(lens), dtype=np.uint64).astype(np.uint32))


def test_empty_and_all_empty(sorted_path):
    rng = np.random.default_rng(13)
    host = rng.integers(0, 256, 4096, dtype=np.uint8)
    _check(sorted_path, host, [0, 5, 9], [0, 0, 0], ctx="all empty")
    lens = np.array([0, 3, 0, 0, 200, 0, 1, 0])
    _check(sorted_path, host, np.arange(8) * 300, lens, ctx="some empty")
    st = rng.integers(0, 2 ** 32, 8, dtype=np.uint64).astype(np.uint32)
    _check(sorted_path, host, np.arange(8) * 300, lens, ctx="some empty upd", states=st)


def test_long_payloads_among_short(sorted_path):
    # single payloads of 1 and 3 MiB (one lane group walks thousands of rounds), then long payloads among
    # short ones (every length class in one launch)
    rng = np.random.default_rng(14)
    host = rng.integers(0, 256, (3 << 20) + 777, dtype=np.uint8)
    _check(sorted_path, host, [3], [1 << 20], ctx="1 MiB")
    _check(sorted_path, host, [77], [(3 << 20) - 100], ctx="3 MiB")
    lens = rng.integers(0, 100, 2000)
    lens[::97] = rng.integers(100_000, 400_000, lens[::97].size)
    offs = rng.integers(0, host.size - lens + 1)
    _check(sorted_path, host, offs, lens, ctx="mixed")
    st = rng.integers(0, 2 ** 32, lens.size, dtype=np.uint64).astype(np.uint32)
    _check(sorted_path, host, offs, lens, ctx="mixed upd", states=st)


def test_fuzz_layouts(sorted_path):
    from test_gpu_fuzz import _layout, _lengths

    rng = np.random.default_rng(20261017)
    cap = 8 << 20
    for fam in range(40):
        n = int(rng.choice([1, 7, 300, 1500, 4000, 20000]))
        lens = _lengths(rng, n)
        kind, offs, lens = _layout(rng, lens, cap // 4)
        need = int((offs + lens).max()) + 1
        if need > cap:
            lens = (lens * cap / need * 0.5).astype(np.int64)
            offs = (offs * cap / need * 0.5).astype(np.int64)
        host = rng.integers(0, 256, cap, dtype=np.uint8)
        states = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32) if fam % 3 == 2 else None
        _check(sorted_path, host, offs, lens, ctx=(fam, kind, n), states=states)


def test_repeated_calls_changing_sizes_and_streams(sorted_path):
    # the counting sort's two cursor sets alternate per call on a stream's slot and each call zeroes the set
    # of the next: sizes that grow and shrink, then the same on four streams in turn
    import torch

    import annety_amd

    rng = np.random.default_rng(15)
    host = rng.integers(0, 256, 4 << 20, dtype=np.uint8)
    d = torch.from_numpy(host).to(sorted_path)
    streams = [torch.cuda.Stream(device=sorted_path) for _ in range(4)]
    for rep, n in enumerate([5000, 100, 9000, 9000, 1, 20000, 2048, 2049, 4096, 300]):
        lens = rng.integers(0, 400, n)
        offs = rng.integers(0, host.size - 400, n)
        want = oracle.batch_var_mt(host, offs.astype(np.uint64), lens.astype(np.uint32), threads=8)
        for s in [None] + (streams if rep % 3 == 0 else []):
            with torch.cuda.stream(s) if s is not None else torch.cuda.stream(torch.cuda.current_stream()):
                o = torch.from_numpy(offs).to(sorted_path)
                ln = torch.from_numpy(lens.astype(np.int32)).to(sorted_path)
                out = annety_amd.crc32_batch_var(d, o, ln)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            assert np.array_equal(got, want), (rep, n, int((got != want).sum()))
    for s in streams:
        annety_amd.stream_release(s)
