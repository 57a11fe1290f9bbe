"""The line-stream variable path (crc32_stream.hip: scan + stream + cross-chunk fixup) against the oracle.

Every batch runs through annety_crc32_batch_var / annety_crc32_update_batch_var with the path set to "stream"
(annety_crc_set_var_path). Small batches already exercise the chunk machinery hard: the stream launch cuts the
positions into one chunk per wave (2048 waves on 256 CUs), so a batch of a few thousand lines has a chunk
boundary every 64 lines and most payloads cross one; a single long payload crosses hundreds (the fixup's
per-lane pieces and its loop over 64-piece groups). Edge cases after the reference's own (empty payloads,
lengths 1-3 at line ends, payloads of exactly one line, the init's four bytes spilling into the next line),
layouts from the fuzz families (packed, gapped, shuffled, overlapping, repeated), update registers, repeated
calls of changing sizes on one stream (the scan's alternating status sets) and on several streams, and the
full BASELINE config-3 batch."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture
def stream_path(gpu):
    import annety_amd

    prev = annety_amd.set_var_path("stream")
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
    assert annety_amd.last_kernels().startswith("crc32_stream_scan_kernel"), annety_amd.last_kernels()
    return res.cpu().numpy().view(np.uint32)


def _check(dev, host, offs, lens, ctx="", states=None):
    got = _run(dev, host, offs, lens, states=states)
    want = oracle.batch_var_mt(host, np.asarray(offs, dtype=np.uint64), np.asarray(lens, dtype=np.uint32), threads=8,
                               states=None if states is None else np.asarray(states, dtype=np.uint32))
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (ctx, bad.size, bad[:8].tolist(), np.asarray(lens)[bad[:8]].tolist())


def test_golden_fixtures(stream_path, golden):
    """The compiled reference's recorded digests: every length 0..300 and a sweep to 64 KiB at 12 start
    alignments, and the Zipf batch; then packed batches of 1..1000 payloads against the oracle."""
    import annety_amd
    import torch

    dev = stream_path
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


def test_every_short_length_at_every_line_offset(stream_path):
    # lengths 0..300 starting at every offset of a 128-byte line (the init spill, 1-3 byte payloads at line
    # ends, exactly-one-line payloads), each as its own payload in one batch over one buffer
    rng = np.random.default_rng(12)
    host = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    lens, offs = [], []
    for L in range(0, 301):
        for a in (0, 1, 60, 64, 124, 125, 126, 127):
            lens.append(L)
            offs.append(1024 + 128 * ((L * 7 + a) % 300) + a)
    _check(stream_path, host, offs, lens, ctx="short")
    _check(stream_path, host, offs, lens, ctx="short-upd",
           states=rng.integers(0, 2 ** 32, len(lens), dtype=np.uint64).astype(np.uint32))


def test_empty_and_all_empty(stream_path):
    rng = np.random.default_rng(13)
    host = rng.integers(0, 256, 4096, dtype=np.uint8)
    _check(stream_path, host, [0, 5, 9], [0, 0, 0], ctx="all empty")
    lens = np.array([0, 3, 0, 0, 200, 0, 1, 0])
    _check(stream_path, host, np.arange(8) * 300, lens, ctx="some empty")
    st = rng.integers(0, 2 ** 32, 8, dtype=np.uint64).astype(np.uint32)
    _check(stream_path, host, np.arange(8) * 300, lens, ctx="some empty upd", states=st)


def test_long_payloads_across_many_chunks(stream_path):
    # one payload of 1 MiB (8192 lines: with a chunk per 64 lines it crosses 127 boundaries, two rounds of
    # the fixup's 64 lanes), then long payloads among short ones
    rng = np.random.default_rng(14)
    host = rng.integers(0, 256, (3 << 20) + 777, dtype=np.uint8)
    _check(stream_path, host, [3], [1 << 20], ctx="1 MiB")
    _check(stream_path, host, [77], [(3 << 20) - 100], ctx="3 MiB")
    lens = rng.integers(0, 100, 2000)
    lens[::97] = rng.integers(100_000, 400_000, lens[::97].size)
    offs = rng.integers(0, host.size - lens + 1)
    _check(stream_path, host, offs, lens, ctx="mixed")
    st = rng.integers(0, 2 ** 32, lens.size, dtype=np.uint64).astype(np.uint32)
    _check(stream_path, host, offs, lens, ctx="mixed upd", states=st)


def test_fuzz_layouts(stream_path):
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
        _check(stream_path, host, offs, lens, ctx=(fam, kind, n), states=states)


def test_repeated_calls_changing_sizes_and_streams(stream_path):
    # the scan's status sets alternate per call on a stream's slot and each call zeroes the records the
    # previous one left: sizes that grow and shrink (more and fewer tiles than the call before), then the
    # same on four streams in turn
    import torch

    import annety_amd

    rng = np.random.default_rng(15)
    host = rng.integers(0, 256, 4 << 20, dtype=np.uint8)
    d = torch.from_numpy(host).to(stream_path)
    streams = [torch.cuda.Stream(device=stream_path) for _ in range(4)]
    for rep, n in enumerate([5000, 100, 9000, 9000, 1, 20000, 2048, 2049, 4096, 300]):
        lens = rng.integers(0, 400, n)
        offs = rng.integers(0, host.size - 400, n)
        want = oracle.batch_var_mt(host, offs.astype(np.uint64), lens.astype(np.uint32), threads=8)
        for s in [None] + (streams if rep % 3 == 0 else []):
            with torch.cuda.stream(s) if s is not None else torch.cuda.stream(torch.cuda.current_stream()):
                o = torch.from_numpy(offs).to(stream_path)
                ln = torch.from_numpy(lens.astype(np.int32)).to(stream_path)
                out = annety_amd.crc32_batch_var(d, o, ln)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            assert np.array_equal(got, want), (rep, n, int((got != want).sum()))
    for s in streams:
        annety_amd.stream_release(s)


def test_config3_full_stream(stream_path):
    import torch

    import annety_amd
    from test_gpu_fullsize import THREADS, _bench

    gpu = stream_path
    lens, offs = _bench().zipf_batch(0x5EED)
    total = int(lens.sum())
    g = torch.Generator(device=gpu)
    g.manual_seed(4242)
    data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=gpu, generator=g)
    d_off = torch.from_numpy(offs).to(gpu)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    got = annety_amd.crc32_batch_var(data, d_off, d_len)
    torch.cuda.synchronize()
    print("config 3 (stream): digests done", flush=True)
    host = data.cpu().numpy()
    want = oracle.batch_var_mt(host, offs, lens, THREADS)
    bad = np.nonzero(got.cpu().numpy().view(np.uint32) != want)[0]
    assert bad.size == 0, f"{bad.size} digest mismatches, first {bad[:8]} (lengths {lens[bad[:8]]})"
    rng = np.random.default_rng(5)
    states = rng.integers(0, 2 ** 32, lens.size, dtype=np.uint64).astype(np.uint32)
    d_state = torch.from_numpy(states.view(np.int32).copy()).to(gpu)
    annety_amd.crc32_update_batch_var(d_state, data, d_off, d_len)
    torch.cuda.synchronize()
    want = oracle.batch_var_mt(host, offs, lens, THREADS, states=states)
    bad = np.nonzero(d_state.cpu().numpy().view(np.uint32) != want)[0]
    assert bad.size == 0, f"{bad.size} register mismatches, first {bad[:8]}"
