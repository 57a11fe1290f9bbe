"""Automatic path choice of annety_crc32_batch_var / annety_crc32_update_batch_var (crc32_capi.cpp
run_var_auto): every call records its batch's extent on the device; once two completed calls on a stream
with the same pointers showed a dense sorted batch the arena path runs, re-checking each call's own extent on
the device. Until the records decide - and on every call with fresh offset/length arrays - the device chooses
within the call (AutoChoice: extent kernel, then both paths' launches, only the chosen one runs). Digests are
checked against the oracle on every call, also when the layout changes under the same pointers (the arena
launches then fold each payload directly) and for sparse batches (sorted path)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _packed(seed, n, gap=0):
    rng = np.random.default_rng(seed)
    lens = np.minimum(65536, 64 * np.minimum(rng.zipf(1.3, n), 1 << 20) + rng.integers(0, 64, n)).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens + gap)[:-1]]).astype(np.int64)
    data = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 256, dtype=np.uint8)
    return data, offs, lens


def _dev(gpu, data, offs, lens):
    import torch

    return (torch.from_numpy(data).to(gpu), torch.from_numpy(offs).to(gpu),
            torch.from_numpy(lens.astype(np.int32)).to(gpu))


def _check(out, data, offs, lens):
    import torch

    torch.cuda.synchronize()
    want = oracle.batch_var(data, offs.astype(np.uint64), lens.astype(np.uint32))
    got = out.cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want), int((got != want).sum())


def test_dense_batch_moves_to_arena(gpu):
    import torch

    import annety_amd

    data, offs, lens = _packed(1, 5000)
    d, o, ln = _dev(gpu, data, offs, lens)
    out = torch.empty(len(lens), dtype=torch.int32, device=gpu)
    s0 = annety_amd.var_path_stats(0)
    for i in range(6):
        out.zero_()
        annety_amd.crc32_batch_var(d, o, ln, out=out)
        _check(out, data, offs, lens)  # synchronises: this call's extent record is complete
    s1 = annety_amd.var_path_stats(0)
    assert s1["device"] - s0["device"] == 2 and s1["arena"] - s0["arena"] == 4, (s0, s1)
    assert s1["sorted"] == s0["sorted"], (s0, s1)
    # back to back without waiting: every digest still exact
    outs = [torch.empty(len(lens), dtype=torch.int32, device=gpu) for _ in range(8)]
    for x in outs:
        annety_amd.crc32_batch_var(d, o, ln, out=x)
    for x in outs:
        _check(x, data, offs, lens)


def test_sparse_batch_stays_sorted(gpu):
    import torch

    import annety_amd

    data, offs, lens = _packed(2, 3000, gap=40000)  # payload bytes ~20 % of the span: never the arena path
    d, o, ln = _dev(gpu, data, offs, lens)
    out = torch.empty(len(lens), dtype=torch.int32, device=gpu)
    s0 = annety_amd.var_path_stats(0)
    for _ in range(4):
        annety_amd.crc32_batch_var(d, o, ln, out=out)
        _check(out, data, offs, lens)
    s1 = annety_amd.var_path_stats(0)
    # the first call's device choice (sorted), then its record sends the rest to the sorted path directly
    assert s1["arena"] == s0["arena"] and s1["device"] - s0["device"] == 1 and s1["sorted"] - s0["sorted"] == 3


def test_layout_changes_under_the_same_pointers(gpu):
    """The arena path is chosen from earlier calls; then the offsets are rewritten in place (a shifted dense
    layout, then one with a 6 KiB gap, then unsorted): the device check sees the difference and every digest
    stays exact."""
    import torch

    import annety_amd

    data, offs, lens = _packed(3, 4000)
    data = np.concatenate([data, np.zeros(70000, dtype=np.uint8)])  # room for every variant below
    d, o, ln = _dev(gpu, data, offs, lens)
    out = torch.empty(len(lens), dtype=torch.int32, device=gpu)
    for _ in range(4):
        annety_amd.crc32_batch_var(d, o, ln, out=out)
        _check(out, data, offs, lens)
    a0 = annety_amd.var_path_stats(0)["arena"]
    variants = [offs + 200, offs.copy(), offs[::-1].copy()]
    variants[1][len(offs) // 2:] += 6000  # one 6 KiB gap
    for v in variants:
        o.copy_(torch.from_numpy(v))  # same pointers, new layout
        annety_amd.crc32_batch_var(d, o, ln, out=out)
        _check(out, data, v, lens)
    assert annety_amd.var_path_stats(0)["arena"] > a0  # the first changed call still took the arena path


def test_update_mode_auto(gpu):
    """Streaming registers through the automatic path: the same fragment layout every call (a receive ring),
    registers carried across calls, equal to the oracle's crc32_update chain."""
    import torch

    import annety_amd

    data, offs, lens = _packed(4, 2000)
    d, o, ln = _dev(gpu, data, offs, lens)
    state = torch.full((len(lens),), -1, dtype=torch.int32, device=gpu)
    want = np.full(len(lens), 0xFFFFFFFF, dtype=np.uint32)
    for _ in range(5):
        annety_amd.crc32_update_batch_var(state, d, o, ln)
        want = oracle.batch_var_mt(data, offs.astype(np.uint64), lens.astype(np.uint32), threads=8, states=want)
        torch.cuda.synchronize()
        assert np.array_equal(state.cpu().numpy().view(np.uint32), want)


def test_sorted_calls_back_to_back(gpu):
    """The sorted path's counting sort alternates two cursor sets per stream slot, each zeroed by the call
    before (crc32_kernels.h BucketArgs): ten calls on one stream with no wait between them, alternating the
    explicit sorted entry (n < 1024) and the automatic one (sparse, unsorted batches of 1024+ payloads with
    empty payloads), each with its own batch and all checked afterwards."""
    import torch

    import annety_amd

    cases, outs = [], []
    for i in range(10):
        n = 700 + 37 * i if i % 2 == 0 else 2500 + 301 * i
        rng = np.random.default_rng(100 + i)
        lens = np.minimum(40000, 64 * np.minimum(rng.zipf(1.4, n), 1 << 20) + rng.integers(0, 300, n)).astype(np.int64)
        lens[rng.integers(0, n, n // 20)] = 0
        offs = np.concatenate([[0], np.cumsum(lens + 5000)[:-1]]).astype(np.int64)
        perm = rng.permutation(n)  # unsorted descriptors
        offs, lens = offs[perm].copy(), lens[perm].copy()
        data = rng.integers(0, 256, int((offs + lens).max()) + 256, dtype=np.uint8)
        cases.append((data, offs, lens, _dev(gpu, data, offs, lens)))
    s0 = annety_amd.var_path_stats(0)
    for data, offs, lens, (d, o, ln) in cases:
        out = torch.full((len(lens),), 7, dtype=torch.int32, device=gpu)
        annety_amd.crc32_batch_var(d, o, ln, out=out)
        outs.append(out)
    for (data, offs, lens, _), out in zip(cases, outs):
        _check(out, data, offs, lens)
    s1 = annety_amd.var_path_stats(0)
    # every batch is new to the stream: the device chose (the sorted path: sparse, unsorted)
    assert s1["arena"] == s0["arena"] and s1["device"] - s0["device"] == 5, (s0, s1)


def test_unrecorded_arena_calls_between_records(gpu):
    """Between two calls that record their extent (one in kAutoRefresh), the arena path runs without the
    extent kernel and without the device check: the declared range is checked on the host to lie in one
    allocation and payloads outside it are folded directly. Twenty calls, the layout rewritten in place
    three times inside such windows, every digest exact."""
    import torch

    import annety_amd

    data, offs, lens = _packed(6, 3000)
    data = np.concatenate([data, np.zeros(70000, dtype=np.uint8)])
    d, o, ln = _dev(gpu, data, offs, lens)
    out = torch.empty(len(lens), dtype=torch.int32, device=gpu)
    s0 = annety_amd.var_path_stats(0)
    layouts = {9: offs + 300, 13: offs[::-1].copy(), 17: offs.copy()}
    layouts[17][len(offs) // 3:] += 9000  # a 9 KiB gap: the payloads after it leave the declared range
    cur = offs
    for i in range(20):
        if i in layouts:
            cur = layouts[i]
            o.copy_(torch.from_numpy(cur))
        out.fill_(7)
        annety_amd.crc32_batch_var(d, o, ln, out=out)
        _check(out, data, cur, lens)
    s1 = annety_amd.var_path_stats(0)
    assert s1["arena_unrecorded"] - s0["arena_unrecorded"] >= 10, (s0, s1)


@pytest.mark.parametrize("layout", ["shuffled", "gapped"])
def test_dense_unsorted_or_gapped_batch_moves_to_arena(gpu, layout):
    """Dense batches (payload bytes >= 2/3 of the span) in any order, or with gaps of 4 KiB and more, take the
    arena path once the span is seen to lie inside one device allocation (crc32_capi.cpp run_var_auto,
    check_any_order); the device check then accepts the recorded extent whatever its order."""
    import torch

    import annety_amd

    if layout == "shuffled":
        data, offs, lens = _packed(7, 5000)
        perm = np.random.default_rng(8).permutation(len(offs))
        offs, lens = offs[perm].copy(), lens[perm].copy()
    else:
        rng = np.random.default_rng(9)
        lens = rng.integers(40000, 65536, 1100).astype(np.int64)
        offs = np.concatenate([[0], np.cumsum(lens + 5000)[:-1]]).astype(np.int64)  # 5 KiB gaps, ~90% dense
        data = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 256, dtype=np.uint8)
    d, o, ln = _dev(gpu, data, offs, lens)
    out = torch.empty(len(lens), dtype=torch.int32, device=gpu)
    s0 = annety_amd.var_path_stats(0)
    for _ in range(12):
        out.fill_(7)
        annety_amd.crc32_batch_var(d, o, ln, out=out)
        _check(out, data, offs, lens)
    s1 = annety_amd.var_path_stats(0)
    # (the device cannot see allocations: it runs these on the sorted path until the host's records decide)
    assert s1["device"] - s0["device"] == 2 and s1["arena"] - s0["arena"] == 10, (s0, s1)


@pytest.mark.parametrize("density,arena", [(0.655, False), (0.680, True)])
def test_density_boundary_inside_one_allocation(gpu, density, arena):
    """The 2/3-density rule (crc32_capi.cpp run_var_auto: payload bytes * 3 >= span * 2) pinned from both sides on
    one allocation: equal 40,000-byte payloads with equal gaps of >= 4 KiB (so the small-gap rule does not apply),
    at 0.655 of the span the sorted path stays, at 0.680 the arena takes over after the two recording calls.
    Every digest is exact either way."""
    import torch

    import annety_amd

    n, L = 1200, 40000
    gap = int(round(L / density)) - L
    lens = np.full(n, L, dtype=np.int64)
    offs = (np.arange(n, dtype=np.int64) * (L + gap)).astype(np.int64)
    span = int(offs[-1] + L)
    assert (n * L * 3 >= span * 2) == arena  # the layout is on the intended side of the rule
    data = np.random.default_rng(11).integers(0, 256, span + 256, dtype=np.uint8)
    d, o, ln = _dev(gpu, data, offs, lens)
    out = torch.empty(n, dtype=torch.int32, device=gpu)
    s0 = annety_amd.var_path_stats(0)
    for _ in range(6):
        out.fill_(7)
        annety_amd.crc32_batch_var(d, o, ln, out=out)
        _check(out, data, offs, lens)
    s1 = annety_amd.var_path_stats(0)
    if arena:
        # (the first call may go to the sorted path on the host's word: torch can hand this test the addresses of the
        # previous case's tensors, whose records - same pointers, another layout - are not dense)
        assert s1["device"] + s1["sorted"] - s0["device"] - s0["sorted"] == 2 and s1["arena"] - s0["arena"] == 4, (s0, s1)
    else:
        assert s1["arena"] == s0["arena"] and s1["device"] - s0["device"] == 1, (s0, s1)
        assert s1["sorted"] - s0["sorted"] == 5, (s0, s1)


def _fresh_calls(gpu, data, offs, lens, calls, update=False):
    """`calls` calls with fresh offset/length tensors each time (per-connection batches), every result checked;
    returns the device time of the last call (ms, HIP events) and the stats delta."""
    import torch

    import annety_amd

    d = torch.from_numpy(data).to(gpu)
    s0 = annety_amd.var_path_stats(0)
    ms = None
    want = np.full(len(lens), 0xFFFFFFFF, dtype=np.uint32)
    state = torch.full((len(lens),), -1, dtype=torch.int32, device=gpu)
    keep = []  # every call's arrays stay alive, so no two calls share an address (the caching allocator would reuse)
    for i in range(calls):
        o = torch.from_numpy(offs.copy()).to(gpu)
        ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
        out = torch.full((len(lens),), 7, dtype=torch.int32, device=gpu)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if update:
            annety_amd.crc32_update_batch_var(state, d, o, ln)
        else:
            annety_amd.crc32_batch_var(d, o, ln, out=out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        if update:
            want = oracle.batch_var_mt(data, offs.astype(np.uint64), lens.astype(np.uint32), threads=16, states=want)
            assert np.array_equal(state.cpu().numpy().view(np.uint32), want)
        else:
            want = oracle.batch_var_mt(data, offs.astype(np.uint64), lens.astype(np.uint32), threads=16)
            assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
        keep.append((o, ln, out))
    s1 = annety_amd.var_path_stats(0)
    return ms, {k: s1[k] - s0[k] for k in s1}


def _small_frames(seed, n):
    """n LengthHeaderCodec-like payloads of 16 B-1 KiB packed with 8-byte gaps (a received frame stream)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(16, 1025, n).astype(np.int64)
    offs = (np.concatenate([[0], np.cumsum(lens + 8)[:-1]]) + 4).astype(np.int64)
    data = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 260, dtype=np.uint8)
    return data, offs, lens


def test_fresh_pointers_reach_the_arena(gpu):
    """a caller passing new offset/length tensors on every call never has two records for the
    same pointers, so only the device's choice can take it to the arena path. 2M small frames: the sorted path
    takes ~457 us, the arena ~284 us; each call here must be on the arena's side (the first call may run sorted
    while the stream's scratch grows to the recorded span)."""
    import annety_amd

    data, offs, lens = _small_frames(21, 2 << 20)
    ms, st = _fresh_calls(gpu, data, offs, lens, 4)
    prev = annety_amd.set_var_path("sorted")
    try:
        ms_sorted, _ = _fresh_calls(gpu, data, offs, lens, 2)
    finally:
        annety_amd.set_var_path(prev)
    print(f"2M small frames, fresh pointers per call: {ms * 1e3:.1f} us (sorted path {ms_sorted * 1e3:.1f} us)")
    assert st["device"] == 4 and st["arena"] == 0 and st["sorted"] == 0, st
    assert ms < 0.8 * ms_sorted, (ms, ms_sorted)
    # the records a device-chosen arena call publishes carry the whole batch's extent (every lane of the stitch's
    # wave reduces the partials): the same pointers again go to the arena path on the host's word from the third call
    import torch

    d = torch.from_numpy(data).to(gpu)
    o = torch.from_numpy(offs).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    out = torch.empty(len(lens), dtype=torch.int32, device=gpu)
    s0 = annety_amd.var_path_stats(0)
    for _ in range(5):
        annety_amd.crc32_batch_var(d, o, ln, out=out)
        torch.cuda.synchronize()
    s1 = annety_amd.var_path_stats(0)
    assert s1["arena"] - s0["arena"] == 3 and s1["device"] - s0["device"] == 2, (s0, s1)
    want = oracle.batch_var_mt(data, offs.astype(np.uint64), lens.astype(np.uint32), threads=16)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want)


def test_fresh_pointers_update_and_sparse(gpu):
    """The device choice in update mode (registers carried over calls, fresh pointers each call), and on sparse
    batches (the device keeps them on the sorted path)."""
    data, offs, lens = _small_frames(22, 30000)
    _fresh_calls(gpu, data, offs, lens, 3, update=True)
    rng = np.random.default_rng(23)
    lens = rng.integers(0, 3000, 5000).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens + 20000)[:-1]]).astype(np.int64)
    data = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 256, dtype=np.uint8)
    _, st = _fresh_calls(gpu, data, offs, lens, 3)
    assert st["device"] == 3, st
