"""Parity of the MI355X kernels (through the C-ABI) with the reference, on the GPU.

Small cases: bit-exact against the golden fixtures written by the compiled reference
(tests/golden/make_golden.py) and against the CPU oracle on the same seeded inputs.
Full size (BASELINE config 1, 1M x 1 KiB): bit-exact against the multi-threaded oracle on every
payload, plus size-independent properties (combine identity, bit-flip detection).
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def H(x: str) -> int:
    return int(x, 16)


def to_dev(arr: np.ndarray, device):
    import torch

    return torch.from_numpy(np.ascontiguousarray(arr)).to(device)


def digests(out) -> np.ndarray:
    import torch

    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def test_lcg_1024x1k_golden(golden, gpu):
    import annety_amd

    g = golden("lcg_1024x1k.json")
    arena = oracle.lcg_bytes(g["n"] * g["len"], g["seed"])
    out = annety_amd.crc32_batch(to_dev(arena, gpu), g["n"], g["len"])
    d = digests(out)
    assert [int(x) for x in d] == [H(x) for x in g["digests"]]
    assert int(np.bitwise_xor.reduce(d)) == H(g["xor_all"])


def test_fixed_batches_golden(golden, gpu):
    """Assorted lengths/strides: aligned fast path (FULL and end-aligned virtual-lead layouts, G=1..32)
    and the general kernel for odd shapes (len % 16 != 0, stride % 16 != 0)."""
    import annety_amd

    g = golden("fixed_batches.json")
    arena = to_dev(oracle.lcg_bytes(g["arena_bytes"], g["seed"]), gpu)
    for c in g["cases"]:
        out = annety_amd.crc32_batch(arena, c["n"], c["len"], c["stride"])
        assert [int(x) for x in digests(out)] == [H(x) for x in c["digests"]], (c["n"], c["len"], c["stride"])


def test_fixed_with_offset_base(golden, gpu):
    """Same fixtures through a misaligned base pointer (routes to the general kernel)."""
    import annety_amd
    import torch

    g = golden("fixed_batches.json")
    host = oracle.lcg_bytes(g["arena_bytes"], g["seed"])
    buf = torch.zeros(g["arena_bytes"] + 64, dtype=torch.uint8, device=gpu)
    for shift in (1, 3, 8):
        buf[shift:shift + g["arena_bytes"]] = to_dev(host, gpu)
        for c in g["cases"][:10]:
            out = torch.empty(c["n"], dtype=torch.int32, device=gpu)
            import annety_amd._lib as L

            st = L.get().annety_crc32_batch_fixed(buf.data_ptr() + shift, c["n"], c["len"], c["stride"], out.data_ptr(),
                                                  torch.cuda.current_stream().cuda_stream)
            assert st == 0
            assert [int(x) for x in digests(out)] == [H(x) for x in c["digests"]], (shift, c["len"])


def test_lengths_unaligned_var(golden, gpu):
    """Every length 0..300 and a sweep to 64 KiB at 12 start alignments (variable-length kernel)."""
    import annety_amd
    import torch

    g = golden("lengths.json")
    arena = to_dev(oracle.lcg_bytes(g["arena_bytes"], g["seed"]), gpu)
    lens = torch.tensor(g["lengths"], dtype=torch.int32, device=gpu)
    for row in g["rows"]:
        offs = torch.full((len(g["lengths"]),), row["start"], dtype=torch.int64, device=gpu)
        got = digests(annety_amd.crc32_batch_var(arena, offs, lens))
        want = np.array([H(x) for x in row["crc"]], dtype=np.uint32)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"start {row['start']}: lengths {[g['lengths'][i] for i in bad[:10]]}"


def test_zipf_var(golden, gpu):
    import annety_amd
    import torch

    g = golden("zipf.json")
    arena = to_dev(oracle.lcg_bytes(g["total_bytes"], g["seed_bytes"]), gpu)
    offs = torch.tensor(g["offsets"], dtype=torch.int64, device=gpu)
    lens = torch.tensor(g["lengths"], dtype=torch.int32, device=gpu)
    got = digests(annety_amd.crc32_batch_var(arena, offs, lens))
    assert [int(x) for x in got] == [H(x) for x in g["digests"]]


def test_big_payloads(golden, gpu):
    """4 MiB (config 2 shape), 4 MiB + 12345 (tail), 64 MiB (LengthHeaderCodec max_payload)."""
    import annety_amd
    import torch

    for c in golden("big.json")["cases"]:
        b = to_dev(oracle.lcg_bytes(c["bytes"], c["seed"]), gpu)
        out = annety_amd.crc32_batch(b, 1, c["bytes"])
        assert int(digests(out)[0]) == H(c["crc"]), c
        got = digests(annety_amd.crc32_batch_var(b, torch.zeros(1, dtype=torch.int64, device=gpu),
                                                 torch.tensor([c["bytes"]], dtype=torch.int32, device=gpu)))
        assert int(got[0]) == H(c["crc"]), c


def test_config2_shape_reduced(gpu):
    """64 x 4 MiB (config 2 layout at 1/64 of the count) vs the oracle."""
    import annety_amd

    n, L = 64, 4 << 20
    host = oracle.lcg_bytes(n * L, 2024)
    got = digests(annety_amd.crc32_batch(to_dev(host, gpu), n, L))
    want = oracle.batch_fixed_mt(host, n, L, threads=16)
    assert np.array_equal(got, want)


def test_update_batch(gpu):
    """crc32_update semantics (include/Crc32c.h:71-82) from arbitrary registers."""
    import annety_amd
    import torch

    rng = np.random.default_rng(5)
    for n, L in [(300, 1024), (50, 4096), (7, 48), (33, 65536), (5, 1040)]:
        host = oracle.lcg_bytes(n * L, 77 + L)
        s0 = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
        st = torch.from_numpy(s0.view(np.int32).copy()).to(gpu)
        annety_amd.crc32_update_batch(st, to_dev(host, gpu), n, L)
        got = digests(st)
        want = np.array([oracle.crc32_update(int(s0[i]), host[i * L:(i + 1) * L]) for i in range(n)], dtype=np.uint32)
        assert np.array_equal(got, want), (n, L)


def test_host_staged_path(golden, gpu):
    import annety_amd

    g = golden("lcg_1024x1k.json")
    arena = oracle.lcg_bytes(g["n"] * g["len"], g["seed"])
    got = annety_amd.crc32_batch_host(arena, g["n"], g["len"])
    assert [int(x) for x in got] == [H(x) for x in g["digests"]]
    # odd stride/len through the staging packer
    gf = golden("fixed_batches.json")
    a2 = oracle.lcg_bytes(gf["arena_bytes"], gf["seed"])
    for c in gf["cases"]:
        got = annety_amd.crc32_batch_host(a2, c["n"], c["len"], c["stride"])
        assert [int(x) for x in got] == [H(x) for x in c["digests"]], c


def test_empty_and_edge(gpu):
    import annety_amd
    import torch

    buf = torch.zeros(4096, dtype=torch.uint8, device=gpu)
    out = torch.full((5,), 7, dtype=torch.int32, device=gpu)
    annety_amd.crc32_batch(buf, 5, 0, 16, out=out)
    assert digests(out).tolist() == [0] * 5
    out = annety_amd.crc32_batch(buf, 0, 16)
    assert out.numel() == 0
    # zero-length entries in a variable batch
    offs = torch.tensor([0, 5, 9], dtype=torch.int64, device=gpu)
    lens = torch.tensor([0, 0, 3], dtype=torch.int32, device=gpu)
    got = digests(annety_amd.crc32_batch_var(buf, offs, lens))
    assert got.tolist() == [0, 0, oracle.crc32_long(bytes(3))]


@pytest.fixture(scope="module")
def config1(gpu):
    """BASELINE config 1: 1M x 1 KiB random payloads, contiguous in HBM."""
    import torch

    n, L = 1 << 20, 1024
    g = torch.Generator(device=gpu)
    g.manual_seed(1234)
    data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=gpu, generator=g)
    return n, L, data


def test_config1_full_bitexact(config1):
    import annety_amd

    n, L, data = config1
    got = digests(annety_amd.crc32_batch(data, n, L))
    assert annety_amd.last_kernels() == "crc32_onekib_nt_kernel"  # the kernel bench.py's roofline names
    host = data.cpu().numpy()
    want = oracle.batch_fixed_mt(host, n, L, threads=16)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first {bad[:8]}"


def test_config1_properties(config1):
    """Size-independent checks at full size: one bit flipped in every 4097th payload changes exactly
    those digests; digests of adjacent payload pairs join to the digest of the 2 KiB concatenation."""
    import annety_amd

    n, L, data = config1
    base = digests(annety_amd.crc32_batch(data, n, L)).copy()
    flipped = data.clone()
    idx = np.arange(0, n, 4097)
    pos = (idx * L + (idx * 7919) % L).astype(np.int64)
    import torch

    p = torch.from_numpy(pos).to(data.device)
    flipped[p] ^= (1 << (torch.from_numpy(idx % 8).to(data.device))).to(torch.uint8)
    after = digests(annety_amd.crc32_batch(flipped, n, L))
    changed = np.nonzero(after != base)[0]
    assert np.array_equal(changed, idx)
    pairs = digests(annety_amd.crc32_batch(data, n // 2, 2 * L))
    joined = np.array([oracle.crc32_combine(int(base[2 * i]), int(base[2 * i + 1]), L) for i in range(0, n // 2, 509)],
                      dtype=np.uint32)
    assert np.array_equal(pairs[::509], joined)


def test_update_batch_var(gpu):
    """Streaming update (§8f row 4): arbitrary registers, unaligned fragments of every length class,
    including the < 4-byte fragments whose register cannot be injected as payload bytes."""
    import annety_amd
    import torch

    rng = np.random.default_rng(77)
    n = 6000
    lens = np.concatenate([np.arange(0, 300), rng.integers(0, 5000, n - 400), rng.integers(16384, 70000, 100)])
    rng.shuffle(lens)
    offs = np.cumsum(np.concatenate([[0], lens[:-1] + rng.integers(0, 7, n - 1)])).astype(np.int64)
    arena = oracle.lcg_bytes(int(offs[-1] + lens[-1]) + 16, 404)
    states = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    d_state = to_dev(states.view(np.int32), gpu)
    annety_amd.crc32_update_batch_var(d_state, to_dev(arena, gpu), to_dev(offs, gpu),
                                      to_dev(lens.astype(np.int32), gpu))
    got = digests(d_state)
    want = np.array([oracle.crc32_update(int(s), arena[o : o + L]) for s, o, L in zip(states, offs, lens)],
                    dtype=np.uint32)
    assert np.array_equal(got, want)


def test_streaming_fragments(gpu):
    """Streams delivered in random fragments over several calls end at crc32_long of the whole."""
    import annety_amd
    import torch

    rng = np.random.default_rng(78)
    ns = 500
    total = rng.integers(0, 40000, ns)
    bodies = [oracle.lcg_bytes(int(t), 1000 + i) for i, t in enumerate(total)]
    cuts = [np.sort(rng.integers(0, int(t) + 1, 4)) for t in total]
    sc = annety_amd.StreamingCrc(ns, gpu)
    for call in range(5):
        frags = []
        for i in range(ns):
            edges = np.concatenate([[0], cuts[i], [total[i]]])
            frags.append(bodies[i][edges[call] : edges[call + 1]])
        lens = np.array([f.size for f in frags], dtype=np.int32)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        arena = np.concatenate(frags + [np.zeros(1, np.uint8)])
        sc.update(to_dev(arena, gpu), to_dev(offs, gpu), to_dev(lens, gpu))
    got = digests(sc.digests())
    want = np.array([oracle.crc32_long(b) for b in bodies], dtype=np.uint32)
    assert np.array_equal(got, want)


def test_update_batch_fixed_odd_shapes(gpu):
    """Raw update over shapes the aligned kernel does not take (general kernel, update mode)."""
    import annety_amd
    import torch

    rng = np.random.default_rng(79)
    host = oracle.lcg_bytes(1 << 20, 55)
    d = to_dev(host, gpu)
    for n, L, stride, off in [(100, 1000, 1003, 1), (7, 3, 5, 2), (33, 4097, 4097, 0), (5, 100000, 100001, 3)]:
        states = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
        d_state = to_dev(states.view(np.int32), gpu)
        annety_amd.crc32_update_batch(d_state, d[off:], n, L, stride)
        want = [oracle.crc32_update(int(states[i]), host[off + i * stride : off + i * stride + L]) for i in range(n)]
        assert [int(x) for x in digests(d_state)] == want, (n, L, stride, off)


def test_host_registrations(gpu):
    """annety_crc_host_register: page-aligned ranges only, no two sharing a page; only buffers pinned here
    are DMA'd in place, anything else (a view that leaves the pinned range, memory after unregister) goes
    through the pack - the digests are the same either way."""
    import ctypes
    import mmap

    import annety_amd
    from annety_amd import _lib

    lib = _lib.get()
    pg = mmap.PAGESIZE
    m = mmap.mmap(-1, 8 * pg)
    buf = np.frombuffer(m, dtype=np.uint8)
    buf[:] = oracle.lcg_bytes(buf.size, 91)
    base = buf.ctypes.data
    assert lib.annety_crc_host_register(base, 2 * pg + 100) == 0
    assert lib.annety_crc_host_register(base + 2 * pg, pg) == -1  # shares the first range's last page
    assert lib.annety_crc_host_register(base + pg, pg) == -1       # inside it
    assert lib.annety_crc_host_register(base + 3 * pg, 2 * pg) == 0
    assert lib.annety_crc_host_unregister(base + pg) == -1         # not a range start
    n, L = 40, 64
    want = oracle.batch_fixed(buf, n, L)
    assert np.array_equal(annety_amd.crc32_batch_host(buf[: n * L], n, L), want)  # inside range 1: in place
    want2 = oracle.batch_fixed(buf[2 * pg:], 100, 64)
    assert np.array_equal(annety_amd.crc32_batch_host(buf[2 * pg: 2 * pg + 6400], 100, 64), want2)  # spans both
    assert lib.annety_crc_host_unregister(base) == 0
    assert lib.annety_crc_host_unregister(base + 3 * pg) == 0
    assert lib.annety_crc_host_unregister(base) == -1
    assert np.array_equal(annety_amd.crc32_batch_host(buf[: n * L], n, L), want)
    p = annety_amd.PinnedHostBuffer(3 * pg + 5)
    assert p.array.ctypes.data % pg == 0 and p.array.size == 3 * pg + 5
    p.array[:] = buf[: p.array.size]
    assert np.array_equal(annety_amd.crc32_batch_host(p.array, n, L), want)
    p.close()
    del buf
    m.close()
