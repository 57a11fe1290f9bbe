"""Arena path (annety_crc32_batch_var_arena / _update_ / annety_lhc_verify_stream):
one payload-agnostic pass over the arena's lines, then a per-payload stitch. Checked bit-exactly
against the golden fixtures written by the compiled reference and against the oracle, including
every length 0..300 at 12 start alignments, payloads crossing 1 KiB / 8 KiB unit boundaries, payloads
outside the declared arena (direct-fold fallback), an empty arena, and update-mode registers."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def H(x: str) -> int:
    return int(x, 16)


def to_dev(arr, device):
    import torch

    return torch.from_numpy(np.ascontiguousarray(arr)).to(device)


def u32(t):
    import torch

    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint32)


def test_arena_lengths_golden(golden, gpu):
    import torch

    import annety_amd

    g = golden("lengths.json")
    arena = to_dev(oracle.lcg_bytes(g["arena_bytes"], g["seed"]), gpu)
    lens = torch.tensor(g["lengths"], dtype=torch.int32, device=gpu)
    for row in g["rows"]:
        offs = torch.full((len(g["lengths"]),), row["start"], dtype=torch.int64, device=gpu)
        got = u32(annety_amd.crc32_batch_var(arena, offs, lens, arena=True))
        want = np.array([H(x) for x in row["crc"]], dtype=np.uint32)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"start {row['start']}: lengths {[g['lengths'][i] for i in bad[:10]]}"


def test_arena_zipf_golden(golden, gpu):
    import torch

    import annety_amd

    g = golden("zipf.json")
    arena = to_dev(oracle.lcg_bytes(g["total_bytes"], g["seed_bytes"]), gpu)
    offs = torch.tensor(g["offsets"], dtype=torch.int64, device=gpu)
    lens = torch.tensor(g["lengths"], dtype=torch.int32, device=gpu)
    got = u32(annety_amd.crc32_batch_var(arena, offs, lens, arena=True))
    assert [int(x) for x in got] == [H(x) for x in g["digests"]]


def _random_batch(rng, n, max_len, arena_bytes):
    lens = rng.integers(0, max_len + 1, n)
    offs = rng.integers(0, arena_bytes - max_len, n)
    return offs.astype(np.int64), lens.astype(np.int64)


def test_arena_unit_boundaries(gpu):
    """Payloads straddling the 128 B / 1 KiB / 8 KiB units of the arena pass in every way: random
    starts, lengths up to 200 KiB (c64 steps), overlapping and out-of-order payloads."""
    import annety_amd

    rng = np.random.default_rng(11)
    nbytes = 4 << 20
    host = oracle.lcg_bytes(nbytes, 99)
    d = to_dev(host, gpu)
    for max_len in (300, 5000, 70000, 200000):
        offs, lens = _random_batch(rng, 3000, max_len, nbytes)
        got = u32(annety_amd.crc32_batch_var(d, to_dev(offs, gpu), to_dev(lens.astype(np.int32), gpu), arena=True))
        want = oracle.batch_var_mt(host, offs, lens, 8)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (max_len, offs[bad[:4]], lens[bad[:4]])


def test_arena_outside_and_empty(gpu):
    """Payloads beyond the declared arena bytes (and an empty arena) take the direct-fold path."""
    import annety_amd

    rng = np.random.default_rng(12)
    nbytes = 1 << 20
    host = oracle.lcg_bytes(nbytes, 7)
    d = to_dev(host, gpu)
    offs, lens = _random_batch(rng, 800, 20000, nbytes)
    want = oracle.batch_var_mt(host, offs, lens, 8)
    d_off, d_len = to_dev(offs, gpu), to_dev(lens.astype(np.int32), gpu)
    for arena in (nbytes // 3, 1, 0):
        got = u32(annety_amd.crc32_batch_var(d, d_off, d_len, arena=arena))
        assert np.array_equal(got, want), arena
    # offset base pointer: the arena starts mid-line
    sub = d[37:]
    offs2 = np.clip(offs - 37, 0, None)
    want2 = oracle.batch_var_mt(host[37:], offs2, np.minimum(lens, nbytes - 37 - offs2), 8)
    got2 = u32(annety_amd.crc32_batch_var(sub, to_dev(offs2, gpu),
                                          to_dev(np.minimum(lens, nbytes - 37 - offs2).astype(np.int32), gpu),
                                          arena=True))
    assert np.array_equal(got2, want2)


def test_arena_update(gpu):
    """crc32_update semantics (include/Crc32c.h:71-82) through the arena stitch: arbitrary registers,
    every length class including < 4-byte fragments; zero-length fragments keep their register."""
    import annety_amd

    rng = np.random.default_rng(13)
    n = 6000
    lens = np.concatenate([np.arange(0, 300), rng.integers(0, 5000, n - 400), rng.integers(16384, 70000, 100)])
    rng.shuffle(lens)
    offs = np.cumsum(np.concatenate([[0], lens[:-1] + rng.integers(0, 7, n - 1)])).astype(np.int64)
    host = oracle.lcg_bytes(int(offs[-1] + lens[-1]) + 16, 404)
    states = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    d_state = to_dev(states.view(np.int32), gpu)
    annety_amd.crc32_update_batch_var(d_state, to_dev(host, gpu), to_dev(offs, gpu), to_dev(lens.astype(np.int32), gpu),
                                      arena=True)
    want = oracle.batch_var_mt(host, offs, lens, 8, states=states)
    assert np.array_equal(u32(d_state), want)


def test_arena_streaming_fragments(gpu):
    """Streams in random fragments over several arena calls end at crc32_long of the whole."""
    import annety_amd

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
            frags.append(bodies[i][edges[call]: edges[call + 1]])
        lens = np.array([f.size for f in frags], dtype=np.int32)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        arena = np.concatenate(frags + [np.zeros(1, np.uint8)])
        sc.update(to_dev(arena, gpu), to_dev(offs, gpu), to_dev(lens, gpu), arena=True)
    got = u32(sc.digests())
    want = np.array([oracle.crc32_long(b) for b in bodies], dtype=np.uint32)
    assert np.array_equal(got, want)


def test_arena_partial_ends(gpu):
    """Arenas that start and end mid-line and mid-superblock, with nonzero bytes around them in the
    same lines: payloads touching the first and last arena byte, every start/end offset within the
    boundary lines, arenas inside one line, one superblock and across two (no whole superblock)."""
    import annety_amd

    rng = np.random.default_rng(21)
    host = oracle.lcg_bytes(3 << 20, 5)
    d = to_dev(host, gpu)
    for lo, size in ((37, 90), (5, 200), (8100, 300), (8190, 8200), (40, 16384 + 1000), (4096 + 77, (1 << 20) + 333),
                     (8192, 65536), (8192 + 64, (2 << 20) - 8192 - 64 - 13)):
        sub = d[lo:lo + size]
        offs, lens = [], []
        for a in range(0, min(size, 160)):  # starts in the first lines, ends anywhere
            offs.append(a)
            lens.append(int(rng.integers(0, size - a + 1)))
        for e in range(max(0, size - 160), size + 1):  # ends in the last lines
            a = int(rng.integers(0, e + 1))
            offs.append(a)
            lens.append(e - a)
        offs.append(0)
        lens.append(size)
        for _ in range(400):
            a = int(rng.integers(0, size))
            offs.append(a)
            lens.append(int(rng.integers(0, size - a + 1)))
        offs = np.array(offs, np.int64)
        lens = np.array(lens, np.int64)
        want = oracle.batch_var_mt(host[lo:lo + size], offs, lens, 8)
        got = u32(annety_amd.crc32_batch_var(sub, to_dev(offs, gpu), to_dev(lens.astype(np.int32), gpu), arena=True))
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (lo, size, offs[bad[:4]], lens[bad[:4]])
        st = rng.integers(0, 2 ** 32, offs.size, dtype=np.uint64).astype(np.uint32)
        d_state = to_dev(st.view(np.int32), gpu)
        annety_amd.crc32_update_batch_var(d_state, sub, to_dev(offs, gpu), to_dev(lens.astype(np.int32), gpu),
                                          arena=True)
        assert np.array_equal(u32(d_state), oracle.batch_var_mt(host[lo:lo + size], offs, lens, 8, states=st)), (lo, size)
