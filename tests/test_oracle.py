"""The CPU oracle (oracle/crc32_oracle.c) pinned against the compiled reference's golden fixtures
(tests/golden/*.json, written by tests/golden/make_golden.py from /root/reference/src/Crc32c.cc) and
against Python's zlib.crc32 (an independent implementation of the same CRC-32/ISO-HDLC)."""
import zlib

import numpy as np
import pytest

import oracle


def H(x: str) -> int:
    return int(x, 16)


def test_tables_match_reference(golden):
    k = golden("kat.json")
    t256, t16 = oracle.tables()
    assert [int(x) for x in t256] == [H(x) for x in k["table256"]]
    assert [int(x) for x in t16] == [H(x) for x in k["table16"]]
    assert int(t256[1]) == 0x77073096  # src/Crc32c.cc:28: IEEE, not Castagnoli


def test_kats(golden):
    k = golden("kat.json")
    for kat in k["kats"]:
        data = bytes.fromhex(kat["hex"])
        assert oracle.crc32_long(data) == H(kat["crc32_long"]), kat["name"]
        assert oracle.crc32_short(data) == H(kat["crc32_short"]), kat["name"]
        assert zlib.crc32(data) == H(kat["crc32_long"]), kat["name"]
    assert oracle.crc32_long(b"123456789") == 0xCBF43926
    assert oracle.crc32_update(0, b"123456789") == H(k["update"]["from_zero_123456789"])
    s = oracle.crc32_update(oracle.crc32_update(0xFFFFFFFF, b"1234"), b"56789")
    assert s ^ 0xFFFFFFFF == H(k["update"]["split_4_5_final"])


def test_lcg_batch(golden):
    g = golden("lcg_1024x1k.json")
    arena = oracle.lcg_bytes(g["n"] * g["len"], g["seed"])
    assert arena[:4].tolist() == g["first_bytes"]
    d = oracle.batch_fixed(arena, g["n"], g["len"])
    assert [int(x) for x in d] == [H(x) for x in g["digests"]]
    assert int(np.bitwise_xor.reduce(d)) == H(g["xor_all"])
    assert oracle.crc32_long(arena) == H(g["arena_crc"])
    mt = oracle.batch_fixed_mt(arena, g["n"], g["len"], threads=4)
    assert np.array_equal(mt, d)


def test_lengths_and_unaligned(golden):
    g = golden("lengths.json")
    arena = oracle.lcg_bytes(g["arena_bytes"], g["seed"])
    for row in g["rows"]:
        s = row["start"]
        offs = np.full(len(g["lengths"]), s, dtype=np.uint64)
        got = oracle.batch_var(arena, offs, np.array(g["lengths"], dtype=np.uint32))
        assert [int(x) for x in got] == [H(x) for x in row["crc"]], f"start {s}"
        # short == long on the same inputs, spot-check the short range
        for ln, want in zip(g["lengths"][:80], row["crc"][:80]):
            assert oracle.crc32_short(arena[s:s + ln]) == H(want)


def test_fixed_batches(golden):
    g = golden("fixed_batches.json")
    arena = oracle.lcg_bytes(g["arena_bytes"], g["seed"])
    for c in g["cases"]:
        got = oracle.batch_fixed(arena, c["n"], c["len"], c["stride"])
        assert [int(x) for x in got] == [H(x) for x in c["digests"]], c


def test_big(golden):
    for c in golden("big.json")["cases"]:
        b = oracle.lcg_bytes(c["bytes"], c["seed"])
        assert oracle.crc32_long(b) == H(c["crc"])
        assert zlib.crc32(b.tobytes()) == H(c["crc"])


def test_zipf(golden):
    g = golden("zipf.json")
    arena = oracle.lcg_bytes(g["total_bytes"], g["seed_bytes"])
    got = oracle.batch_var(arena, np.array(g["offsets"], dtype=np.uint64), np.array(g["lengths"], dtype=np.uint32))
    assert [int(x) for x in got] == [H(x) for x in g["digests"]]


def test_update_fragments(golden):
    g = golden("update_fragments.json")
    arena = oracle.lcg_bytes(g["arena_bytes"], g["seed"])
    for c in g["cases"]:
        st = 0xFFFFFFFF
        for a, b in zip(c["cuts"][:-1], c["cuts"][1:]):
            st = oracle.crc32_update(st, arena[a:b])
        assert st == H(c["final_state"])
        assert st ^ 0xFFFFFFFF == H(c["crc"])


def test_combine(golden):
    for c in golden("combine.json")["cases"]:
        assert oracle.crc32_combine(H(c["crcA"]), H(c["crcB"]), c["lenB"]) == H(c["crcAB"]), c


@pytest.mark.skipif(not oracle.ref_available(), reason="compiled reference not present (GPU box)")
def test_oracle_equals_compiled_reference_random():
    ref = oracle.ref_lib()
    rng = np.random.default_rng(3)
    for _ in range(300):
        n = int(rng.integers(0, 3000))
        a = rng.integers(0, 256, n, dtype=np.uint8)
        assert oracle.crc32_long(a) == ref.ref_crc32_long(a.ctypes.data, n)
        assert oracle.crc32_short(a) == ref.ref_crc32_short(a.ctypes.data, n)


@pytest.mark.skipif(not oracle.ref_available(), reason="compiled reference not present (GPU box)")
def test_compiled_reference_var_batch_mt():
    """The reference's own crc32_long/short over a variable batch on several threads (bench.py's config-3
    cpu_baseline leg, kind "reference") equals the oracle, including empty and <= 60-byte payloads."""
    ref = oracle.ref_lib()
    rng = np.random.default_rng(11)
    lens = rng.integers(0, 5000, 3001).astype(np.uint32)
    lens[:5] = [0, 1, 60, 61, 0]
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64))[:-1]]).astype(np.uint64)
    buf = oracle.lcg_bytes(int(lens.sum()), 19)
    want = oracle.batch_var(buf, offs, lens)
    for threads in (1, 3, 16):
        out = np.zeros(lens.size, dtype=np.uint32)
        assert ref.ref_crc32_batch_var_mt(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, lens.size,
                                          out.ctypes.data, threads) == 0
        assert np.array_equal(out, want), threads
