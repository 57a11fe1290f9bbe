"""Generate the golden fixtures in tests/golden/ from the COMPILED REFERENCE.

Run here (where /root/reference exists):   python tests/golden/make_golden.py
It builds oracle/_ref/libref_crc32.so from /root/reference/src/Crc32c.cc + include/Crc32c.h
(oracle/Makefile `ref` target) and records inputs (as generator specs or explicit lengths/offsets)
and the reference's outputs. Nothing here is copied reference source: every file written is data.

Payload bytes come from the SURVEY.md §8c LCG (oracle.lcg_bytes), so the GPU box can regenerate them
without the reference.
"""
from __future__ import annotations

import json
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

import oracle  # noqa: E402

oracle.build(ref=True)
ref = oracle.ref_lib()


def rlong(a: np.ndarray, want: int | None = None) -> int:
    a = np.ascontiguousarray(a, dtype=np.uint8)
    if want is not None:
        assert a.size == want, "fixture slice out of range"
    return int(ref.ref_crc32_long(a.ctypes.data, a.size))


def rshort(a: np.ndarray) -> int:
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return int(ref.ref_crc32_short(a.ctypes.data, a.size))


def rupdate(state: int, a: np.ndarray) -> int:
    import ctypes

    a = np.ascontiguousarray(a, dtype=np.uint8)
    s = ctypes.c_uint32(state)
    ref.ref_crc32_update(ctypes.byref(s), a.ctypes.data, a.size)
    return int(s.value)


def u8(b: bytes) -> np.ndarray:
    return np.frombuffer(b, dtype=np.uint8)


def h(x: int) -> str:
    return f"{x:08x}"


def dump(name: str, obj) -> None:
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", name)


# ---- 1. known-answer tests (include/Crc32c.h:41-82) ----
kat_inputs = {
    "empty": b"",
    "a": b"a",
    "check_123456789": b"123456789",
    "quick_brown_fox": b"The quick brown fox jumps over the lazy dog",
    "bytes_0_255": bytes(range(256)),
    "zeros_1k": bytes(1024),
    "ff_1k": b"\xff" * 1024,
    "ramp_1k": bytes(i & 0xFF for i in range(1024)),
    "hello_world_frame": b"hello-world",
}
kats = []
for name, data in kat_inputs.items():
    a = u8(data)
    kats.append({"name": name, "hex": data.hex(), "crc32_long": h(rlong(a)), "crc32_short": h(rshort(a)),
                 "zlib": h(zlib.crc32(data))})
upd = {
    "from_zero_123456789": h(rupdate(0, u8(b"123456789"))),
    "split_4_5_final": h(rupdate(rupdate(0xFFFFFFFF, u8(b"1234")), u8(b"56789")) ^ 0xFFFFFFFF),
}
t256 = np.zeros(256, dtype=np.uint32)
t16 = np.zeros(16, dtype=np.uint32)
ref.ref_tables(t256.ctypes.data, t16.ctypes.data)
dump("kat.json", {"kats": kats, "update": upd, "table256": [h(int(x)) for x in t256],
                  "table16": [h(int(x)) for x in t16],
                  "source": "reference include/Crc32c.h + src/Crc32c.cc compiled by oracle/Makefile (ref)"})

# ---- 2. 1024 x 1 KiB LCG batch (config 0) ----
n, L = 1024, 1024
arena = oracle.lcg_bytes(n * L, 42)
dig = [rlong(arena[i * L:(i + 1) * L]) for i in range(n)]
x = 0
for d in dig:
    x ^= d
dump("lcg_1024x1k.json", {"seed": 42, "n": n, "len": L, "digests": [h(d) for d in dig], "xor_all": h(x),
                          "arena_crc": h(rlong(arena)), "first_bytes": arena[:4].tolist()})

# ---- 3. ragged lengths and unaligned starts over one arena ----
arena = oracle.lcg_bytes((1 << 16) + 256, 1234)
lengths = list(range(0, 301)) + list(range(301, 4097, 7)) + [4096, 8191, 8192, 16384, 65535, 65536 - 17]
starts = [0, 1, 2, 3, 5, 7, 13, 16, 63, 64, 127, 128]
rows = []
for s in starts:
    rows.append({"start": s, "crc": [h(rlong(arena[s:s + ln], ln)) for ln in lengths]})
dump("lengths.json", {"seed": 1234, "arena_bytes": (1 << 16) + 256, "lengths": lengths, "rows": rows})

# ---- 4. fixed-length batches of assorted lengths/strides (exercise G / round / tail layouts) ----
arena = oracle.lcg_bytes(1 << 22, 99)  # 4 MiB
cases = []
for (cn, clen, cstride) in [(64, 1024, 1024), (37, 2048, 2048), (100, 16, 16), (100, 48, 64), (50, 128, 128),
                            (33, 1040, 1056), (20, 4096, 4096), (9, 8192, 8192), (7, 12288, 12304),
                            (5, 65536, 65536), (3, 1000000, 1000016), (200, 1, 1), (64, 61, 61), (64, 60, 61),
                            (17, 129, 200), (8, 65520, 65536)]:
    digs = [rlong(arena[i * cstride:i * cstride + clen]) if clen > 60 else rshort(arena[i * cstride:i * cstride + clen])
            for i in range(cn)]
    cases.append({"n": cn, "len": clen, "stride": cstride, "digests": [h(d) for d in digs]})
dump("fixed_batches.json", {"seed": 99, "arena_bytes": 1 << 22, "cases": cases})

# ---- 5. big payloads (config 2 shape at reduced count; 64 MiB = LengthHeaderCodec max_payload) ----
big = []
for seed, nbytes in [(7, 4 << 20), (8, (4 << 20) + 12345), (9, 64 << 20)]:
    b = oracle.lcg_bytes(nbytes, seed)
    big.append({"seed": seed, "bytes": nbytes, "crc": h(rlong(b))})
dump("big.json", {"cases": big})

# ---- 6. Zipf mixed lengths, packed back-to-back (config 3 shape, reduced N) ----
# lengths: k ~ Zipf(s=1.1) over ranks 1..1024 (inverse CDF driven by the LCG), L = min(65536, 64k + r)
ranks = np.arange(1, 1025, dtype=np.float64)
cdf = np.cumsum(ranks ** -1.1)
cdf /= cdf[-1]
u = oracle.lcg_bytes(4 * 3000, 0x5EED).reshape(-1, 4).astype(np.uint64)
u32 = (u[:, 0] << 24) | (u[:, 1] << 16) | (u[:, 2] << 8) | u[:, 3]
lens = []
for i in range(0, 3000, 2):
    k = int(np.searchsorted(cdf, u32[i] / 2.0 ** 32)) + 1
    r = int(u32[i + 1] & 63)
    lens.append(min(65536, 64 * k + r))
lens = np.array(lens, dtype=np.uint64)
offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
total = int(lens.sum())
zarena = oracle.lcg_bytes(total, 0x5EED + 1)
zd = [rlong(zarena[int(o):int(o) + int(ln)]) for o, ln in zip(offs, lens)]
dump("zipf.json", {"seed_bytes": 0x5EED + 1, "lengths": [int(x) for x in lens], "offsets": [int(x) for x in offs],
                   "total_bytes": total, "digests": [h(d) for d in zd]})

# ---- 7. streaming update in fragments (crc32_update, include/Crc32c.h:71-82) ----
arena = oracle.lcg_bytes(1 << 15, 555)
frags = []
rng_state = 0
for t in range(40):
    cuts = sorted({int(c) for c in (oracle.lcg_bytes(8, 1000 + t).astype(np.int64) * 97) % (1 << 15)})
    cuts = [0] + cuts + [1 << 15]
    st = 0xFFFFFFFF
    for a_, b_ in zip(cuts[:-1], cuts[1:]):
        st = rupdate(st, arena[a_:b_])
    frags.append({"cuts": cuts, "final_state": h(st), "crc": h(st ^ 0xFFFFFFFF)})
dump("update_fragments.json", {"seed": 555, "arena_bytes": 1 << 15, "cases": frags})

# ---- 8. combine identity on reference digests ----
arena = oracle.lcg_bytes(1 << 16, 777)
comb = []
for a_ in [0, 1, 100, 3000, 4096, 30000]:
    for b_ in [0, 1, 7, 5192, 12345]:
        A = arena[:a_]
        B = arena[a_:a_ + b_]
        comb.append({"lenA": a_, "lenB": b_, "crcA": h(rlong(A)), "crcB": h(rlong(B)), "crcAB": h(rlong(arena[:a_ + b_]))})
dump("combine.json", {"seed": 777, "cases": comb})
