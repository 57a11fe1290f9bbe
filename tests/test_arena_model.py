"""CPU model of the arena path (crc32_arena_lines.h + crc32_arena.hip), step for step:
the line pass's block/superblock suffix CRCs S and SB over an arena at an arbitrary absolute address
(bytes outside it in its boundary lines read as zeros), and the stitch's virtual-register formulation -
two half-line windows, at most four map steps acc = M1(acc) ^ M2(X ^ Y) plus one per whole superblock,
and the final inverse shift. Checked against zlib.crc32 (crc32_long, include/Crc32c.h:58-69) and a
direct crc32_update (include/Crc32c.h:71-82) over every head/tail case the kernel distinguishes.
No GPU: this pins the math the kernels implement; tests/test_gpu_arena.py pins the kernels."""
import zlib

import numpy as np
import pytest

POLY = 0xEDB88320
T256 = []
for _e in range(256):
    _c = _e
    for _ in range(8):
        _c = (_c >> 1) ^ (POLY & -(_c & 1))
    T256.append(_c & 0xFFFFFFFF)


def raw(data: bytes, s: int = 0) -> int:
    """Register after absorbing `data` from register s (no init, no final xor)."""
    for b in data:
        s = T256[(s ^ b) & 0xFF] ^ (s >> 8)
    return s


def _cols(nbytes: int):
    return [raw(bytes(nbytes), 1 << i) for i in range(32)]  # image of each bit: shift_nbytes


def _apply(cols, x: int) -> int:
    r = 0
    i = 0
    while x:
        if x & 1:
            r ^= cols[i]
        x >>= 1
        i += 1
    return r


def _inverse(cols):
    rows = [sum(((cols[c] >> r) & 1) << c for c in range(32)) | (1 << (32 + r)) for r in range(32)]
    for c in range(32):
        p = next(r for r in range(c, 32) if (rows[r] >> c) & 1)
        rows[c], rows[p] = rows[p], rows[c]
        for r in range(32):
            if r != c and (rows[r] >> c) & 1:
                rows[r] ^= rows[c]
    return [sum(((rows[r] >> (32 + c)) & 1) << r for r in range(32)) for c in range(32)]


_SH, _UN = {}, {}


def shift(x: int, n: int) -> int:
    if n not in _SH:
        _SH[n] = _cols(n)
    return _apply(_SH[n], x)


def unshift(x: int, n: int) -> int:
    if n not in _UN:
        _UN[n] = _inverse(_cols(n))
    return _apply(_UN[n], x)


class Arena:
    """The line pass: absolute 128-byte lines, 1 KiB blocks, 8 KiB superblocks."""

    def __init__(self, data: bytes, addr: int):
        self.data, self.lo, self.hi = data, addr, addr + len(data)

    def byte(self, a: int) -> int:
        return self.data[a - self.lo] if self.lo <= a < self.hi else 0

    def line(self, i: int) -> bytes:
        return bytes(self.byte(a) for a in range(i * 128, i * 128 + 128))

    def S(self, b: int, a: int) -> int:  # raw(lines a..7 of block b); S[8] = 0
        return raw(b"".join(self.line(b * 8 + x) for x in range(a, 8))) if a < 8 else 0

    def SB(self, s: int, g: int) -> int:  # raw(blocks g..7 of superblock s); SB[8] = 0
        return raw(b"".join(self.line(s * 64 + x) for x in range(g * 8, 64))) if g < 8 else 0


def stitch(ar: Arena, A: int, E: int, s0: int) -> int:
    """The stitch kernel's arithmetic for payload [A, E) (absolute addresses inside the arena)."""
    L0, L1 = A >> 7, (E - 1) >> 7
    lead, te = A & 127, ((E - 1) & 127) + 1
    head_x, tail_x = lead < 64, te >= 64
    line_lo, line_hi = ar.lo >> 7, (ar.hi - 1) >> 7
    cl = lambda L: (ar.lo & 127) if L == line_lo else 0  # noqa: E731
    ch = lambda L: ((ar.hi - 1) & 127) + 1 if L == line_hi else 128  # noqa: E731

    def window(L, off, keep_lo, keep_hi):  # 64-byte window of line L with bytes outside [keep) zeroed
        return bytes(ar.byte(L * 128 + off + i) if keep_lo <= off + i < keep_hi else 0 for i in range(64))

    wh = raw(window(L0, 0, cl(L0), lead)) if head_x else raw(window(L0, 64, lead, ch(L0)))
    wt = raw(window(L1, 64, te, ch(L1))) if tail_x else raw(window(L1, 0, cl(L1), te))
    # head: V(first line start) or V(first line end)
    acc = unshift(s0, lead) ^ unshift(wh, 64) if head_x else unshift(shift(s0, 128), lead) ^ wh
    I0, I1 = L0 + (0 if head_x else 1), L1 - (0 if tail_x else 1)
    F = lambda x, m: shift(x, 128 * m)  # noqa: E731
    G = lambda x, m: shift(x, 1024 * m)  # noqa: E731
    UL = lambda x, q: unshift(x, 128 * q)  # noqa: E731
    UB = lambda x, q: unshift(x, 1024 * q)  # noqa: E731
    if I1 >= I0:
        b0, a, b1, z = I0 >> 3, I0 & 7, I1 >> 3, I1 & 7
        if b0 == b1:  # step 0, whole run inside one block
            acc = F(acc, z - a + 1) ^ UL(ar.S(b0, a) ^ ar.S(b0, z + 1), 7 - z)
        else:
            acc = F(acc, 8 - a) ^ ar.S(b0, a)  # step 0: head block
            if b1 >= b0 + 2:
                B0, B1 = b0 + 1, b1 - 1
                s0_, g0, s1_, g1 = B0 >> 3, B0 & 7, B1 >> 3, B1 & 7
                if s0_ == s1_:  # step 1, the block run inside one superblock
                    acc = G(acc, g1 - g0 + 1) ^ UB(ar.SB(s0_, g0) ^ ar.SB(s0_, g1 + 1), 7 - g1)
                else:
                    acc = G(acc, 8 - g0) ^ ar.SB(s0_, g0)  # step 1
                    for s in range(s0_ + 1, s1_):  # whole superblocks
                        acc = G(acc, 8) ^ ar.SB(s, 0)
                    acc = G(acc, g1 + 1) ^ UB(ar.SB(s1_, 0) ^ ar.SB(s1_, g1 + 1), 7 - g1)  # step 2
            acc = F(acc, z + 1) ^ UL(ar.S(b1, 0) ^ ar.S(b1, z + 1), 7 - z)  # step 3: tail block
    # tail: drop the bytes after E
    return unshift(acc ^ wt, 128 - te) if tail_x else unshift(shift(acc, 128) ^ shift(wt, 64), 128 - te)


@pytest.mark.parametrize("addr", [8192 * 5, 8192 * 5 + 37, 8192 * 7 - 200])
def test_stitch_model_matches_crc(addr):
    rng = np.random.default_rng(addr)
    data = rng.integers(0, 256, 3 * 8192 + 700, dtype=np.uint8).tobytes()
    ar = Arena(data, addr)
    n = len(data)
    cases = [(0, n), (0, 1), (n - 1, n), (0, 64), (63, 65), (64, 128), (127, 129), (5, 1030), (1000, 9000)]
    for _ in range(60):
        a = int(rng.integers(0, n))
        cases.append((a, int(rng.integers(a + 1, min(n, a + 20000) + 1))))
    for a, e in cases:
        payload = data[a:e]
        got = stitch(ar, addr + a, addr + e, 0xFFFFFFFF) ^ 0xFFFFFFFF
        assert got == zlib.crc32(payload), (addr, a, e)
        s0 = int(rng.integers(0, 2**32))
        assert stitch(ar, addr + a, addr + e, s0) == raw(payload, s0), (addr, a, e, "update")


def test_every_head_and_tail_case():
    """lead < 64 / >= 64 and te >= 64 / < 64, single-line payloads, one-block, one-superblock runs."""
    addr = 8192 * 3 + 100
    data = bytes((i * 7 + 3) & 0xFF for i in range(20000))
    ar = Arena(data, addr)
    for a in (0, 1, 27, 63, 64, 65, 100, 127, 128, 130):
        for ln in (1, 2, 30, 63, 64, 65, 127, 128, 129, 300, 1024, 1100, 8192, 9000):
            if a + ln <= len(data):
                assert stitch(ar, addr + a, addr + a + ln, 0xFFFFFFFF) ^ 0xFFFFFFFF == zlib.crc32(data[a:a + ln])
