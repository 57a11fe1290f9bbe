"""Host frame walks (crc32_capi.cpp FrameWalks) against a plain sequential walk written here from
LengthHeaderCodec::decode (include/codec/LengthHeaderCodec.h:71-137: signed big-endian length of T bytes,
length in [4, max_payload] when max_payload > 0, stop on an incomplete frame) and ProtobufCodec's framing
(include/protobuf/ProtobufCodec.h:149-153: T = 4, length in [10, 64 MiB]).

With the walk segment at its 4 KiB minimum, every buffer here is cut into many segments whose walks start
from speculative entries, so these cases exercise the join: random payloads (entries right), payloads made
of header-like bytes (entries wrong, the join redoes the segments), an invalid length, an incomplete tail,
frame caps that cut inside later segments. No GPU needed."""
import numpy as np
import pytest

import annety_amd
from annety_amd.codec import LengthHeaderCodec, ProtobufCodecFrames as ProtobufCodec


def ref_walk(buf: bytes, T: int, lo: int, hi: int, cap: int):
    pos, offs, lens, invalid = 0, [], [], False
    while len(offs) < cap and len(buf) - pos >= T:
        L = int.from_bytes(buf[pos:pos + T], "big", signed=True)
        if L < lo or (hi > 0 and L > hi):
            invalid = True
            break
        if len(buf) - pos - T < L:
            break
        offs.append(pos + T)
        lens.append(L - 4)
        pos += T + L
    return offs, lens, pos, invalid


def make_stream(seed: int, T: int, n: int, maxlen: int, filler=None) -> bytes:
    rng = np.random.default_rng(seed)
    out = bytearray()
    for _ in range(n):
        L = int(rng.integers(0, maxlen + 1))
        body = bytes(filler(L)) if filler else rng.integers(0, 256, L + 4, dtype=np.uint8).tobytes()[:L]
        out += (L + 4).to_bytes(T, "big", signed=True) + body + rng.integers(0, 256, 4, dtype=np.uint8).tobytes()
    return bytes(out)


@pytest.fixture
def small_segments():
    annety_amd.set_walk_segment(4096)
    yield
    annety_amd.set_walk_segment(0)


def _check(codec, buf, T, lo, hi, cap=None):
    got_off, got_len, used, invalid = codec.parse(buf, max_frames=cap)
    want = ref_walk(buf, T, lo, hi, len(buf) if cap is None else cap)
    assert np.array_equal(got_off, np.array(want[0], dtype=np.uint64))
    assert np.array_equal(got_len, np.array(want[1], dtype=np.uint32))
    assert (used, invalid) == (want[2], want[3])
    return len(want[0])


@pytest.mark.parametrize("T,maxlen", [(1, 123), (2, 3000), (4, 9000), (8, 9000)])
def test_random_payloads(small_segments, T, maxlen):
    buf = make_stream(T, T, 2000 if T > 1 else 9000, maxlen)
    assert _check(LengthHeaderCodec(T), buf, T, 4, 64 << 20) > 100


def test_no_payload_limit(small_segments):
    buf = make_stream(5, 4, 400, 20000)
    _check(LengthHeaderCodec(4, max_payload=0), buf, 4, 4, 0)


def test_header_like_payloads(small_segments):
    """Payload bytes that parse as chains of valid headers everywhere: the speculative entries are wrong and
    the join walks those segments itself."""
    pattern = lambda L: (b"\x00\x00\x01\x00" * (L // 4 + 1))[:L]  # noqa: E731 (length 256 at every 4th byte)
    buf = make_stream(6, 4, 600, 6000, filler=pattern)
    _check(LengthHeaderCodec(4), buf, 4, 4, 64 << 20)
    pattern2 = lambda L: (b"\x00\x00\x00\x08" * (L // 4 + 1))[:L]  # noqa: E731 (length 8: chains of 12 bytes)
    buf = make_stream(7, 4, 600, 6000, filler=pattern2)
    _check(LengthHeaderCodec(4), buf, 4, 4, 64 << 20)


def test_invalid_length_in_a_later_segment(small_segments):
    buf = bytearray(make_stream(8, 4, 1500, 4000))
    off, ln, _, _ = LengthHeaderCodec(4).parse(bytes(buf))
    k = int(len(off) * 0.7)
    buf[int(off[k]) - 4:int(off[k])] = (2).to_bytes(4, "big")  # length 2 < min_payload 4
    assert _check(LengthHeaderCodec(4), bytes(buf), 4, 4, 64 << 20) == k


def test_incomplete_tail_and_caps(small_segments):
    buf = make_stream(9, 4, 1500, 4000)
    codec = LengthHeaderCodec(4)
    _check(codec, buf[:-1000], 4, 4, 64 << 20)
    for cap in (1, 3, 700, 1111, 1499, 1500, 5000):
        _check(codec, buf, 4, 4, 64 << 20, cap=cap)


def test_tiny_buffers(small_segments):
    codec = LengthHeaderCodec(4)
    for buf in (b"", b"\x00", b"\x00\x00\x00\x05", b"\x00\x00\x00\x04abcd", b"\xff\xff\xff\xff"):
        _check(codec, buf, 4, 4, 64 << 20)


def test_protobuf_framing(small_segments):
    buf = make_stream(10, 4, 1500, 5000)
    got_off, got_len, used, invalid = ProtobufCodec().parse(buf)
    want = ref_walk(buf, 4, 10, 64 << 20, len(buf))
    assert np.array_equal(got_off, np.array(want[0], dtype=np.uint64))
    assert (used, invalid) == (want[2], want[3])


def test_default_segment_matches(small_segments):
    """The same buffer with the default segment (walked whole) and with 4 KiB segments."""
    buf = make_stream(11, 4, 3000, 5000)
    a = LengthHeaderCodec(4).parse(buf)
    annety_amd.set_walk_segment(0)
    b = LengthHeaderCodec(4).parse(buf)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2:] == b[2:]


def test_many_tiny_frames_past_the_first_bound():
    """Empty payloads (8-byte frames): more frames than the wrapper's first output bound (codec._frame_caps),
    so the call is repeated with the worst-case bound and still returns every frame."""
    n = 100_000
    buf = b"\x00\x00\x00\x04\x00\x00\x00\x00" * n
    off, ln, used, invalid = LengthHeaderCodec(4).parse(buf)
    assert off.size == n and int(ln.max()) == 0 and used == len(buf) and not invalid
    assert np.array_equal(off[:3], np.array([4, 12, 20], dtype=np.uint64))


def test_concurrent_parses_share_the_walk_pool(small_segments):
    """Several threads parsing at once: their segment walks share the persistent walk pool (each caller
    also takes its own queued walks), and every result equals the sequential walk."""
    import threading

    bufs = [make_stream(20 + i, 4, 800, 6000) for i in range(6)]
    want = [ref_walk(b, 4, 4, 64 << 20, len(b)) for b in bufs]
    errors = []

    def work(i):
        try:
            for _ in range(3):
                off, ln, used, invalid = LengthHeaderCodec(4).parse(bufs[i])
                w = want[i]
                assert np.array_equal(off, np.array(w[0], dtype=np.uint64)) and (used, invalid) == (w[2], w[3])
        except Exception as e:  # noqa: BLE001 (reported below)
            errors.append(e)

    threads = [threading.Thread(target=work, args=(i,)) for i in range(len(bufs))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors, errors
