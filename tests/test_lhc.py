"""LengthHeaderCodec batch path.

CPU tests pin the oracle's codec restatement to fixtures recorded from the reference's own
LengthHeaderCodec (tests/golden/lhc.json, tests/golden/make_lhc_golden.py) and check the host logic
of the C-ABI (header walk, encode plan, recv outcome). GPU tests run decode/encode through the C-ABI
and compare with the fixtures and the oracle.
"""
import numpy as np
import pytest

import oracle
from annety_amd.codec import LengthHeaderCodec, recv_result


def _payload(n, seed):
    return oracle.lcg_bytes(n, seed).tobytes()


def _expected_encode(c):
    if c["out_len"] == 0:
        return b""
    return bytes.fromhex(c["header"]) + _payload(c["len"], c["seed"]) + bytes.fromhex(c["trailer"])


# ---------------- oracle vs the reference's recorded behaviour ----------------
def test_oracle_encode_matches_reference(golden):
    g = golden("lhc.json")
    assert len(g["encode"]) >= 100
    for c in g["encode"]:
        rt, out = oracle.lhc_encode(_payload(c["len"], c["seed"]), c["T"], c["max_payload"])
        assert rt == c["rt"], c
        assert out == _expected_encode(c), c


def test_oracle_recv_matches_reference(golden):
    for c in golden("lhc.json")["decode"]:
        frames, used, rt = oracle.lhc_recv(bytes.fromhex(c["stream"]), c["T"], c["max_payload"])
        assert [list(f) for f in frames] == c["frames"], c["name"]
        assert (used, rt) == (c["consumed"], c["rt"]), c["name"]


# ---------------- host logic of the C-ABI (no device work) ----------------
def _cpu_verdicts(stream, off, ln):
    """Test-side checksum verdicts from the oracle, standing in for the device verify."""
    s = np.frombuffer(stream, dtype=np.uint8)
    ok = np.zeros(off.size, dtype=np.uint8)
    for i, (o, n) in enumerate(zip(off.tolist(), ln.tolist())):
        want = int.from_bytes(stream[o + n : o + n + 4], "big")
        ok[i] = oracle.crc32_long(s[o : o + n]) == want
    return ok


def test_parse_and_recv_outcome_match_reference(golden):
    for c in golden("lhc.json")["decode"]:
        codec = LengthHeaderCodec(c["T"], True, c["max_payload"])
        stream = bytes.fromhex(c["stream"])
        off, ln, used, invalid = codec.parse(stream)
        r = recv_result(c["T"], off, ln, used, invalid, _cpu_verdicts(stream, off, ln))
        assert [[int(o), int(n)] for o, n in zip(r.payload_off, r.payload_len)] == c["frames"], c["name"]
        assert (r.consumed, r.rt) == (c["consumed"], c["rt"]), c["name"]


def test_parse_walks_every_frame_of_a_long_stream():
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 3000, size=2000)
    lens[::7] = 0
    for T in (2, 4, 8):
        stream = b"".join(oracle.lhc_encode(_payload(int(n), i), T)[1] for i, n in enumerate(lens))
        off, ln, used, invalid = LengthHeaderCodec(T).parse(stream)
        want = [int(n) for n in lens if n > 0]
        assert ln.tolist() == want and used == len(stream) and not invalid
        exp_off, pos = [], 0
        for n in want:
            exp_off.append(pos + T)
            pos += T + n + 4
        assert off.tolist() == exp_off
        # a truncated tail is left for the next read
        off2, ln2, used2, _ = LengthHeaderCodec(T).parse(stream[:-1])
        assert ln2.tolist() == want[:-1] and used2 == len(stream) - (T + want[-1] + 4)
        # max_frames bounds the walk
        off3, _, used3, _ = LengthHeaderCodec(T).parse(stream, max_frames=3)
        assert off3.size == 3 and used3 == exp_off[3] - T


def test_encode_plan_matches_reference(golden):
    for c in golden("lhc.json")["encode"]:
        off, rt, total = LengthHeaderCodec(c["T"], True, c["max_payload"]).plan(np.array([c["len"], 1]))
        assert int(rt[0]) == c["rt"] and int(off[0]) == 0
        assert int(off[1]) == c["out_len"], c
        assert total == c["out_len"] + c["T"] + 5


def test_codec_argument_checks():
    with pytest.raises(ValueError):
        LengthHeaderCodec(3)
    with pytest.raises(ValueError):
        LengthHeaderCodec(4, enable_checksum=False)
    off, ln, used, invalid = LengthHeaderCodec(4).parse(b"")
    assert off.size == 0 and used == 0 and not invalid


# ---------------- device path ----------------
@pytest.mark.gpu
def test_gpu_decode_matches_reference(golden, gpu):
    for c in golden("lhc.json")["decode"]:
        codec = LengthHeaderCodec(c["T"], True, c["max_payload"])
        r = codec.decode_batch(bytes.fromhex(c["stream"]), device=gpu)
        assert [[int(o), int(n)] for o, n in zip(r.payload_off, r.payload_len)] == c["frames"], c["name"]
        assert (r.consumed, r.rt) == (c["consumed"], c["rt"]), c["name"]


@pytest.mark.gpu
def test_gpu_encode_matches_reference(golden, gpu):
    import torch

    cases = golden("lhc.json")["encode"]
    for key in sorted({(c["T"], c["max_payload"]) for c in cases}):
        group = [c for c in cases if (c["T"], c["max_payload"]) == key]
        src = b"".join(_payload(c["len"], c["seed"]) for c in group)
        lens = np.array([c["len"] for c in group], dtype=np.uint32)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
        d_src = torch.frombuffer(bytearray(src) or bytearray(1), dtype=torch.uint8).to(gpu)
        r = LengthHeaderCodec(key[0], True, key[1]).encode_batch(d_src, offs, lens)
        assert r.rt.tolist() == [c["rt"] for c in group]
        assert r.frames.cpu().numpy().tobytes() == b"".join(_expected_encode(c) for c in group), key


@pytest.mark.gpu
def test_gpu_encode_decode_round_trip_and_corruption(gpu):
    import torch

    rng = np.random.default_rng(11)
    n = 20000
    lens = rng.integers(0, 2500, size=n).astype(np.uint32)
    lens[rng.integers(0, n, size=50)] = rng.integers(60000, 200000, size=50)
    # payloads at arbitrary (unaligned) offsets inside one arena
    gaps = rng.integers(0, 5, size=n)
    offs = np.cumsum(np.concatenate([[0], (lens + gaps)[:-1]])).astype(np.uint64)
    arena = oracle.lcg_bytes(int(offs[-1] + lens[-1]) + 8, 99)
    d_src = torch.from_numpy(arena.copy()).to(gpu)
    for T in (4, 8):
        codec = LengthHeaderCodec(T)
        r = codec.encode_batch(d_src, offs, lens)
        frames = r.frames.cpu().numpy().tobytes()
        want = b"".join(oracle.lhc_encode(arena[int(o) : int(o) + int(L)], T)[1] for o, L in zip(offs, lens))
        assert frames == want
        d = codec.decode_batch(frames, d_stream=r.frames)
        assert d.rt == 0 and d.consumed == len(frames) and d.ok.all()
        assert d.payload_len.tolist() == [int(L) for L in lens if L]
        # corrupt one payload byte deep in the stream: frames before it are delivered, then -1
        k = int(d.payload_off.size * 2 // 3)
        bad = bytearray(frames)
        bad[int(d.payload_off[k]) + int(d.payload_len[k]) // 2] ^= 0x04
        e = codec.decode_batch(bytes(bad), device=gpu)
        assert e.rt == -1 and e.payload_off.size == k and e.consumed == int(d.payload_off[k]) - T
        assert int((e.ok == 0).sum()) == 1
