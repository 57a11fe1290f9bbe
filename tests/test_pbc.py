"""ProtobufCodec framing (include/protobuf/ProtobufCodec.h, checksum on), batched: the C-ABI's header walk
and encode plan against the oracle's restatement of ProtobufCodec::decode/encode (:127-247), and the
device verify/encode path on the GPU. Parity with the reference codec itself is UNPINNED: its header
needs libprotobuf, which is absent here, so the oracle restatement (line-cited) is the checker. The
boundary lengths 9/10 (min_payload), 64 MiB (max_payload) and the encode minimum of 6 are covered."""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

import oracle
from annety_amd.codec import ProtobufCodecFrames

MAXP = 64 * 1024 * 1024


def _stream(lengths, seed=5, corrupt=()):
    parts = []
    for i, L in enumerate(lengths):
        rt, fr = oracle.pbc_encode(oracle.lcg_bytes(L, seed + i))
        assert rt == 1
        fr = bytearray(fr)
        if i in corrupt:
            fr[4] ^= 1
        parts.append(bytes(fr))
    return b"".join(parts)


def test_oracle_limits():
    assert oracle.pbc_encode(b"")[0] == 0
    assert oracle.pbc_encode(b"x" * 5)[0] == -1  # < min_payload - checksum = 6
    assert oracle.pbc_encode(b"x" * 6)[0] == 1
    frames, used, rt = oracle.pbc_recv(bytes.fromhex("00000009") + b"\0" * 9)
    assert frames == [] and used == 0 and rt == -1  # length 9 < 10
    frames, used, rt = oracle.pbc_recv(bytes.fromhex("04000001"))
    assert rt == -1  # length 64 MiB + 1
    frames, used, rt = oracle.pbc_recv(bytes.fromhex("04000000"))
    assert rt == 0  # 64 MiB is valid, incomplete


def test_parse_matches_oracle():
    codec = ProtobufCodecFrames()
    lens = [6, 7, 60, 61, 1000, 70000, 6]
    s = _stream(lens)
    off, ln, used, invalid = codec.parse(s + b"\x00\x00")
    frames, oused, ort = oracle.pbc_recv(s + b"\x00\x00")
    assert [(int(o), int(n)) for o, n in zip(off, ln)] == frames and used == oused and not invalid
    for bad in (bytes.fromhex("00000009"), bytes.fromhex("ffffffff"), bytes.fromhex("04000001")):
        off, ln, used, invalid = codec.parse(s + bad)
        frames, oused, ort = oracle.pbc_recv(s + bad)
        assert invalid and ort == -1 and used == oused == len(s)


def test_plan_matches_oracle():
    codec = ProtobufCodecFrames()
    lens = np.array([0, 5, 6, 100, MAXP, MAXP + 1, 7], dtype=np.uint32)
    off, rt, total = codec.plan(lens)
    assert rt.tolist() == [0, -1, 1, 1, 1, -1, 1]
    sizes = [8 + int(L) if r == 1 else 0 for L, r in zip(lens, rt)]
    assert off.tolist() == np.concatenate([[0], np.cumsum(sizes)[:-1]]).tolist() and total == sum(sizes)


@settings(max_examples=60, deadline=None)
@given(st.lists(st.integers(0, 300), max_size=30), st.binary(max_size=12))
def test_property_walk_equals_oracle(lens, tail):
    lens = [L for L in lens if L >= 6]
    s = _stream(lens) + tail
    off, ln, used, invalid = ProtobufCodecFrames().parse(s)
    frames, oused, ort = oracle.pbc_recv(s)  # all checksums good: the walk alone decides
    assert [(int(o), int(n)) for o, n in zip(off, ln)] == frames
    assert used == oused and invalid == (ort == -1)


@pytest.mark.gpu
def test_gpu_pbc_decode_encode(gpu):
    import torch

    codec = ProtobufCodecFrames()
    lens = [6, 10, 61, 5000, 70000, 6, 123456, 8]
    s = _stream(lens, corrupt=(4,)) + bytes.fromhex("0000")
    r = codec.decode_host(s)
    frames, oused, ort = oracle.pbc_recv(s)
    assert [(int(o), int(n)) for o, n in zip(r.payload_off, r.payload_len)] == frames
    assert (r.consumed, r.rt) == (oused, ort) and r.ok.tolist() == [1, 1, 1, 1, 0, 1, 1, 1]
    d = torch.frombuffer(bytearray(s), dtype=torch.uint8).to(gpu)
    r2 = codec.decode_batch(s, d_stream=d)
    assert (r2.consumed, r2.rt) == (oused, ort)
    # encode on the device == sequential ProtobufCodec::encode calls
    pl = [oracle.lcg_bytes(L, 40 + i) for i, L in enumerate([0, 5, 6, 99, 4096, 1])]
    src = np.concatenate(pl + [np.zeros(1, np.uint8)])
    lens_a = np.array([p.size for p in pl], dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens_a)[:-1]]).astype(np.uint64)
    enc = codec.encode_batch(torch.from_numpy(src).to(gpu), offs, lens_a)
    want = [oracle.pbc_encode(p) for p in pl]
    assert enc.rt.tolist() == [w[0] for w in want]
    assert enc.frames.cpu().numpy().tobytes() == b"".join(w[1] for w in want)
