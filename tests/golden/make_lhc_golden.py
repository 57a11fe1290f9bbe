"""Generate tests/golden/lhc.json from the reference's OWN LengthHeaderCodec.

Run here (where /root/reference exists):   python tests/golden/make_lhc_golden.py
It builds oracle/_ref/libref_codec.so (oracle/Makefile `ref`: the unmodified
include/codec/LengthHeaderCodec.h over the reference's src/*.cc) and records, for seeded payloads and
hand-made streams, what LengthHeaderCodec::encode appends and what successive decode calls return
(Codec::recv's loop, include/codec/Codec.h:52-76). Every file written is data.

Payload bytes come from oracle.lcg_bytes(len, seed) so the GPU box can regenerate them.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

import oracle  # noqa: E402

oracle.build(ref=True)
ref = oracle.ref_codec_lib()
MAXP = oracle.DEFAULT_MAX_PAYLOAD


def ref_encode(T: int, maxp: int, payload: bytes) -> tuple[int, bytes]:
    cap = len(payload) + 16
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t()
    rt = ref.ref_lhc_encode(T, maxp, payload, len(payload), out, cap, ctypes.byref(n))
    assert rt != -100
    return rt, out.raw[: n.value]


def ref_recv(T: int, maxp: int, stream: bytes) -> tuple[list, int, int]:
    """decode until rt != 1; returns ([(payload_off, payload_len)], consumed, last rt)."""
    frames, pos = [], 0
    while True:
        rest = stream[pos:]
        cap = len(rest) + 1
        buf = ctypes.create_string_buffer(cap)
        pl, used = ctypes.c_size_t(), ctypes.c_size_t()
        rt = ref.ref_lhc_decode(T, maxp, rest, len(rest), buf, cap, ctypes.byref(pl), ctypes.byref(used))
        assert rt != -100
        if rt != 1:
            assert used.value == 0
            return frames, pos, rt
        # the payload the reference hands out is the stream slice after the header
        assert buf.raw[: pl.value] == stream[pos + T : pos + T + pl.value]
        frames.append((pos + T, pl.value))
        pos += used.value


def payload(n: int, seed: int) -> bytes:
    return oracle.lcg_bytes(n, seed).tobytes()


LENS = [0, 1, 2, 3, 4, 5, 15, 16, 59, 60, 61, 64, 100, 119, 120, 123, 124, 127, 128, 200, 251, 252, 255, 256,
        1000, 1024, 4093, 32763, 32764, 32767, 65536, 70000]


def encode_cases() -> list:
    cases = []
    for T in (1, 2, 4, 8):
        for n in LENS:
            seed = 1000 * T + n
            rt, out = ref_encode(T, MAXP, payload(n, seed))
            c = {"T": T, "max_payload": MAXP, "len": n, "seed": seed, "rt": rt, "out_len": len(out)}
            if out:
                assert out[T : T + n] == payload(n, seed)  # the payload is copied verbatim
                c["header"] = out[:T].hex()
                c["trailer"] = out[T + n :].hex()
            cases.append(c)
    for maxp, n in ((100, 100), (100, 101), (1, 1), (1, 2), (0, 70000), (-1, 5000)):
        seed = 77 + n
        rt, out = ref_encode(4, maxp, payload(n, seed))
        c = {"T": 4, "max_payload": maxp, "len": n, "seed": seed, "rt": rt, "out_len": len(out)}
        if out:
            c["header"] = out[:4].hex()
            c["trailer"] = out[4 + n :].hex()
        cases.append(c)
    return cases


def stream_of(T: int, lens: list, seed: int) -> bytes:
    s = b""
    for i, n in enumerate(lens):
        rt, out = ref_encode(T, MAXP, payload(n, seed + i))
        s += out
    return s


def decode_cases() -> list:
    cases = []

    def add(name: str, T: int, maxp: int, stream: bytes) -> None:
        frames, used, rt = ref_recv(T, maxp, stream)
        cases.append({"name": name, "T": T, "max_payload": maxp, "stream": stream.hex(), "frames": frames,
                      "consumed": used, "rt": rt})

    for T in (1, 2, 4, 8):
        lens = [1, 5, 60, 61, 100] if T == 1 else [1, 5, 60, 61, 100, 300, 1000]
        s = stream_of(T, lens, 500 + T)
        add(f"stream_T{T}", T, MAXP, s)
        add(f"stream_T{T}_cut", T, MAXP, s[:-3])
        for cut in range(0, T + 8):
            add(f"prefix_T{T}_{cut}", T, MAXP, s[:cut])
        bad = bytearray(s)
        bad[T + 2] ^= 0x10  # payload bit flip in frame 1
        add(f"flip_payload_T{T}", T, MAXP, bytes(bad))
        f1 = T + 1 + 4
        bad = bytearray(s)
        bad[f1 + T] ^= 0x01  # payload flip in frame 2: frame 1 is delivered first
        add(f"flip_frame2_T{T}", T, MAXP, bytes(bad))
        bad = bytearray(s)
        bad[T + 1 + 3] ^= 0x80  # trailer flip in frame 1
        add(f"flip_trailer_T{T}", T, MAXP, bytes(bad))
        for hdr in (0, 1, 3, 4, -1, -(2 ** (8 * T - 1))):
            h = (hdr & ((1 << (8 * T)) - 1)).to_bytes(T, "big")
            add(f"hdr_T{T}_{hdr}", T, MAXP, h + b"\x00" * 8)
    # length field > max_payload, == max_payload (the field counts the 4 checksum bytes)
    s = stream_of(4, [96, 97], 900)
    add("max_payload_100", 4, 100, s)
    add("max_payload_0_unlimited", 4, 0, s)
    # an over-long T=1 payload: encode truncates the header (append_int8), decode rejects it
    _, out = ref_encode(1, MAXP, payload(200, 3))
    add("t1_truncated_header", 1, MAXP, out)
    # an empty-payload frame written by hand: length field 4, no payload, crc32("") = 0
    add("empty_payload_frame", 4, MAXP, (4).to_bytes(4, "big") + b"\x00" * 4 + stream_of(4, [7], 901))
    return cases


def main() -> None:
    obj = {"source": "reference LengthHeaderCodec (include/codec/LengthHeaderCodec.h) via oracle/ref_codec.cc",
           "payload_gen": "oracle.lcg_bytes(len, seed)", "encode": encode_cases(), "decode": decode_cases()}
    with open(os.path.join(HERE, "lhc.json"), "w") as f:
        json.dump(obj, f, indent=0, sort_keys=True)
        f.write("\n")
    print("encode", len(obj["encode"]), "decode", len(obj["decode"]))


if __name__ == "__main__":
    main()
