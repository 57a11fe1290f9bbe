"""LengthHeaderCodec batch path.

CPU tests pin the oracle's codec restatement to fixtures recorded from the reference's own
LengthHeaderCodec (tests/golden/lhc.json, tests/golden/make_lhc_golden.py) and check the host logic
of the C-ABI (header walk, encode plan, recv outcome). GPU tests run decode/encode through the C-ABI
and compare with the fixtures and the oracle.
"""
import os

import numpy as np
import pytest

import oracle
from annety_amd.codec import LengthHeaderCodec, recv_result

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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
def test_gpu_decode_host_matches_reference(golden, gpu):
    """annety_lhc_verify_host (walk overlapped with the upload, verify on the device) = Codec::recv."""
    for c in golden("lhc.json")["decode"]:
        codec = LengthHeaderCodec(c["T"], True, c["max_payload"])
        r = codec.decode_host(bytes.fromhex(c["stream"]))
        assert [[int(o), int(n)] for o, n in zip(r.payload_off, r.payload_len)] == c["frames"], c["name"]
        assert (r.consumed, r.rt) == (c["consumed"], c["rt"]), c["name"]


@pytest.mark.gpu
def test_gpu_decode_host_large_stream(gpu):
    """A 200 MiB frame stream (several staging pieces) through decode_host, pageable and pinned,
    with corrupted frames: verdicts equal the oracle's on every frame."""
    import annety_amd

    rng = np.random.default_rng(9)
    lens = np.minimum(65536, 64 * np.minimum(rng.zipf(1.3, 6000), 1 << 20) + rng.integers(0, 64, 6000)).astype(np.int64)
    body = oracle.lcg_bytes(int(lens.sum()), 31)
    pieces, pos = [], 0
    for L in lens.tolist():
        rt, fr = oracle.lhc_encode(body[pos:pos + L], 4)
        pieces.append(fr)
        pos += L
    stream = bytearray(b"".join(pieces))
    reps = 200 * 2 ** 20 // len(stream) + 1
    stream = bytearray(bytes(stream) * reps)
    bad = rng.choice(len(lens) * reps, 25, replace=False)
    starts = np.concatenate([[0], np.cumsum(np.tile(lens + 8, reps))[:-1]])
    for b in bad:
        stream[int(starts[b]) + 4] ^= 0x40  # flip a payload bit -> checksum mismatch
    codec = LengthHeaderCodec(4)
    want_ok = np.ones(len(starts), dtype=np.uint8)
    want_ok[bad] = 0
    r = codec.decode_host(bytes(stream))
    assert np.array_equal(r.ok, want_ok)
    assert r.rt == -1 and r.consumed == int(starts[np.sort(bad)[0]])
    pinned = annety_amd.PinnedHostBuffer(len(stream))
    pinned.array[:] = np.frombuffer(bytes(stream), dtype=np.uint8)
    r2 = codec.decode_host(pinned.array)
    assert np.array_equal(r2.ok, want_ok)
    pinned.close()


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


@pytest.mark.gpu
def test_gpu_encode_fused_every_alignment(gpu):
    """The one-pass encoder (crc32_frames.hip lhc_encode_fused_kernel) at every edge its copy has: payload lengths
    0..300 (empty frames write nothing; 1-3 byte payloads are all edge bytes), source starts at every offset of
    a 128-byte line, destination alignments from the packed frames of every header width, payloads that end in
    the first bytes of a line (the copy's dword straddling two lines), and lengths just around whole lines and
    whole 8-line rounds; every frame against the oracle's encoder."""
    import torch

    rng = np.random.default_rng(20261018)
    lens = np.concatenate([np.arange(0, 301), rng.integers(0, 3000, 400),
                           np.array([128 * k + d for k in (1, 7, 8, 9, 15, 16, 17, 64) for d in (-5, -1, 0, 1, 3)])])
    lens = rng.permutation(lens).astype(np.uint32)
    starts = rng.integers(0, 128, lens.size)
    offs = (np.arange(lens.size, dtype=np.uint64) * 4096 + starts.astype(np.uint64)).astype(np.uint64)
    arena = oracle.lcg_bytes(int(offs[-1]) + 4096 + 8, 123)
    d_src = torch.from_numpy(arena.copy()).to(gpu)
    for T in (1, 2, 4, 8):
        codec = LengthHeaderCodec(T, True, 4000 if T > 1 else 200)
        r = codec.encode_batch(d_src, offs, lens)
        frames = r.frames.cpu().numpy().tobytes()
        want = b"".join(oracle.lhc_encode(arena[int(o): int(o) + int(L)], T, codec.max_payload)[1]
                        for o, L in zip(offs, lens))
        assert frames == want, T


@pytest.mark.gpu
def test_gpu_encode_four_lane_groups(gpu):
    """Batches of mostly short frames run the encoder with 4 lanes per frame (crc32_frames.hip lhc_encode_fused_kernel
    picks it when >= 3/4 of 512 sampled frames fit one 4-line round): short frames at every source alignment, frames
    of several 4-line rounds among them (lengths around whole lines and rounds), empty ones, and frames of more than
    256 KiB that the 4-lane groups hand to the long path; every header width, every frame against the oracle."""
    import torch

    rng = np.random.default_rng(4)
    short = rng.integers(0, 497, 3000)
    multi = np.array([128 * k + d for k in range(3, 28) for d in (-3, 0, 5)])  # 2 to 7 rounds of 4 lines
    lens = rng.permutation(np.concatenate([short, multi, [300000, 262145, 400000]])).astype(np.uint32)
    starts = rng.integers(0, 128, lens.size).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum((lens.astype(np.uint64) + 127) // 128 * 128 + 128)[:-1]]) + starts
    arena = oracle.lcg_bytes(int(offs[-1] + lens[-1]) + 256, 321)
    d_src = torch.from_numpy(arena.copy()).to(gpu)
    for T, maxp in ((1, 100), (2, 30000), (4, 1 << 26), (8, 1 << 26)):
        codec = LengthHeaderCodec(T, True, maxp)
        r = codec.encode_batch(d_src, offs.astype(np.uint64), lens)
        frames = r.frames.cpu().numpy().tobytes()
        want = b"".join(oracle.lhc_encode(arena[int(o): int(o) + int(L)], T, maxp)[1] for o, L in zip(offs, lens))
        assert frames == want, T


# ---------------- the reference codec itself, linked against the drop-in ----------------
@pytest.mark.skipif(not os.path.isdir("/root/reference/src"), reason="reference tree not present")
def test_reference_codec_runs_on_dropin(golden, tmp_path):
    """annety's own LengthHeaderCodec (include/codec/LengthHeaderCodec.h) compiled with the drop-in
    Crc32c.h first on the include path and linked with libannety_crc.so in place of src/Crc32c.cc
     reproduces every recorded encode output and decode sequence."""
    import ctypes
    import glob
    import subprocess

    from annety_amd import _lib

    oracle.build(ref=True)
    objs = [o for o in glob.glob(os.path.join(ROOT, "oracle", "_ref", "obj", "*.o"))
            if os.path.basename(o) != "Crc32c.o"]
    assert len(objs) > 40
    so = tmp_path / "libdropin_codec.so"
    libdir = os.path.dirname(_lib.lib_path())
    subprocess.run(["g++", "-std=c++11", "-O2", "-fPIC", "-shared", "-w", "-include", "functional",
                    f"-I{ROOT}/include/annety", f"-I{ROOT}/include", "-I/root/reference/include",
                    "-I/root/reference/src", os.path.join(ROOT, "oracle", "ref_codec.cc"), *objs, "-o", str(so),
                    f"-L{libdir}", "-lannety_crc", f"-Wl,-rpath,{libdir}", "-lpthread"], check=True)
    # the tables must come from the engine library, not from a stray copy of src/Crc32c.cc
    nm = subprocess.run(["nm", "-D", "--defined-only", str(so)], capture_output=True, text=True).stdout
    assert "_ZN6annety8internal14crc32_table256E" not in nm
    lib = ctypes.CDLL(str(so))
    sp = ctypes.POINTER(ctypes.c_size_t)
    lib.ref_lhc_encode.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                   ctypes.c_size_t, sp]
    lib.ref_lhc_decode.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                   ctypes.c_size_t, sp, sp]
    g = golden("lhc.json")
    for c in g["encode"]:
        p = _payload(c["len"], c["seed"])
        out = ctypes.create_string_buffer(len(p) + 16)
        n = ctypes.c_size_t()
        rt = lib.ref_lhc_encode(c["T"], c["max_payload"], p, len(p), out, len(p) + 16, ctypes.byref(n))
        assert rt == c["rt"] and out.raw[: n.value] == _expected_encode(c), c
    for c in g["decode"]:
        s = bytes.fromhex(c["stream"])
        frames, pos = [], 0
        while True:
            rest = s[pos:]
            buf = ctypes.create_string_buffer(len(rest) + 1)
            pl, used = ctypes.c_size_t(), ctypes.c_size_t()
            rt = lib.ref_lhc_decode(c["T"], c["max_payload"], rest, len(rest), buf, len(rest) + 1, ctypes.byref(pl),
                                    ctypes.byref(used))
            if rt != 1:
                break
            frames.append([pos + c["T"], pl.value])
            pos += used.value
        assert frames == c["frames"] and (pos, rt) == (c["consumed"], c["rt"]), c["name"]


CPP_BATCH = r"""
// Host side of include/annety/LengthHeaderCodecBatch.h (no device calls): locate + recv_outcome with
// verdicts from the drop-in's host Crc32c, and plan. Reads a stream file, prints what recv would do.
#define ANNETY_CRC_NO_STRINGPIECE
#include "annety/Crc32c.h"
#include "annety/LengthHeaderCodecBatch.h"
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  if (argc != 4) return 1;
  const int T = std::atoi(argv[2]);
  const long long maxp = std::atoll(argv[3]);
  std::FILE* f = std::fopen(argv[1], "rb");
  std::vector<char> buf;
  int ch;
  while ((ch = std::fgetc(f)) != EOF) buf.push_back((char)ch);
  std::fclose(f);
  annety::LengthHeaderCodecBatch codec((annety::LengthHeaderCodecBatch::LENGTH_TYPE)T, maxp);
  annety::LengthHeaderCodecBatch::Frames fr;
  if (codec.locate(buf.data(), buf.size(), &fr) != 0) return 2;
  std::vector<uint8_t> ok(fr.payload_off.size());
  for (size_t i = 0; i < ok.size(); i++) {
    const unsigned char* t = reinterpret_cast<const unsigned char*>(buf.data() + fr.payload_off[i] + fr.payload_len[i]);
    const uint32_t want = (uint32_t)t[0] << 24 | (uint32_t)t[1] << 16 | (uint32_t)t[2] << 8 | t[3];
    ok[i] = annety::Crc32c::crc32_long(buf.data() + fr.payload_off[i], fr.payload_len[i]) == want;
  }
  size_t delivered = 0, consumed = 0;
  const int rt = codec.recv_outcome(fr, ok.data(), &delivered, &consumed);
  std::printf("%d %zu %zu", rt, delivered, consumed);
  for (size_t i = 0; i < delivered; i++) std::printf(" %llu:%u", (unsigned long long)fr.payload_off[i], fr.payload_len[i]);
  std::printf("\n");
  // plan over the payload lengths found (+ an empty one and one above max_payload when it is set)
  std::vector<uint32_t> lens(fr.payload_len.begin(), fr.payload_len.end());
  lens.push_back(0);
  if (maxp > 0) lens.push_back((uint32_t)maxp + 1);
  std::vector<uint64_t> off(lens.size());
  std::vector<int8_t> prt(lens.size());
  uint64_t total = 0;
  if (codec.plan(lens.data(), lens.size(), off.data(), prt.data(), &total) != 0) return 3;
  std::printf("%llu", (unsigned long long)total);
  for (size_t i = 0; i < lens.size(); i++) std::printf(" %d:%llu", prt[i], (unsigned long long)off[i]);
  std::printf("\n");
  return 0;
}
"""


def test_cpp_batch_codec_host_side(golden, tmp_path):
    """The C++ batch codec's host logic equals Codec::recv on the reference-recorded streams and on
    long generated ones; its plan() equals encode()'s decisions."""
    import subprocess

    from annety_amd import _lib

    src = tmp_path / "b.cc"
    src.write_text(CPP_BATCH)
    exe = tmp_path / "b"
    libdir = os.path.dirname(_lib.lib_path())
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Wextra", "-Werror", f"-I{ROOT}/include", str(src), "-o",
                    str(exe), f"-L{libdir}", "-lannety_crc", f"-Wl,-rpath,{libdir}"], check=True)
    cases = [(c["T"], c["max_payload"], bytes.fromhex(c["stream"])) for c in golden("lhc.json")["decode"]]
    rng = np.random.default_rng(9)
    for T in (1, 2, 4, 8):
        lens = rng.integers(0, 120 if T == 1 else 3000, 300)
        s = b"".join(oracle.lhc_encode(_payload(int(n), i), T)[1] for i, n in enumerate(lens))
        bad = bytearray(s)
        bad[len(s) // 2] ^= 1
        cases += [(T, 1 << 26, s), (T, 1 << 26, s[:-7]), (T, 1 << 26, bytes(bad)), (T, 500, s)]
    for T, maxp, s in cases:
        f = tmp_path / "s.bin"
        f.write_bytes(s)
        out = subprocess.run([str(exe), str(f), str(T), str(maxp)], capture_output=True, text=True, check=True)
        line1, line2 = out.stdout.strip().split("\n")
        head = line1.split()
        frames, used, rt = oracle.lhc_recv(s, T, maxp)
        assert int(head[0]) == rt and int(head[1]) == len(frames) and int(head[2]) == used
        assert [tuple(map(int, x.split(":"))) for x in head[3:]] == [tuple(x) for x in frames]
        plan = line2.split()
        lens = [n for _, n in frames] if rt == 0 else None
        if lens is not None:
            pos, want = 0, []
            for n in lens + [0] + ([maxp + 1] if maxp > 0 else []):
                r = 0 if n == 0 else (-1 if maxp > 0 and n > maxp else 1)
                want.append(f"{r}:{pos}")
                pos += T + n + 4 if r == 1 else 0
            assert plan[1:] == want and int(plan[0]) == pos


# ---------------- property tests of the host walk (hypothesis) ----------------
from hypothesis import given, settings, strategies as st  # noqa: E402


@st.composite
def _streams(draw):
    T = draw(st.sampled_from([1, 2, 4, 8]))
    maxp = draw(st.sampled_from([0, -1, 40, 1 << 26]))
    parts = []
    for i in range(draw(st.integers(0, 12))):
        kind = draw(st.sampled_from(["frame", "frame", "frame", "flip", "junk"]))
        if kind == "junk":
            parts.append(draw(st.binary(min_size=1, max_size=12)))
            continue
        n = draw(st.integers(1, 100 if T == 1 else 300))
        _, f = oracle.lhc_encode(_payload(n, 31 * i + n), T, 0)
        if kind == "flip" and len(f) > T:
            b = bytearray(f)
            b[draw(st.integers(T, len(f) - 1))] ^= 1 << draw(st.integers(0, 7))
            f = bytes(b)
        parts.append(f)
    s = b"".join(parts)
    cut = draw(st.integers(0, len(s)))
    return T, maxp, s[:cut]


@settings(max_examples=300, deadline=None)
@given(_streams())
def test_property_walk_and_recv_equal_reference_semantics(case):
    """On arbitrary streams (valid frames, bit flips anywhere including headers, junk, truncation), the
    host walk + per-frame verdicts give exactly the oracle's Codec::recv sequence."""
    T, maxp, s = case
    codec = LengthHeaderCodec(T, True, maxp)
    off, ln, used, invalid = codec.parse(s)
    r = recv_result(T, off, ln, used, invalid, _cpu_verdicts(s, off, ln))
    frames, consumed, rt = oracle.lhc_recv(s, T, maxp)
    assert [(int(o), int(n)) for o, n in zip(r.payload_off, r.payload_len)] == frames
    assert (r.consumed, r.rt) == (consumed, rt)


@settings(max_examples=200, deadline=None)
@given(st.lists(st.integers(0, 5000), max_size=40), st.sampled_from([1, 2, 4, 8]),
       st.sampled_from([0, -1, 100, 4096]))
def test_property_plan_equals_sequential_encode(lens, T, maxp):
    """encode_plan = what consecutive LengthHeaderCodec::encode calls append to one buffer."""
    off, rt, total = LengthHeaderCodec(T, True, maxp).plan(np.array(lens, dtype=np.uint32))
    pos = 0
    for i, n in enumerate(lens):
        r, out = oracle.lhc_encode(_payload(n, i), T, maxp)
        assert int(rt[i]) == r and int(off[i]) == pos
        pos += len(out)
    assert total == pos


@pytest.fixture(params=[True, False], ids=["pack", "pageable"])
def frames_pack(request, gpu):
    """Both upload modes of the frame paths for buffers not pinned here: packed into the library's pinned
    ring (the default) and handed to the runtime's pageable copy (annety_crc_set_frames_pack)."""
    import annety_amd

    annety_amd.set_frames_pack(request.param)
    yield request.param
    annety_amd.set_frames_pack(True)


@pytest.mark.gpu
def test_gpu_decode_host_iov_replays_every_recorded_stream(golden, frames_pack):
    """annety_lhc_verify_host_iov: the reference codec's 95 recorded decode streams as 95 connections'
    receive buffers, one call per codec configuration (T, max_payload) - all 95 in as many calls as there
    are configurations, 93 of them in the four largest calls - each connection's frames, consumed bytes
    and rt equal to the reference's Codec::recv sequence. Then the same with the buffers pinned
    (page-aligned registrations of their own pages, PinnedHostBuffer)."""
    import annety_amd

    groups = {}
    for c in golden("lhc.json")["decode"]:
        groups.setdefault((c["T"], c["max_payload"]), []).append(c)
    assert sum(len(v) for v in groups.values()) == 95
    for (T, mp), cases in groups.items():
        codec = LengthHeaderCodec(T, True, mp)
        bufs = [bytes.fromhex(c["stream"]) for c in cases]
        res = codec.decode_host_iov(bufs)
        assert len(res) == len(cases)
        for c, r in zip(cases, res):
            assert [[int(o), int(n)] for o, n in zip(r.payload_off, r.payload_len)] == c["frames"], c["name"]
            assert (r.consumed, r.rt) == (c["consumed"], c["rt"]), c["name"]
        pinned = []
        for b in bufs:
            p = annety_amd.PinnedHostBuffer(max(1, len(b)))
            p.array[: len(b)] = np.frombuffer(b, dtype=np.uint8)
            pinned.append(p)
        res2 = codec.decode_host_iov([p.array[: len(b)] for p, b in zip(pinned, bufs)])
        for c, r in zip(cases, res2):
            assert [[int(o), int(n)] for o, n in zip(r.payload_off, r.payload_len)] == c["frames"], c["name"]
            assert (r.consumed, r.rt) == (c["consumed"], c["rt"]), c["name"]
        for p in pinned:
            p.close()


@pytest.mark.gpu
def test_gpu_decode_host_iov_large(frames_pack):
    """Many connections whose buffers cross the 64 MiB staging chunks (frames and headers straddle chunk
    boundaries, the walk follows the pack), with corrupted frames and ragged tails: every connection's
    verdicts equal the single-stream path's and the oracle's."""
    rng = np.random.default_rng(21)
    codec = LengthHeaderCodec(4)
    bufs, want = [], []
    for conn in range(40):
        n = int(rng.integers(0, 900))
        lens = (np.minimum(65536, 64 * np.minimum(rng.zipf(1.3, n), 1 << 20) + rng.integers(0, 64, n)).astype(np.int64)
                if n else [])
        body = oracle.lcg_bytes(int(np.sum(lens)) if n else 0, 500 + conn)
        out, pos, starts = [], 0, []
        for L in (lens.tolist() if n else []):
            starts.append(sum(len(x) for x in out))
            out.append(oracle.lhc_encode(body[pos:pos + L], 4)[1])
            pos += L
        s = bytearray(b"".join(out))
        if n and conn % 3 == 0:  # a corrupted frame
            b = int(rng.integers(0, n))
            s[starts[b] + 4] ^= 1
        s += bytes(int(rng.integers(0, 30)))  # ragged tail: an incomplete next frame
        bufs.append(bytes(s))
        want.append(codec.decode_host(bytes(s)))
    assert sum(len(b) for b in bufs) > 150 << 20  # several staging chunks
    got = codec.decode_host_iov(bufs)
    for w, g in zip(want, got):
        assert np.array_equal(w.payload_off, g.payload_off) and np.array_equal(w.payload_len, g.payload_len)
        assert (w.consumed, w.rt) == (g.consumed, g.rt) and np.array_equal(w.ok, g.ok)
    # a frame cap smaller than the total: later connections report no frames
    capped = codec.decode_host_iov(bufs, max_frames=100)
    assert sum(int(r.ok.size) for r in capped) == 100


@pytest.mark.gpu
@pytest.mark.parametrize("T,n", [(1, 3000), (2, 1200), (4, 1200), (8, 300)])
def test_cpp_batch_codec_device(T, n):
    """The C++ batch codec's device methods (include/annety/LengthHeaderCodecBatch.h encode/verify) called from C++:
    tests/native/lhc_batch_device.cpp (built with the library by annety_amd/build.py) encodes a batch on the device
    with empty and over-long payloads among it, checks every frame byte against the drop-in's host Crc32c, verifies
    the stream on the device and checks recv_outcome() against Codec::recv, before and after a flipped byte."""
    import subprocess

    exe = os.path.join(ROOT, "tests", "native", "lhc_batch_device")
    assert os.path.exists(exe), "tests/native/lhc_batch_device is built by annety_amd/build.py"
    r = subprocess.run([exe, str(T), str(n), str(17 + T)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("ok "), r.stdout + r.stderr
    accepted, total = map(int, r.stdout.split()[1:3])
    assert accepted > n // 2 and total > 0
