"""Batched LengthHeaderCodec: frame verify (decode) and frame build (encode) for annety's wire format.

Mirrors annety::LengthHeaderCodec (include/codec/LengthHeaderCodec.h:37-231) with the checksum
enabled: same length types, same max_payload rule, same return codes. Where the reference handles one
frame per call on an I/O thread, this class handles a whole receive stream (decode) or a whole batch
of payloads (encode) per call, with every CRC computed on the GPU:

  decode_batch  = Codec::recv's loop (include/codec/Codec.h:52-76) over a stream: the host walks the
                  length headers (annety_lhc_parse: a sequential chain, a few ns per frame), the device
                  checks every trailer in one batch (annety_lhc_verify_batch); the frames delivered are
                  those before the first bad one, exactly the reference's sequence of decode() results.
  encode_batch  = one encode() per payload appended to one NetBuffer (:146-201): host plan of the
                  output offsets (annety_lhc_encode_plan), then one device pass writing header, payload
                  copy and trailer of every frame (annety_lhc_encode_batch).

There is no CPU fallback: the checksum work runs on the device or the call fails.
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass

import numpy as np

from . import _lib
from .crc32c import BytesLike, _dev_ptr, _host_view, _on_device, _require_device, _stream_handle

DEFAULT_MAX_PAYLOAD = 64 * 1024 * 1024  # LengthHeaderCodec ctor default (:50)


@dataclass
class DecodeResult:
    """What Codec::recv would have produced on this stream.

    payload_off/payload_len: the frames decode() returned 1 for, in order (offsets into the stream).
    consumed: bytes those frames took (the reference's has_read total).
    rt: the decode() result that ended the loop: 0 (incomplete / stream exhausted) or -1 (invalid
        length or checksum: the reference shuts the connection down).
    ok: per-frame checksum verdicts of every complete frame the header walk found (device output).
    """

    payload_off: np.ndarray
    payload_len: np.ndarray
    consumed: int
    rt: int
    ok: np.ndarray


@dataclass
class EncodeResult:
    """frames: uint8 device tensor holding every accepted frame back to back; frame_off[i] = start of
    payload i's frame; rt[i] = the reference's encode() result for payload i (1, 0 empty, -1 too long)."""

    frames: object
    frame_off: np.ndarray
    rt: np.ndarray


def recv_result(length_type: int, off: np.ndarray, ln: np.ndarray, used: int, invalid: bool,
                ok: np.ndarray) -> DecodeResult:
    """Codec::recv's outcome from the header walk and the per-frame checksum verdicts: frames are
    delivered in order until the first bad checksum (decode -1 at :128-132), else until the walk
    stopped (incomplete: 0; invalid length: -1 at :102-106)."""
    bad = np.flatnonzero(ok == 0)
    if bad.size:
        k = int(bad[0])
        return DecodeResult(off[:k], ln[:k], int(off[k]) - length_type, -1, ok)
    return DecodeResult(off, ln, used, -1 if invalid else 0, ok)


_scratch = threading.local()
# Largest bound whose arrays a thread keeps between calls: 16M frames (208 MB), above the first bound of a
# 1 GiB stream (_frame_caps: ~8.4M). A worst-case retry (a frame per T + 4 bytes: 134M frames, 1.7 GB for
# 1 GiB) gets arrays of its own that go with the call.
_CACHE_MAX_FRAMES = 16 << 20


def _out_arrays(cap: int):
    """This thread's output arrays for a frame walk of at most `cap` frames (grow-only up to
    _CACHE_MAX_FRAMES, reused by every call; the results are copied out of them). Arrays of the bound's size
    allocated per call cost more than the verify itself on a 1 GiB stream: 110 MB of them, 28 GiB/s against
    51 with arrays of the exact frame count."""
    c = max(int(cap), 1)
    if c > _CACHE_MAX_FRAMES:
        return np.empty(c, np.uint64), np.empty(c, np.uint32), np.empty(c, np.uint8)
    have = getattr(_scratch, "arrays", None)
    if have is None or have[0].size < c:
        have = (np.empty(c, np.uint64), np.empty(c, np.uint32), np.empty(c, np.uint8))
        _scratch.arrays = have
    return have[0][:c], have[1][:c], have[2][:c]


def _frame_caps(worst: int, max_frames):
    """Output bounds to try in turn. The result arrays are sized by the bound, and worst-case arrays (a
    frame per T + 4 bytes) for a 1 GiB buffer cost more than the verify itself (1.7 GB of fresh arrays per
    call: 20 against 49 GiB/s): first a bound for frames of 128 bytes or more on
    average, the worst case only when a call filled that one (and is then repeated)."""
    if max_frames is not None:
        return [int(max_frames)]
    first = min(worst, worst // 16 + 4096)
    return [first] if first >= worst else [first, worst]


def _iov_results(call, name, length_type, streams, max_frames):
    """Shared body of decode_host_iov: K receive buffers through one *_verify_host_iov call; returns one
    DecodeResult per buffer (what Codec::recv would have produced on that connection)."""
    views = [_host_view(b) for b in streams]
    k = len(views)
    addrs = (ctypes.c_void_p * max(k, 1))(*[v[0] or None for v in views])
    sizes = np.array([v[1] for v in views] or [0], dtype=np.uint64)
    caps = _frame_caps(sum(v[1] // (length_type + 4) + 1 for v in views), max_frames)
    for cap in caps:
        off, ln, ok = _out_arrays(cap)
        nfr = np.zeros(max(k, 1), dtype=np.uint64)
        used = np.zeros(max(k, 1), dtype=np.uint64)
        rts = np.zeros(max(k, 1), dtype=np.int32)
        st = call(addrs, sizes.ctypes.data, k, off.ctypes.data, ln.ctypes.data, ok.ctypes.data, cap, nfr.ctypes.data,
                  used.ctypes.data, rts.ctypes.data)
        _lib.check(st, name)
        if int(nfr[:k].sum()) < cap:
            break
    total = int(nfr[:k].sum())
    off, ln, ok = off[:total].copy(), ln[:total].copy(), ok[:total].copy()
    out, pos = [], 0
    for c in range(k):
        n = int(nfr[c])
        if rts[c] < 0:
            _lib.check(int(rts[c]), name)
        out.append(recv_result(length_type, off[pos:pos + n], ln[pos:pos + n], int(used[c]), rts[c] == 1,
                               ok[pos:pos + n]))
        pos += n
    return out


class LengthHeaderCodec:
    kLengthType8 = 1
    kLengthType16 = 2
    kLengthType32 = 4
    kLengthType64 = 8

    def __init__(self, length_type: int = kLengthType32, enable_checksum: bool = True,
                 max_payload: int = DEFAULT_MAX_PAYLOAD):
        # constructor checks of :48-61
        if length_type not in (1, 2, 4, 8):
            raise ValueError(f"length_type must be 1, 2, 4 or 8, got {length_type}")
        if not enable_checksum:
            raise ValueError("the batch codec is the checksum path; enable_checksum=False has no device work")
        self.length_type = int(length_type)
        self.max_payload = int(max_payload)

    # ---------------- decode ----------------
    def parse(self, stream: BytesLike, max_frames: int | None = None):
        """Host header walk (annety_lhc_parse): (payload_off u64[k], payload_len u32[k], consumed,
        stopped_on_invalid_length)."""
        addr, size, keep = _host_view(stream)
        for cap in _frame_caps(size // (self.length_type + 4) + 1, max_frames):
            off, ln, _ = _out_arrays(cap)
            k, used = ctypes.c_size_t(), ctypes.c_size_t()
            st = _lib.get().annety_lhc_parse(addr or None, size, self.length_type, self.max_payload, off.ctypes.data,
                                             ln.ctypes.data, cap, ctypes.byref(k), ctypes.byref(used))
            if st < 0:
                _lib.check(st, "annety_lhc_parse")
            if k.value < cap:
                break
        return off[: k.value].copy(), ln[: k.value].copy(), int(used.value), st == 1

    def verify(self, d_stream, d_off, d_len, out_ok=None, out_digest=None, stream=None, arena=True):
        """Device checksum check of located frames: ok uint8[n] (1 = trailer matches).
        arena=True (default): the frames fill d_stream, one pass over the stream (annety_lhc_verify_stream);
        False: the general variable-length path (annety_lhc_verify_batch)."""
        import torch

        _require_device(d_stream, "d_stream")
        n = int(d_off.numel())
        if out_ok is None:
            out_ok = torch.empty(n, dtype=torch.uint8, device=d_stream.device)
        dig = _dev_ptr(out_digest) if out_digest is not None else None
        with _on_device(d_stream, d_off, d_len, out_ok):
            sh = _stream_handle(stream, out_ok)
            if arena:
                nbytes = int(d_stream.numel() * d_stream.element_size())
                st = _lib.get().annety_lhc_verify_stream(_dev_ptr(d_stream), nbytes, _dev_ptr(d_off), _dev_ptr(d_len),
                                                         n, _dev_ptr(out_ok), dig, sh)
            else:
                st = _lib.get().annety_lhc_verify_batch(_dev_ptr(d_stream), _dev_ptr(d_off), _dev_ptr(d_len), n,
                                                        _dev_ptr(out_ok), dig, sh)
        _lib.check(st, "annety_lhc_verify_" + ("stream" if arena else "batch"))
        return out_ok

    def decode_batch(self, stream: BytesLike, d_stream=None, device=None) -> DecodeResult:
        """Codec::recv over a whole stream. `stream` is the host copy the headers are read from;
        `d_stream` the same bytes in device memory (uploaded here when not given)."""
        import torch

        off, ln, used, invalid = self.parse(stream)
        if d_stream is None:
            addr, size, keep = _host_view(stream)
            h = np.asarray(keep, dtype=np.uint8).reshape(-1)
            h = h if h.flags.writeable else h.copy()  # torch.from_numpy wants a writable array
            d_stream = torch.from_numpy(h).to(device if device is not None else "cuda")
        n = off.size
        if n:
            d_off = torch.from_numpy(off.view(np.int64)).to(d_stream.device)
            d_len = torch.from_numpy(ln.view(np.int32)).to(d_stream.device)
            ok = self.verify(d_stream, d_off, d_len).cpu().numpy()
        else:
            ok = np.zeros(0, dtype=np.uint8)
        return recv_result(self.length_type, off, ln, used, invalid, ok)

    def decode_host(self, stream: BytesLike, max_frames: int | None = None) -> DecodeResult:
        """Codec::recv over a host receive buffer in one call (annety_lhc_verify_host): the header walk
        overlaps the stream's copy to the current device, the CRCs are checked there."""
        addr, size, keep = _host_view(stream)
        for cap in _frame_caps(size // (self.length_type + 4) + 1, max_frames):
            off, ln, ok = _out_arrays(cap)
            k, used = ctypes.c_size_t(), ctypes.c_size_t()
            st = _lib.get().annety_lhc_verify_host(addr or None, size, self.length_type, self.max_payload,
                                                   off.ctypes.data, ln.ctypes.data, ok.ctypes.data, cap, ctypes.byref(k),
                                                   ctypes.byref(used))
            if st < 0:
                _lib.check(st, "annety_lhc_verify_host")
            if k.value < cap:
                break
        n = k.value
        return recv_result(self.length_type, off[:n].copy(), ln[:n].copy(), int(used.value), st == 1, ok[:n].copy())

    def decode_host_iov(self, streams, max_frames: int | None = None) -> list:
        """Codec::recv over K connections' receive buffers in one call (annety_lhc_verify_host_iov): one
        device stream, one arena verify; returns one DecodeResult per buffer, offsets relative to it."""
        lib = _lib.get()

        def call(addrs, sizes, k, off, ln, ok, cap, nfr, used, rts):
            return lib.annety_lhc_verify_host_iov(addrs, sizes, k, self.length_type, self.max_payload, off, ln, ok,
                                                  cap, nfr, used, rts)

        return _iov_results(call, "annety_lhc_verify_host_iov", self.length_type, streams, max_frames)

    # ---------------- encode ----------------
    def _encode_call(self, d_src, d_soff, d_len, n, frames, d_foff, sh):
        return _lib.get().annety_lhc_encode_batch(_dev_ptr(d_src), _dev_ptr(d_soff), _dev_ptr(d_len), n,
                                                  self.length_type, self.max_payload, _dev_ptr(frames),
                                                  _dev_ptr(d_foff), sh), "annety_lhc_encode_batch"

    def plan(self, lengths: np.ndarray):
        """annety_lhc_encode_plan: (frame_off u64[n], rt i8[n], total bytes)."""
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        off = np.zeros(ln.size, dtype=np.uint64)
        rt = np.zeros(ln.size, dtype=np.int8)
        total = ctypes.c_uint64()
        st = _lib.get().annety_lhc_encode_plan(ln.ctypes.data, ln.size, self.length_type, self.max_payload,
                                               off.ctypes.data, rt.ctypes.data, ctypes.byref(total))
        _lib.check(st, "annety_lhc_encode_plan")
        return off, rt, int(total.value)

    def encode_batch(self, d_src, src_off: np.ndarray, lengths: np.ndarray, stream=None) -> EncodeResult:
        """Frames for payload i = d_src[src_off[i] : src_off[i] + lengths[i]] (host index arrays)."""
        import torch

        _require_device(d_src, "d_src")
        src_off = np.ascontiguousarray(src_off, dtype=np.uint64)
        lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
        if src_off.size != lengths.size:
            raise ValueError("src_off and lengths differ in size")
        if lengths.size and int((src_off + lengths.astype(np.uint64)).max()) > d_src.numel():
            raise ValueError("a payload extends past the end of d_src")
        frame_off, rt, total = self.plan(lengths)
        dev = d_src.device
        frames = torch.empty(total, dtype=torch.uint8, device=dev)
        n = lengths.size
        if n and total:
            d_soff = torch.from_numpy(src_off.view(np.int64)).to(dev)
            d_len = torch.from_numpy(lengths.view(np.int32)).to(dev)
            d_foff = torch.from_numpy(frame_off.view(np.int64)).to(dev)
            with _on_device(d_src, frames):
                st, name = self._encode_call(d_src, d_soff, d_len, n, frames, d_foff, _stream_handle(stream, frames))
            _lib.check(st, name)
        return EncodeResult(frames, frame_off, rt)


class ProtobufCodecFrames(LengthHeaderCodec):
    """Batched framing of annety's ProtobufCodec (include/protobuf/ProtobufCodec.h, checksum on): the
    LengthHeaderCodec wire layout with a 4-byte length and the codec's fixed limits (decode: length field
    in [10, 64 MiB], :149-156, :273-283; encode: payload of 6 .. 64 MiB bytes, :223-230). The CRC covers
    the whole payload (nameLen + typeName + message bytes, :235-247); the message itself stays opaque
    (parsing it is the caller's, with libprotobuf)."""

    MIN_PAYLOAD = 10
    MAX_PAYLOAD = 64 * 1024 * 1024

    def __init__(self):
        super().__init__(self.kLengthType32, True, self.MAX_PAYLOAD)

    def parse(self, stream: BytesLike, max_frames: int | None = None):
        addr, size, keep = _host_view(stream)
        for cap in _frame_caps(size // 8 + 1, max_frames):
            off, ln, _ = _out_arrays(cap)
            k, used = ctypes.c_size_t(), ctypes.c_size_t()
            st = _lib.get().annety_pbc_parse(addr or None, size, off.ctypes.data, ln.ctypes.data, cap, ctypes.byref(k),
                                             ctypes.byref(used))
            if st < 0:
                _lib.check(st, "annety_pbc_parse")
            if k.value < cap:
                break
        return off[: k.value].copy(), ln[: k.value].copy(), int(used.value), st == 1

    def decode_host(self, stream: BytesLike, max_frames: int | None = None) -> DecodeResult:
        addr, size, keep = _host_view(stream)
        for cap in _frame_caps(size // 8 + 1, max_frames):
            off, ln, ok = _out_arrays(cap)
            k, used = ctypes.c_size_t(), ctypes.c_size_t()
            st = _lib.get().annety_pbc_verify_host(addr or None, size, off.ctypes.data, ln.ctypes.data, ok.ctypes.data,
                                                   cap, ctypes.byref(k), ctypes.byref(used))
            if st < 0:
                _lib.check(st, "annety_pbc_verify_host")
            if k.value < cap:
                break
        n = k.value
        return recv_result(self.length_type, off[:n].copy(), ln[:n].copy(), int(used.value), st == 1, ok[:n].copy())

    def decode_host_iov(self, streams, max_frames: int | None = None) -> list:
        lib = _lib.get()

        def call(addrs, sizes, k, off, ln, ok, cap, nfr, used, rts):
            return lib.annety_pbc_verify_host_iov(addrs, sizes, k, off, ln, ok, cap, nfr, used, rts)

        return _iov_results(call, "annety_pbc_verify_host_iov", self.length_type, streams, max_frames)

    def plan(self, lengths: np.ndarray):
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        off = np.zeros(ln.size, dtype=np.uint64)
        rt = np.zeros(ln.size, dtype=np.int8)
        total = ctypes.c_uint64()
        st = _lib.get().annety_pbc_encode_plan(ln.ctypes.data, ln.size, off.ctypes.data, rt.ctypes.data,
                                               ctypes.byref(total))
        _lib.check(st, "annety_pbc_encode_plan")
        return off, rt, int(total.value)

    def _encode_call(self, d_src, d_soff, d_len, n, frames, d_foff, sh):
        return _lib.get().annety_pbc_encode_batch(_dev_ptr(d_src), _dev_ptr(d_soff), _dev_ptr(d_len), n,
                                                  _dev_ptr(frames), _dev_ptr(d_foff), sh), "annety_pbc_encode_batch"
