"""TEST INFRASTRUCTURE ONLY — ctypes access to the CPU oracle.

Two checkers live here:
  * ``liboracle.so``  — the plain-C restatement of annety's checksum path (crc32_oracle.c, every
    function citing the reference file:line it restates). It is built from this directory by
    ``make`` and travels with the repository.
  * ``_ref/libref_crc32.so`` — the reference's own ``src/Crc32c.cc`` + ``include/Crc32c.h`` compiled
    where they lie (``make ref``), present only where /root/reference exists (never on the GPU box
    unless it was built here and shipped with the snapshot).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package. The
product library (annety_amd, libannety_crc.so) never loads it.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(HERE, "liboracle.so")
_REF = os.path.join(HERE, "_ref", "libref_crc32.so")
_REF_CODEC = os.path.join(HERE, "_ref", "libref_codec.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)


def build(ref: bool = False) -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if ref and os.path.isdir("/root/reference"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def _load_oracle() -> ctypes.CDLL:
    if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(os.path.join(HERE, "crc32_oracle.c")):
        build()
    lib = ctypes.CDLL(_LIB)
    lib.oracle_crc32_long.restype = ctypes.c_uint32
    lib.oracle_crc32_long.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.oracle_crc32_short.restype = ctypes.c_uint32
    lib.oracle_crc32_short.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.oracle_crc32_update.restype = None
    lib.oracle_crc32_update.argtypes = [_u32p, ctypes.c_void_p, ctypes.c_size_t]
    lib.oracle_crc32_combine.restype = ctypes.c_uint32
    lib.oracle_crc32_combine.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
    lib.oracle_shift_bytes.restype = ctypes.c_uint32
    lib.oracle_shift_bytes.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
    lib.oracle_crc32_batch_fixed.restype = None
    lib.oracle_crc32_batch_fixed.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                             ctypes.c_void_p]
    lib.oracle_crc32_batch_var.restype = None
    lib.oracle_crc32_batch_var.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.c_void_p]
    lib.oracle_crc32_batch_fixed_mt.restype = ctypes.c_int
    lib.oracle_crc32_batch_fixed_mt.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                                ctypes.c_void_p, ctypes.c_int]
    lib.oracle_crc32_batch_var_mt.restype = ctypes.c_int
    lib.oracle_crc32_batch_var_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                              ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.oracle_lcg_fill.restype = ctypes.c_uint64
    lib.oracle_lcg_fill.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64]
    lib.oracle_tables.restype = None
    lib.oracle_tables.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    _sp = ctypes.POINTER(ctypes.c_size_t)
    lib.oracle_lhc_encode.restype = ctypes.c_int
    lib.oracle_lhc_encode.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_void_p, _sp]
    lib.oracle_lhc_decode.restype = ctypes.c_int
    lib.oracle_lhc_decode.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t, _sp, _sp, _sp]
    lib.oracle_pbc_encode.restype = ctypes.c_int
    lib.oracle_pbc_encode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, _sp]
    lib.oracle_pbc_decode.restype = ctypes.c_int
    lib.oracle_pbc_decode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, _sp, _sp, _sp]
    return lib


_lib = _load_oracle()


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _as_u8(data) -> np.ndarray:
    if isinstance(data, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(data), dtype=np.uint8)
    return np.ascontiguousarray(data, dtype=np.uint8)


def crc32_long(data) -> int:
    a = _as_u8(data)
    return int(_lib.oracle_crc32_long(_ptr(a), a.size))


def crc32_short(data) -> int:
    a = _as_u8(data)
    return int(_lib.oracle_crc32_short(_ptr(a), a.size))


def crc32_update(state: int, data) -> int:
    a = _as_u8(data)
    s = ctypes.c_uint32(state)
    _lib.oracle_crc32_update(ctypes.byref(s), _ptr(a), a.size)
    return int(s.value)


def crc32_combine(crc1: int, crc2: int, len2: int) -> int:
    return int(_lib.oracle_crc32_combine(crc1, crc2, len2))


def shift_bytes(state: int, nbytes: int) -> int:
    return int(_lib.oracle_shift_bytes(state, nbytes))


def tables() -> tuple[np.ndarray, np.ndarray]:
    t256 = np.zeros(256, dtype=np.uint32)
    t16 = np.zeros(16, dtype=np.uint32)
    _lib.oracle_tables(_ptr(t256), _ptr(t16))
    return t256, t16


def batch_fixed(buf: np.ndarray, n: int, length: int, stride: int | None = None) -> np.ndarray:
    stride = length if stride is None else stride
    a = _as_u8(buf)
    if n and (n - 1) * stride + length > a.size:
        raise ValueError("batch exceeds buffer")
    out = np.zeros(n, dtype=np.uint32)
    _lib.oracle_crc32_batch_fixed(_ptr(a), n, length, stride, _ptr(out))
    return out


def batch_fixed_mt(buf: np.ndarray, n: int, length: int, stride: int | None = None, threads: int = 1) -> np.ndarray:
    stride = length if stride is None else stride
    a = _as_u8(buf)
    if n and (n - 1) * stride + length > a.size:
        raise ValueError("batch exceeds buffer")
    out = np.zeros(n, dtype=np.uint32)
    if _lib.oracle_crc32_batch_fixed_mt(_ptr(a), n, length, stride, _ptr(out), threads) != 0:
        raise RuntimeError("pthread_create failed")
    return out


def batch_var(buf: np.ndarray, offsets: np.ndarray, lengths: np.ndarray) -> np.ndarray:
    a = _as_u8(buf)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    if off.size and int((off + ln.astype(np.uint64)).max()) > a.size:
        raise ValueError("batch exceeds buffer")
    out = np.zeros(off.size, dtype=np.uint32)
    _lib.oracle_crc32_batch_var(_ptr(a), _ptr(off), _ptr(ln), off.size, _ptr(out))
    return out


def batch_var_mt(buf: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, threads: int = 1,
                 states: np.ndarray | None = None) -> np.ndarray:
    """Variable batch over `threads` host threads: crc32_long per payload, or (states given)
    crc32_update of each payload from its register (returns the new registers)."""
    a = _as_u8(buf)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    if off.size and int((off + ln.astype(np.uint64)).max()) > a.size:
        raise ValueError("batch exceeds buffer")
    if states is None:
        out = np.zeros(off.size, dtype=np.uint32)
    else:
        out = np.array(states, dtype=np.uint32, copy=True)
        if out.size != off.size:
            raise ValueError("one register per payload")
    if _lib.oracle_crc32_batch_var_mt(_ptr(a), _ptr(off), _ptr(ln), off.size, _ptr(out), int(states is not None),
                                      threads) != 0:
        raise RuntimeError("pthread_create failed")
    return out


def lcg_bytes(nbytes: int, seed: int) -> np.ndarray:
    """SURVEY.md §8c payload generator (s = s*6364136223846793005 + 1442695040888963407, byte = s>>56)."""
    out = np.empty(nbytes, dtype=np.uint8)
    _lib.oracle_lcg_fill(_ptr(out), nbytes, seed)
    return out


# ---- LengthHeaderCodec frames (include/codec/LengthHeaderCodec.h), checksum enabled ----
DEFAULT_MAX_PAYLOAD = 64 * 1024 * 1024  # LengthHeaderCodec ctor default (:50)


def lhc_encode(payload, length_type: int = 4, max_payload: int = DEFAULT_MAX_PAYLOAD) -> tuple[int, bytes]:
    """One LengthHeaderCodec::encode (:146-201): (rt, bytes appended to the stream)."""
    a = _as_u8(payload)
    out = np.zeros(a.size + 12, dtype=np.uint8)
    n = ctypes.c_size_t()
    rt = _lib.oracle_lhc_encode(length_type, max_payload, _ptr(a), a.size, _ptr(out), ctypes.byref(n))
    return int(rt), out[: n.value].tobytes()


def lhc_decode(stream, length_type: int = 4, max_payload: int = DEFAULT_MAX_PAYLOAD) -> tuple[int, int, int, int]:
    """One LengthHeaderCodec::decode (:71-137): (rt, payload_off, payload_len, consumed)."""
    a = _as_u8(stream)
    off, ln, used = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    rt = _lib.oracle_lhc_decode(length_type, max_payload, _ptr(a) if a.size else None, a.size, ctypes.byref(off),
                                ctypes.byref(ln), ctypes.byref(used))
    return int(rt), off.value, ln.value, used.value


def lhc_recv(stream, length_type: int = 4, max_payload: int = DEFAULT_MAX_PAYLOAD):
    """Codec::recv's loop (include/codec/Codec.h:52-76): decode while rt == 1.
    Returns (frames [(payload_off, payload_len) relative to stream], consumed, last rt)."""
    a = _as_u8(stream)
    frames, pos = [], 0
    while True:
        rt, off, ln, used = lhc_decode(a[pos:], length_type, max_payload)
        if rt != 1:
            return frames, pos, rt
        frames.append((pos + off, ln))
        pos += used


# ---- ProtobufCodec framing (include/protobuf/ProtobufCodec.h) - parity unpinned (needs libprotobuf) ----
def pbc_encode(payload) -> tuple[int, bytes]:
    a = _as_u8(payload)
    out = np.zeros(a.size + 8, dtype=np.uint8)
    n = ctypes.c_size_t()
    rt = _lib.oracle_pbc_encode(_ptr(a) if a.size else None, a.size, _ptr(out), ctypes.byref(n))
    return int(rt), out[: n.value].tobytes()


def pbc_recv(stream):
    """Codec::recv's loop over ProtobufCodec::decode: (frames [(off, len)], consumed, last rt)."""
    a = _as_u8(stream)
    frames, pos = [], 0
    while True:
        off, ln, used = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        sub = a[pos:]
        rt = _lib.oracle_pbc_decode(_ptr(sub) if sub.size else None, sub.size, ctypes.byref(off), ctypes.byref(ln),
                                    ctypes.byref(used))
        if rt != 1:
            return frames, pos, int(rt)
        frames.append((pos + off.value, ln.value))
        pos += used.value


# ---- the compiled reference (only where /root/reference existed at build time) ----
def ref_available() -> bool:
    return os.path.exists(_REF)


_ref = None


def ref_lib() -> ctypes.CDLL:
    global _ref
    if _ref is None:
        if not ref_available():
            raise FileNotFoundError(_REF)
        lib = ctypes.CDLL(_REF)
        for name in ("ref_crc32_long", "ref_crc32_short"):
            f = getattr(lib, name)
            f.restype = ctypes.c_uint32
            f.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        lib.ref_crc32_update.restype = None
        lib.ref_crc32_update.argtypes = [_u32p, ctypes.c_void_p, ctypes.c_size_t]
        lib.ref_tables.restype = None
        lib.ref_tables.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        lib.ref_crc32_batch_fixed.restype = None
        lib.ref_crc32_batch_fixed.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                              ctypes.c_void_p]
        lib.ref_crc32_batch_fixed_mt.restype = ctypes.c_int
        lib.ref_crc32_batch_fixed_mt.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                                 ctypes.c_void_p, ctypes.c_int]
        lib.ref_crc32_batch_var_mt.restype = ctypes.c_int
        lib.ref_crc32_batch_var_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                               ctypes.c_void_p, ctypes.c_int]
        _ref = lib
    return _ref


def ref_codec_lib() -> ctypes.CDLL:
    """The reference's own LengthHeaderCodec (oracle/ref_codec.cc), for fixture generation."""
    lib = ctypes.CDLL(_REF_CODEC)
    _sp = ctypes.POINTER(ctypes.c_size_t)
    lib.ref_lhc_encode.restype = ctypes.c_int
    lib.ref_lhc_encode.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                   ctypes.c_size_t, _sp]
    lib.ref_lhc_decode.restype = ctypes.c_int
    lib.ref_lhc_decode.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                   ctypes.c_size_t, _sp, _sp]
    return lib
