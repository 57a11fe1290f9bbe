"""Host-side mirror of annety's checksum API over the MI355X engine.

`Crc32c` mirrors the reference class annety::Crc32c (include/Crc32c.h:22-83) method for method:
same names, same argument meaning, same values. The single-buffer methods run on the calling CPU
thread exactly like the reference's inline code (through the C-ABI's host functions); the batch
functions below are the data-parallel hot path and run ONLY on the GPU — there is no CPU fallback.

Batch functions take torch tensors resident on a ROCm device (torch is device-memory/stream plumbing
here) or raw device pointers, and launch on the current torch stream unless one is given.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Union

import numpy as np

from . import _lib

BytesLike = Union[bytes, bytearray, memoryview, np.ndarray]


def _host_view(buff: BytesLike) -> tuple[int, int, object]:
    """(address, length, keepalive) of a host byte buffer without copying when possible."""
    if isinstance(buff, np.ndarray):
        a = np.ascontiguousarray(buff).view(np.uint8).reshape(-1)
        return a.ctypes.data, a.size, a
    if isinstance(buff, str):
        buff = buff.encode()
    if isinstance(buff, (bytes, bytearray, memoryview)):
        a = np.frombuffer(buff, dtype=np.uint8)
        return (a.ctypes.data if a.size else 0), a.size, a
    raise TypeError(f"expected a bytes-like object, got {type(buff).__name__}")


class Crc32c:
    """Drop-in mirror of annety::Crc32c (include/Crc32c.h:22-83)."""

    @staticmethod
    def crc32_short(buff: BytesLike, length: Optional[int] = None) -> int:
        """include/Crc32c.h:41-55 (also the StringPiece overload :25-28)."""
        addr, n, keep = _host_view(buff)
        n = n if length is None else min(length, n)
        return int(_lib.get().annety_crc32_short(addr, n))

    @staticmethod
    def crc32_long(buff: BytesLike, length: Optional[int] = None) -> int:
        """include/Crc32c.h:58-69 (also the StringPiece overload :30-33)."""
        addr, n, keep = _host_view(buff)
        n = n if length is None else min(length, n)
        return int(_lib.get().annety_crc32_long(addr, n))

    @staticmethod
    def crc32_update(crc: int, buff: BytesLike, length: Optional[int] = None) -> int:
        """include/Crc32c.h:71-82. The reference updates `*crc` in place; Python returns the new
        register (no init, no final xor)."""
        addr, n, keep = _host_view(buff)
        n = n if length is None else min(length, n)
        s = ctypes.c_uint32(crc & 0xFFFFFFFF)
        _lib.get().annety_crc32_update(ctypes.byref(s), addr, n)
        return int(s.value)

    # ---- additive batch API (device) ----
    @staticmethod
    def crc32_long_batch(data, n: int, length: int, stride: Optional[int] = None, out=None, stream=None):
        return crc32_batch(data, n, length, stride, out, stream)

    @staticmethod
    def crc32_combine(crc_a: int, crc_b: int, len_b: int) -> int:
        return crc32_combine(crc_a, crc_b, len_b)


def crc32_combine(crc_a: int, crc_b: int, len_b: int) -> int:
    """crc(A||B) from crc(A), crc(B) and |B|."""
    return int(_lib.get().annety_crc32_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, len_b))


def reserve_cus(n: int) -> None:
    """Leave n CUs of every device free of the batch kernels (annety_crc_reserve_cus), e.g. for the RCCL
    kernels of a gather that overlaps the next chunk's checksums; 0 uses every CU."""
    _lib.check(_lib.get().annety_crc_reserve_cus(int(n)), "annety_crc_reserve_cus")


def set_walk_segment(nbytes: int = 0) -> None:
    """annety_crc_set_walk_segment: segment size of the host frame walks (0 = default 64 MiB), process-wide."""
    _lib.check(_lib.get().annety_crc_set_walk_segment(int(nbytes)), "annety_crc_set_walk_segment")


def set_frames_pack(pack: bool = True) -> None:
    """annety_crc_set_frames_pack: receive buffers not pinned through PinnedHostBuffer are packed into the
    library's pinned ring (True, default) or handed to the runtime's pageable copy (False). Process-wide."""
    _lib.check(_lib.get().annety_crc_set_frames_pack(1 if pack else 0), "annety_crc_set_frames_pack")


def last_kernels() -> str:
    """annety_crc_last_kernels: the kernels this thread's latest device call enqueued, in order."""
    return (_lib.get().annety_crc_last_kernels() or b"").decode()


def set_split(mode: int = -1, min_segment: int = 0) -> None:
    """annety_crc_set_split: long-payload split policy (-1 auto, 0 never, 1 always), process-wide."""
    _lib.check(_lib.get().annety_crc_set_split(int(mode), int(min_segment)), "annety_crc_set_split")


def set_split_cap(extra_segments: int = 1 << 18) -> None:
    """annety_crc_set_split_cap: segment descriptors a sorted-path call may add for its long payloads
    (default and maximum 2^18; 0 = long payloads run whole), process-wide."""
    _lib.check(_lib.get().annety_crc_set_split_cap(int(extra_segments)), "annety_crc_set_split_cap")


def scratch_stats(device: int = 0) -> dict:
    """annety_crc_scratch_stats: streams holding a scratch slot on `device`, slot hand-overs between
    streams and device-wide synchronisations so far."""
    import ctypes

    v = [ctypes.c_uint64() for _ in range(3)]
    _lib.check(_lib.get().annety_crc_scratch_stats(int(device), *[ctypes.byref(x) for x in v]),
               "annety_crc_scratch_stats")
    return {"slots": v[0].value, "handoffs": v[1].value, "device_syncs": v[2].value}


VAR_PATHS = {"auto": 0, "sorted": 1}


def set_var_path(path: str) -> str:
    """annety_crc_set_var_path: the path of crc32_batch_var / crc32_update_batch_var, process-wide ("auto" =
    arena or length-sorted from recorded extents, "sorted"). Returns the previous path. Digests do not depend
    on it."""
    lib = _lib.get()
    prev = {v: k for k, v in VAR_PATHS.items()}[lib.annety_crc_get_var_path()]
    _lib.check(lib.annety_crc_set_var_path(VAR_PATHS[path]), "annety_crc_set_var_path")
    return prev


def var_path_stats(device: int = 0) -> dict:
    """annety_crc_var_path_stats: how many automatic variable-batch calls the host sent to the arena / sorted path
    from recorded extents, how many of those arena calls ran without recording their extent ("arena_unrecorded"),
    and how many calls the device chose for ("device")."""
    import ctypes

    a, b, u, d = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    _lib.check(_lib.get().annety_crc_var_path_stats(int(device), ctypes.byref(a), ctypes.byref(b), ctypes.byref(u),
                                                    ctypes.byref(d)), "annety_crc_var_path_stats")
    return {"arena": a.value, "sorted": b.value, "arena_unrecorded": u.value, "device": d.value}


def stream_release(stream) -> None:
    """annety_crc_stream_release: drop a stream's scratch (stream-ordered) before the stream is destroyed."""
    h = stream if isinstance(stream, int) else int(stream.cuda_stream)
    dev = getattr(stream, "device", None)
    with _on_device(stream) if dev is not None else _nullctx():
        _lib.check(_lib.get().annety_crc_stream_release(h), "annety_crc_stream_release")


def _nullctx():
    import contextlib

    return contextlib.nullcontext()


def tables() -> tuple[np.ndarray, np.ndarray]:
    """The drop-in's annety::internal::crc32_table256/16 (src/Crc32c.cc:20-92)."""
    lib = _lib.get()
    t256 = np.ctypeslib.as_array(lib.annety_crc32_table256(), shape=(256,)).copy()
    t16 = np.ctypeslib.as_array(lib.annety_crc32_table16(), shape=(16,)).copy()
    return t256, t16


# ---------------- device batch path ----------------
def _dev_ptr(x) -> int:
    if isinstance(x, int):
        return x
    return int(x.data_ptr())


def _stream_handle(stream, like) -> int:
    if stream is None:
        import torch

        dev = like.device if hasattr(like, "device") else None
        return int(torch.cuda.current_stream(dev).cuda_stream)
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)


def _require_device(t, name: str) -> None:
    if hasattr(t, "is_cuda") and not t.is_cuda:
        raise ValueError(f"{name} must be a device (ROCm) tensor; the batch path has no CPU fallback")


def _on_device(*tensors):
    """Context making the tensors' device current for the C call: the C-ABI picks its per-device state
    (LDS table images, scratch pool) from hipGetDevice(), so it must match where the data lives."""
    import contextlib

    import torch

    devs = {t.device for t in tensors if hasattr(t, "device")}
    if len(devs) > 1:
        raise ValueError(f"batch tensors are on different devices: {sorted(str(d) for d in devs)}")
    return torch.cuda.device(devs.pop()) if devs else contextlib.nullcontext()


def _arena_bytes(data, arena) -> Optional[int]:
    """None: general (sparse) path; True: the whole of `data`; int: that many bytes from data[0]."""
    if arena is None or arena is False:
        return None
    if arena is True:
        if not hasattr(data, "numel"):
            raise ValueError("arena=True needs a tensor; pass the arena size in bytes for a raw pointer")
        return int(data.numel() * data.element_size())
    return int(arena)


def crc32_batch(data, n: int, length: int, stride: Optional[int] = None, out=None, stream=None):
    """Digests of n fixed-length payloads: payload i = data[i*stride : i*stride + length].

    `data`: uint8 device tensor (or raw device pointer with `out` given). Returns `out`, an int32 tensor
    of n digests (bit pattern = the uint32 CRC; `.view(torch.uint32)` or `& 0xFFFFFFFF` to read).
    """
    import torch

    stride = length if stride is None else stride
    _require_device(data, "data")
    if hasattr(data, "numel") and n > 0 and (n - 1) * stride + length > data.numel() * data.element_size():
        raise ValueError("batch extends past the end of `data`")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=data.device)
    _require_device(out, "out")
    with _on_device(data, out):
        st = _lib.get().annety_crc32_batch_fixed(_dev_ptr(data), n, length, stride, _dev_ptr(out),
                                                 _stream_handle(stream, out))
    _lib.check(st, "annety_crc32_batch_fixed")
    return out


def crc32_batch_var(data, offsets, lengths, out=None, stream=None, arena=None):
    """Digests of payload i = data[offsets[i] : offsets[i] + lengths[i]] (any alignment).
    offsets: int64 device tensor, lengths: int32 device tensor.
    arena: None = general path (length-bucketed, any layout); True / a byte count = the payloads lie in
    data[0 : arena] and cover most of it (packed batch, frame stream): one pass over the arena."""
    import torch

    _require_device(data, "data")
    n = int(offsets.numel())
    if offsets.dtype != torch.int64 or lengths.dtype != torch.int32 or lengths.numel() != n:
        raise ValueError("offsets must be int64[n] and lengths int32[n]")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=data.device)
    ab = _arena_bytes(data, arena)
    with _on_device(data, offsets, lengths, out):
        sh = _stream_handle(stream, out)
        if ab is None:
            st = _lib.get().annety_crc32_batch_var(_dev_ptr(data), _dev_ptr(offsets), _dev_ptr(lengths), n,
                                                   _dev_ptr(out), sh)
        else:
            st = _lib.get().annety_crc32_batch_var_arena(_dev_ptr(data), ab, _dev_ptr(offsets), _dev_ptr(lengths), n,
                                                         _dev_ptr(out), sh)
    _lib.check(st, "annety_crc32_batch_var" + ("" if ab is None else "_arena"))
    return out


def crc32_update_batch(state, data, n: int, length: int, stride: Optional[int] = None, stream=None):
    """In-place raw-register update (crc32_update semantics) of state[i] over payload i."""
    stride = length if stride is None else stride
    _require_device(data, "data")
    _require_device(state, "state")
    with _on_device(data, state):
        st = _lib.get().annety_crc32_update_batch_fixed(_dev_ptr(state), _dev_ptr(data), n, length, stride,
                                                        _stream_handle(stream, state))
    _lib.check(st, "annety_crc32_update_batch_fixed")
    return state


def crc32_update_batch_var(state, data, offsets, lengths, stream=None, arena=None):
    """Streaming update: state[i] (int32 device tensor, uint32 bit patterns) advanced in place over
    fragment i = data[offsets[i] : offsets[i] + lengths[i]] (crc32_update semantics). `arena` as in
    crc32_batch_var."""
    import torch

    _require_device(data, "data")
    _require_device(state, "state")
    n = int(offsets.numel())
    if offsets.dtype != torch.int64 or lengths.dtype != torch.int32 or lengths.numel() != n or state.numel() != n:
        raise ValueError("offsets must be int64[n], lengths int32[n], state int32[n]")
    ab = _arena_bytes(data, arena)
    with _on_device(data, offsets, lengths, state):
        sh = _stream_handle(stream, state)
        if ab is None:
            st = _lib.get().annety_crc32_update_batch_var(_dev_ptr(state), _dev_ptr(data), _dev_ptr(offsets),
                                                          _dev_ptr(lengths), n, sh)
        else:
            st = _lib.get().annety_crc32_update_batch_var_arena(_dev_ptr(state), _dev_ptr(data), ab,
                                                                _dev_ptr(offsets), _dev_ptr(lengths), n, sh)
    _lib.check(st, "annety_crc32_update_batch_var" + ("" if ab is None else "_arena"))
    return state


class StreamingCrc:
    """Per-stream CRC registers on the device for payloads that arrive in fragments (one read_fd call
    per connection at a time, src/TcpConnection.cc:445-448): seed 0xFFFFFFFF, crc32_update per
    fragment, final xor - the reference's crc32_update protocol (include/Crc32c.h:71-82) batched over
    streams."""

    def __init__(self, n_streams: int, device=None):
        import torch

        self.state = torch.full((n_streams,), -1, dtype=torch.int32, device=device or "cuda")

    def update(self, data, offsets, lengths, stream=None, arena=None):
        crc32_update_batch_var(self.state, data, offsets, lengths, stream, arena)
        return self

    def digests(self):
        """crc32_long of each stream's bytes so far (int32 device tensor of uint32 bit patterns)."""
        return self.state ^ -1

    def reset(self, mask=None):
        if mask is None:
            self.state.fill_(-1)
        else:
            self.state[mask] = -1


def crc32_batch_host(buf: BytesLike, n: int, length: int, stride: Optional[int] = None) -> np.ndarray:
    """Host-memory batch: staged to the current device and back (synchronous). Returns uint32[n]."""
    stride = length if stride is None else stride
    addr, size, keep = _host_view(buf)
    if n > 0 and (n - 1) * stride + length > size:
        raise ValueError("batch extends past the end of `buf`")
    out = np.zeros(n, dtype=np.uint32)
    st = _lib.get().annety_crc32_batch_fixed_host(addr, n, length, stride, out.ctypes.data)
    _lib.check(st, "annety_crc32_batch_fixed_host")
    return out


class PinnedHostBuffer:
    """A host buffer registered with the device runtime (annety_crc_host_register), e.g. the arena a
    NetBuffer reads sockets into: host batches over it are copied to the device in place.

    The memory is an anonymous mapping of whole pages, so the registration starts on a page boundary and
    shares no page with any other buffer (the library refuses registrations that would: DESIGN.md 7.3)."""

    def __init__(self, nbytes: int):
        import mmap

        nbytes = max(1, int(nbytes))
        pg = mmap.PAGESIZE
        self._map = mmap.mmap(-1, (nbytes + pg - 1) // pg * pg, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        self._pages = np.frombuffer(self._map, dtype=np.uint8)
        self.array = self._pages[:nbytes]
        _lib.check(_lib.get().annety_crc_host_register(self._pages.ctypes.data, self._pages.size),
                   "annety_crc_host_register")

    def close(self):
        if self.array is None:
            return
        _lib.get().annety_crc_host_unregister(self._pages.ctypes.data)
        self.array = self._pages = None
        try:
            self._map.close()  # BufferError while a caller still holds a view: the mapping then goes with it
        except BufferError:
            pass
        self._map = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def digests_to_numpy(out) -> np.ndarray:
    """int32 device tensor of digests -> uint32 numpy array."""
    return out.detach().cpu().numpy().view(np.uint32)
