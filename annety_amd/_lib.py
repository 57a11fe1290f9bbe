"""ctypes binding of libannety_crc.so — the same binding a maintainer would add to a Python caller of
annety's checksum. Loading fails loudly: there is no CPU fallback for the batch
path. The single-buffer functions are the reference's host scalar API and run on the CPU by design.
"""
from __future__ import annotations

import ctypes
import os

from . import build as _build

_c_size = ctypes.c_size_t
_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64

# (name, restype, argtypes) — must match include/annety_crc.h exactly.
SIGNATURES = [
    ("annety_crc_abi_version", ctypes.c_int, []),
    ("annety_crc_init", ctypes.c_int, [ctypes.c_int]),
    ("annety_crc_shutdown", ctypes.c_int, []),
    ("annety_crc_strerror", ctypes.c_char_p, [ctypes.c_int]),
    ("annety_crc_last_hip_error", ctypes.c_int, []),
    ("annety_crc_last_error_stage", ctypes.c_char_p, []),
    ("annety_crc_last_kernels", ctypes.c_char_p, []),
    ("annety_crc_set_frames_pack", ctypes.c_int, [ctypes.c_int]),
    ("annety_crc_reserve_cus", ctypes.c_int, [ctypes.c_int]),
    ("annety_crc_set_split", ctypes.c_int, [ctypes.c_int, _u64]),
    ("annety_crc_set_split_cap", ctypes.c_int, [_u32]),
    ("annety_crc_set_walk_segment", ctypes.c_int, [_u64]),
    ("annety_crc_stream_release", ctypes.c_int, [_vp]),
    ("annety_crc_set_var_path", ctypes.c_int, [ctypes.c_int]),
    ("annety_crc_get_var_path", ctypes.c_int, []),
    ("annety_crc_var_path_stats", ctypes.c_int,
     [ctypes.c_int, ctypes.POINTER(_u64), ctypes.POINTER(_u64), ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    ("annety_crc_scratch_stats", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_u64), ctypes.POINTER(_u64),
                                                ctypes.POINTER(_u64)]),
    ("annety_crc32_long", _u32, [_vp, _c_size]),
    ("annety_crc32_short", _u32, [_vp, _c_size]),
    ("annety_crc32_update", None, [ctypes.POINTER(_u32), _vp, _c_size]),
    ("annety_crc32_combine", _u32, [_u32, _u32, _u64]),
    ("annety_crc32_table16", ctypes.POINTER(_u32), []),
    ("annety_crc32_table256", ctypes.POINTER(_u32), []),
    ("annety_crc32_batch_fixed", ctypes.c_int, [_vp, _c_size, _c_size, _c_size, _vp, _vp]),
    ("annety_crc32_batch_var", ctypes.c_int, [_vp, _vp, _vp, _c_size, _vp, _vp]),
    ("annety_crc32_update_batch_fixed", ctypes.c_int, [_vp, _vp, _c_size, _c_size, _c_size, _vp]),
    ("annety_crc32_update_batch_var", ctypes.c_int, [_vp, _vp, _vp, _vp, _c_size, _vp]),
    ("annety_crc32_batch_var_arena", ctypes.c_int, [_vp, _c_size, _vp, _vp, _c_size, _vp, _vp]),
    ("annety_crc32_update_batch_var_arena", ctypes.c_int, [_vp, _vp, _c_size, _vp, _vp, _c_size, _vp]),
    ("annety_crc32_batch_fixed_host", ctypes.c_int, [_vp, _c_size, _c_size, _c_size, _vp]),
    ("annety_crc_host_register", ctypes.c_int, [_vp, _c_size]),
    ("annety_crc_host_unregister", ctypes.c_int, [_vp]),
    ("annety_crc_shard_plan", ctypes.c_int, [_c_size, ctypes.c_int, _vp, _vp]),
    ("annety_crc_group_schedule", ctypes.c_int, [_vp, ctypes.c_int, _c_size, _vp]),
    ("annety_crc_group_create", ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(_vp)]),
    ("annety_crc_group_destroy", ctypes.c_int, [_vp]),
    ("annety_crc_group_size", ctypes.c_int, [_vp]),
    ("annety_crc32_group_batch_fixed", ctypes.c_int, [_vp, _vp, _vp, _c_size, _c_size, _vp, _c_size]),
    ("annety_crc32_group_batch_fixed_host", ctypes.c_int, [_vp, _vp, _c_size, _c_size, _c_size, _vp]),
    ("annety_lhc_parse", ctypes.c_int, [_vp, _c_size, ctypes.c_int, ctypes.c_int64, _vp, _vp, _c_size,
                                        ctypes.POINTER(_c_size), ctypes.POINTER(_c_size)]),
    ("annety_lhc_verify_batch", ctypes.c_int, [_vp, _vp, _vp, _c_size, _vp, _vp, _vp]),
    ("annety_lhc_verify_stream", ctypes.c_int, [_vp, _c_size, _vp, _vp, _c_size, _vp, _vp, _vp]),
    ("annety_lhc_verify_host", ctypes.c_int, [_vp, _c_size, ctypes.c_int, ctypes.c_int64, _vp, _vp, _vp, _c_size,
                                              ctypes.POINTER(_c_size), ctypes.POINTER(_c_size)]),
    ("annety_lhc_verify_host_iov", ctypes.c_int, [_vp, _vp, _c_size, ctypes.c_int, ctypes.c_int64, _vp, _vp, _vp,
                                                  _c_size, _vp, _vp, _vp]),
    ("annety_pbc_verify_host_iov", ctypes.c_int, [_vp, _vp, _c_size, _vp, _vp, _vp, _c_size, _vp, _vp, _vp]),
    ("annety_pbc_parse", ctypes.c_int, [_vp, _c_size, _vp, _vp, _c_size, ctypes.POINTER(_c_size),
                                        ctypes.POINTER(_c_size)]),
    ("annety_pbc_verify_host", ctypes.c_int, [_vp, _c_size, _vp, _vp, _vp, _c_size, ctypes.POINTER(_c_size),
                                              ctypes.POINTER(_c_size)]),
    ("annety_pbc_encode_plan", ctypes.c_int, [_vp, _c_size, _vp, _vp, ctypes.POINTER(_u64)]),
    ("annety_pbc_encode_batch", ctypes.c_int, [_vp, _vp, _vp, _c_size, _vp, _vp, _vp]),
    ("annety_lhc_encode_plan", ctypes.c_int, [_vp, _c_size, ctypes.c_int, ctypes.c_int64, _vp, _vp,
                                              ctypes.POINTER(_u64)]),
    ("annety_lhc_encode_batch", ctypes.c_int, [_vp, _vp, _vp, _c_size, ctypes.c_int, ctypes.c_int64, _vp, _vp,
                                               _vp]),
]

_lib: ctypes.CDLL | None = None


class CrcError(RuntimeError):
    def __init__(self, status: int, where: str):
        lib = get()
        msg = lib.annety_crc_strerror(status).decode()
        hip = lib.annety_crc_last_hip_error()
        stage = (lib.annety_crc_last_error_stage() or b"").decode()
        super().__init__(f"{where}: {msg} (status {status}, hipError {hip}"
                         + (f", stage: {stage})" if stage and hip else ")"))
        self.status = status
        self.stage = stage


def lib_path() -> str:
    return _build.LIB


def get() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        # ANNETY_CRC_HOST_LIB: a host-only sanitizer build of crc32_host.cpp (annety_amd/csrc/Makefile), for
        # running the host-side tests (frame walks, encode plans, shard plans) under ASan/UBSan or TSan; it
        # exports the host entry points only, so the device ones stay unbound and any call to them fails.
        host_only = os.environ.get("ANNETY_CRC_HOST_LIB")
        # ANNETY_CRC_LIB: another full build of the library (same-box A/B against a baseline commit's build)
        path = host_only or os.environ.get("ANNETY_CRC_LIB") or _build.LIB
        if path == _build.LIB and not os.path.exists(_build.LIB):
            _build.build()  # raises if hipcc is unavailable: no silent fallback
        lib = ctypes.CDLL(path)
        for name, res, args in SIGNATURES:
            if host_only and not hasattr(lib, name):
                continue
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        _lib = lib
    return _lib


def check(status: int, where: str) -> None:
    if status != 0:
        raise CrcError(status, where)
