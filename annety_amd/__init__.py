"""annety_amd — MI355X-native engine for annety's checksum path (CRC-32 batches on gfx950).

Public surface:
  Crc32c                  mirror of annety::Crc32c (include/Crc32c.h:22-83)
  crc32_batch             device-resident fixed-length batch   (C-ABI annety_crc32_batch_fixed)
  crc32_batch_var         device-resident variable-length batch (annety_crc32_batch_var)
  crc32_update_batch      raw-register batch update            (annety_crc32_update_batch_fixed)
  crc32_update_batch_var  streaming update, one fragment/stream (annety_crc32_update_batch_var)
  StreamingCrc            per-stream device registers over crc32_update_batch_var
  crc32_batch_host        host-memory batch, staged over PCIe  (annety_crc32_batch_fixed_host)
  crc32_combine           join two digests                     (annety_crc32_combine)
  LengthHeaderCodec       batched frame verify/build for annety's LengthHeaderCodec wire format
  ProtobufCodecFrames     the same for ProtobufCodec's framing (T = 4, 10 B .. 64 MiB)
  PinnedHostBuffer        host arena registered for in-place DMA (annety_crc_host_register)
  sharded                 multi-GPU batch sharding helpers (torch.distributed / RCCL)
"""
from .crc32c import (  # noqa: F401
    Crc32c,
    crc32_batch,
    crc32_batch_host,
    crc32_batch_var,
    crc32_combine,
    crc32_update_batch,
    crc32_update_batch_var,
    PinnedHostBuffer,
    StreamingCrc,
    digests_to_numpy,
    last_kernels,
    reserve_cus,
    scratch_stats,
    set_frames_pack,
    set_split,
    set_split_cap,
    set_walk_segment,
    stream_release,
    set_var_path,
    var_path_stats,
    tables,
)
from ._lib import CrcError, lib_path  # noqa: F401
from .codec import LengthHeaderCodec, ProtobufCodecFrames  # noqa: F401

__all__ = [
    "Crc32c",
    "crc32_batch",
    "crc32_batch_var",
    "crc32_update_batch",
    "crc32_update_batch_var",
    "StreamingCrc",
    "PinnedHostBuffer",
    "crc32_batch_host",
    "crc32_combine",
    "digests_to_numpy",
    "last_kernels",
    "reserve_cus",
    "scratch_stats",
    "set_frames_pack",
    "set_split",
    "set_split_cap",
    "set_walk_segment",
    "stream_release",
    "set_var_path",
    "var_path_stats",
    "tables",
    "LengthHeaderCodec",
    "ProtobufCodecFrames",
    "CrcError",
    "lib_path",
]
