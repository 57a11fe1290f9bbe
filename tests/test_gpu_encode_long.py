"""Long frames in the fused encode (crc32_kernels.h EncLong): a frame of more than kEncLongMin payload bytes is handed
over by its lane group to the long path (segment digests on crc32_var_sorted_kernel, then lhc_encode_long_kernel's
grid-wide copy, header and trailer). Every frame against the oracle's encoder (LengthHeaderCodec::encode,
include/codec/LengthHeaderCodec.h:146-201): lengths at the threshold, unaligned sources and destinations, frames of
several MiB beside short ones, a frame past 256 MiB (1 MiB segments), more long frames than the segment cap holds
(the rest run on their groups), and a second call on the same stream (the counters of the alternate set)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

LONG = 262144  # kEncLongMin


def _check(gpu, lens, seed, T=4, gap=3, calls=1, max_payload=1 << 30):
    import torch

    from annety_amd.codec import LengthHeaderCodec

    rng = np.random.default_rng(seed)
    lens = np.asarray(lens, dtype=np.uint32)
    gaps = rng.integers(0, gap + 1, lens.size).astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + gaps)[:-1]]).astype(np.uint64) + 5
    arena = oracle.lcg_bytes(int(offs[-1] + lens[-1]) + 64, seed)
    d_src = torch.from_numpy(arena.copy()).to(gpu)
    codec = LengthHeaderCodec(T, True, max_payload)
    kernels = None
    for _ in range(calls):
        r = codec.encode_batch(d_src, offs, lens)
        torch.cuda.synchronize()
        import annety_amd

        kernels = annety_amd.last_kernels()
        frames = r.frames.cpu().numpy()
        pos = 0
        for i, (o, L) in enumerate(zip(offs, lens)):
            rt, want = oracle.lhc_encode(arena[int(o): int(o) + int(L)], T, max_payload)
            got = frames[pos: pos + len(want)].tobytes()
            assert got == want, (i, int(L))
            pos += len(want)
        assert pos == frames.size
        del r, frames
    return kernels


def test_long_frames_at_the_threshold(gpu):
    lens = [LONG, LONG + 1, LONG + 15, LONG + 16384, 300000, (1 << 20) + 7, 5000, 0, 1, 17, LONG + 3]
    kernels = _check(gpu, lens, 1)
    assert "lhc_encode_long_kernel" in kernels


def test_long_frames_among_short_ones(gpu):
    rng = np.random.default_rng(2)
    lens = np.concatenate([rng.integers(0, 3000, 5000), rng.integers(LONG + 1, 3 << 20, 40), [17 << 20, (9 << 20) + 5]])
    for T in (4, 8):
        _check(gpu, rng.permutation(lens), 3, T=T, gap=9)


def test_long_frame_past_256_mib(gpu):
    _check(gpu, [(300 << 20) + 77, 4000, LONG + 9], 4, gap=1)


def test_more_long_frames_than_the_cap(gpu):
    # 16 frames of 4097 segments: 65552 > kEncLongSegCap, so one runs on its lane group
    _check(gpu, [(64 << 20) + 1] * 16 + [100, 200], 5, gap=0)


def test_two_calls_alternate_counters(gpu):
    _check(gpu, [LONG + 100, 2000, (2 << 20) + 3, 0, 64], 6, calls=3)


def test_rejected_long_frames_write_nothing(gpu):
    # payloads over max_payload get no frame (LengthHeaderCodec::encode :169-176), long or not
    _check(gpu, [400000, LONG + 5, 290000, 300001, 1000, 300000], 7, max_payload=300000)
