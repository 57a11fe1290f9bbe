"""Long payloads on the arena path (crc32_arena.hip Stitcher::mid_join): the whole superblocks between a payload's
partial ones are joined on its own lane up to kLongMid = 64 of them, by the whole wave past that (VERDICT r05 item
5: a 64 MiB payload was 8k serial steps on one lane). Digests and update registers against the oracle at the
kLongMid boundary, for payloads of many MiB mixed with short ones at every alignment class, several long payloads
in one wave, and LengthHeaderCodec frames of the codec's largest size (64 MiB, LengthHeaderCodec.h:51) through
annety_lhc_verify_stream, with the call's device time printed."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

SB = 8192


def _dev_bytes(gpu, total, seed):
    import torch

    g = torch.Generator(device=gpu)
    g.manual_seed(seed)
    d = torch.randint(0, 256, (total,), dtype=torch.uint8, device=gpu, generator=g)
    return d, d.cpu().numpy()


def _arena(gpu, lens, seed, update=False, gap=0, calls=1):
    """The payloads packed (with `gap` bytes between them) in one arena; digests (or registers over `calls` calls)
    against the oracle; returns the last call's device time in ms."""
    import torch

    import annety_amd

    lens = np.asarray(lens, dtype=np.int64)
    offs = (np.concatenate([[0], np.cumsum(lens + gap)[:-1]]) + (seed % 113)).astype(np.int64)
    total = int(offs[-1] + lens[-1]) + 64
    d, data = _dev_bytes(gpu, total, seed)
    o = torch.from_numpy(offs).to(gpu)
    ln = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    rng = np.random.default_rng(seed)
    want = rng.integers(0, 1 << 32, lens.size, dtype=np.uint64).astype(np.uint32)
    out = torch.from_numpy(want.view(np.int32).copy()).to(gpu)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(calls):
        e0.record()
        if update:
            annety_amd.crc32_update_batch_var(out, d, o, ln, arena=True)
        else:
            annety_amd.crc32_batch_var(d, o, ln, out=out, arena=True)
        e1.record()
        want = oracle.batch_var_mt(data, offs.astype(np.uint64), lens.astype(np.uint32), threads=16,
                                   states=want if update else None)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, (bad[:8], lens[bad[:8]])
    return e0.elapsed_time(e1)


@pytest.mark.parametrize("update", [False, True])
def test_runs_around_the_wave_threshold(gpu, update):
    """Payloads whose whole-superblock runs are 63..67 long (the lane's chain up to 64, the wave's past it) at
    every 16-byte alignment class, mixed with short ones."""
    rng = np.random.default_rng(1)
    lens = []
    for k in range(63, 68):
        for r in (0, 1, 129, 1023, 1024 + 77, 8191, 8192 + 5):
            lens.append(k * SB + r)
    lens += [int(x) for x in rng.integers(0, 5000, 300)]
    _arena(gpu, [int(x) for x in rng.permutation(lens)], 2, update=update, calls=2 if update else 1)


@pytest.mark.parametrize("update", [False, True])
def test_many_mib_payloads(gpu, update):
    """16 payloads of 20-80 MiB among 4000 short ones: long runs in many waves, several in one wave."""
    rng = np.random.default_rng(3)
    lens = [int(x) for x in rng.integers(20 << 20, 80 << 20, 16)] + [int(x) for x in rng.integers(1, 9000, 4000)]
    ms = _arena(gpu, [int(x) for x in rng.permutation(lens)], 4, update=update, calls=2 if update else 1)
    print(f"arena, 16 long payloads among 4000 short ({'update' if update else 'digests'}): {ms:.3f} ms per call")


def test_adjacent_long_payloads_one_wave(gpu):
    """64 payloads of 1-2 MiB packed back to back: consecutive payloads are consecutive lanes of a wave, so one wave
    joins dozens of runs one after another."""
    rng = np.random.default_rng(5)
    _arena(gpu, [int(x) for x in rng.integers(1 << 20, 2 << 20, 64)], 6)


def test_verify_stream_64mib_frames(gpu):
    """LengthHeaderCodec frames of 64 MiB (the codec's default max_payload) through annety_lhc_verify_stream: every
    verdict 1 and every digest the oracle's, one flipped byte caught, and the device time of one call (one lane per
    frame took ~2 ms for 16 such frames before the wave join)."""
    import torch

    import annety_amd

    n, L = 16, (64 << 20) - 64
    lens = np.full(n, L, dtype=np.int64) - np.arange(n, dtype=np.int64) * 13
    src_off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    d_src, src = _dev_bytes(gpu, int(lens.sum()) + 64, 7)
    codec = annety_amd.LengthHeaderCodec(4, True, 64 << 20)
    enc = codec.encode_batch(d_src, src_off.astype(np.uint64), lens.astype(np.uint32))
    torch.cuda.synchronize()
    frames = enc.frames
    d_off = torch.from_numpy(enc.frame_off.astype(np.int64) + 4).to(gpu)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(gpu)
    want = oracle.batch_var_mt(src, src_off.astype(np.uint64), lens.astype(np.uint32), threads=16)
    ok = torch.zeros(n, dtype=torch.uint8, device=gpu)
    dig = torch.zeros(n, dtype=torch.int32, device=gpu)
    codec.verify(frames, d_off, d_len, out_ok=ok, out_digest=dig)  # warm
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    codec.verify(frames, d_off, d_len, out_ok=ok, out_digest=dig)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    print(f"verify stream, 16 x 64 MiB frames: {ms:.3f} ms per call ({annety_amd.last_kernels()})")
    assert bool((ok == 1).all()) and np.array_equal(dig.cpu().numpy().view(np.uint32), want)
    # a flipped byte in the middle of frame 5 fails that frame only
    pos = int(enc.frame_off[5]) + 4 + L // 2
    frames[pos] ^= 0x40
    codec.verify(frames, d_off, d_len, out_ok=ok, out_digest=dig)
    torch.cuda.synchronize()
    assert np.flatnonzero(ok.cpu().numpy() != 1).tolist() == [5]
    assert ms < 2.0, ms
