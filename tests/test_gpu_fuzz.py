"""Randomised batches through every device entry point against the oracle (seeded, reproducible).

Layouts: packed, gapped (gaps up to 6 KiB), shuffled, overlapping at random offsets, one payload
repeated; lengths from 0 to 200 KB; digests and update registers; fixed batches with unaligned bases and
padded strides. Each variable family keeps its device tensors across rounds and rewrites their contents,
so the automatic path's per-stream records see layouts change under the same pointers (recorded and
unrecorded arena calls, sorted calls, path switches)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _lengths(rng, n):
    kind = rng.integers(0, 4)
    if kind == 0:
        return rng.integers(0, 200, n)
    if kind == 1:
        # zipf draws reach 1e17 and more: clip before scaling, or 64 * z wraps negative
        return np.minimum(200_000, 64 * np.minimum(rng.zipf(1.3, n), 1 << 20) + rng.integers(0, 64, n))
    if kind == 2:
        return rng.integers(0, 20_000, n)
    out = rng.integers(1, 5000, n)
    out[rng.integers(0, n, max(1, n // 10))] = 0
    return out


def _layout(rng, lens, size_hint):
    kind = ["packed", "gapped", "shuffled", "overlap", "repeat"][rng.integers(0, 5)]
    n = len(lens)
    if kind == "packed":
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]) + int(rng.integers(0, 100))
    elif kind == "gapped":
        offs = np.concatenate([[0], np.cumsum(lens + rng.integers(0, 6000, n))[:-1]])
    elif kind == "shuffled":
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
        perm = rng.permutation(n)
        offs, lens = offs[perm], lens[perm]
    elif kind == "overlap":
        span = max(int(size_hint), int(lens.max()) + 1)
        offs = rng.integers(0, span - lens + 1)
    else:
        lens = np.full(n, lens[0])
        offs = np.full(n, int(rng.integers(0, 1000)))
    return kind, offs.astype(np.int64), lens.astype(np.int64)


def test_variable_families(gpu):
    import torch

    import annety_amd

    rng = np.random.default_rng(20261016)
    for fam in range(24):
        n = int(rng.choice([5, 300, 1500, 4000]))
        cap_bytes = 8 << 20
        d = torch.zeros(cap_bytes, dtype=torch.uint8, device=gpu)
        o = torch.zeros(n, dtype=torch.int64, device=gpu)
        ln = torch.zeros(n, dtype=torch.int32, device=gpu)
        out = torch.zeros(n, dtype=torch.int32, device=gpu)
        for rnd in range(6):
            lens = _lengths(rng, n)
            kind, offs, lens = _layout(rng, lens, cap_bytes // 4)
            need = int((offs + lens).max()) + 1
            if need > cap_bytes:  # scale the layout into the buffer
                scale = cap_bytes / need
                lens = (lens * scale * 0.5).astype(np.int64)
                offs = (offs * scale * 0.5).astype(np.int64)
            host = rng.integers(0, 256, cap_bytes, dtype=np.uint8)
            d.copy_(torch.from_numpy(host))
            o.copy_(torch.from_numpy(offs))
            ln.copy_(torch.from_numpy(lens.astype(np.int32)))
            mode = int(rng.integers(0, 3))
            ctx = (fam, rnd, kind, mode, n)
            if mode == 2:  # update registers, automatic path
                st0 = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
                out.copy_(torch.from_numpy(st0.view(np.int32)))
                annety_amd.crc32_update_batch_var(out, d, o, ln)
                want = oracle.batch_var_mt(host, offs.astype(np.uint64), lens.astype(np.uint32), threads=8, states=st0)
            else:
                out.fill_(7)
                annety_amd.crc32_batch_var(d, o, ln, out=out, arena=True if mode == 1 else None)
                want = oracle.batch_var_mt(host, offs.astype(np.uint64), lens.astype(np.uint32), threads=8)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            assert np.array_equal(got, want), (ctx, int((got != want).sum()))


def test_fixed_shapes(gpu):
    import torch

    import annety_amd

    rng = np.random.default_rng(77)
    host = rng.integers(0, 256, 16 << 20, dtype=np.uint8)
    d = torch.from_numpy(host).to(gpu)
    for case in range(40):
        length = int(rng.choice([1, 3, 4, 15, 16, 17, 127, 128, 1000, 1024, 4096, 5000, 65536, 200_000]))
        stride = length + int(rng.choice([0, 0, 1, 16, 100]))
        base = int(rng.integers(0, 64))
        n = int(max(1, min(int(rng.integers(1, 3000)), (len(host) - base - length) // stride + 1)))
        want = oracle.batch_fixed_mt(host[base:], n, length, stride, threads=8)
        got = annety_amd.crc32_batch(d[base:], n, length, stride)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy().view(np.uint32), want), (case, length, stride, base, n)
        st0 = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        state = torch.from_numpy(st0.view(np.int32).copy()).to(gpu)
        annety_amd.crc32_update_batch(state, d[base:], n, length, stride)
        offs = (np.arange(n, dtype=np.uint64) * stride).astype(np.uint64)
        want_u = oracle.batch_var_mt(host[base:], offs, np.full(n, length, np.uint32), threads=8, states=st0)
        torch.cuda.synchronize()
        assert np.array_equal(state.cpu().numpy().view(np.uint32), want_u), ("update", case, length, stride, base, n)


def test_frame_round_trips_with_corruption(gpu):
    """encode_batch on the device, then decode_host: every frame verifies; one flipped payload byte makes
    its frame the first bad one (Codec::recv stops there, decode's -1) and the frames before it verify."""
    import torch

    import annety_amd

    rng = np.random.default_rng(4242)
    for case in range(12):
        T = int(rng.choice([2, 4, 8]))
        n = int(rng.integers(1, 3000))
        lim = 32000 if T == 2 else 60000
        lens = rng.integers(1, lim, n).astype(np.uint32)
        offs = np.concatenate([[0], np.cumsum(lens.astype(np.int64))[:-1]]).astype(np.uint64)
        host = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
        codec = annety_amd.LengthHeaderCodec(T)
        enc = codec.encode_batch(torch.from_numpy(host).to(gpu), offs, lens)
        stream = enc.frames.cpu().numpy().copy()
        r = codec.decode_host(stream)
        assert r.rt == 0 and r.consumed == stream.size and r.ok.all() and r.ok.size == n, (case, T, n)
        assert np.array_equal(r.payload_len, lens)
        bad = int(rng.integers(0, n))
        pos = int(r.payload_off[bad]) + int(rng.integers(0, int(lens[bad])))
        stream[pos] ^= 1 << int(rng.integers(0, 8))
        r2 = codec.decode_host(stream)
        assert r2.rt == -1 and int(np.flatnonzero(r2.ok == 0)[0]) == bad, (case, T, n, bad)
        assert r2.payload_off.size == bad and r2.consumed == int(r.payload_off[bad]) - T
