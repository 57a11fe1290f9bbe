"""The coalesced nontemporal kernels and their fallbacks, shape by shape.

`crc32_onekib_nt_kernel` takes contiguous 1 KiB payloads (stride 1024) when the count is a multiple of 8,
`crc32_fixed32_nt_kernel` G = 32 batches (length a multiple of 4 KiB) when the count is even and the stride
a multiple of 16; every other shape stays on the per-line-load kernels. Each case runs on both sides of
those conditions, with the grid smaller and larger than the chip (tails of the wave-task loop), against the
oracle. The arena line pass's 16-task S bursts end on partial bursts of every length (arena sizes in
superblocks 1..40 around the grid's wave count)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [8, 16, 8 * 256, 8 * 4096 + 8, 7, 9, 8 * 4096 + 3])
def test_onekib_nt_and_fallback(gpu, n):
    import torch

    import annety_amd

    rng = np.random.default_rng(n)
    host = rng.integers(0, 256, n * 1024, dtype=np.uint8)
    d = torch.from_numpy(host).to(gpu)
    got = annety_amd.crc32_batch(d, n, 1024, 1024)
    torch.cuda.synchronize()
    want = oracle.batch_fixed_mt(host, n, 1024, 1024, threads=8)
    assert np.array_equal(got.cpu().numpy().view(np.uint32), want)


@pytest.mark.parametrize("length,stride,n", [(4096, 4096, 2), (4096, 4096, 3), (8192, 8192 + 16, 64),
                                             (65536, 65536, 130), (65536, 65536 + 48, 129), (12288, 12288, 1000),
                                             (4096, 4096, 20000)])
def test_fixed32_nt_and_fallback(gpu, length, stride, n):
    import torch

    import annety_amd

    rng = np.random.default_rng(length + n)
    host = rng.integers(0, 256, (n - 1) * stride + length, dtype=np.uint8)
    d = torch.from_numpy(host).to(gpu)
    got = annety_amd.crc32_batch(d, n, length, stride)
    torch.cuda.synchronize()
    want = oracle.batch_fixed_mt(host, n, length, stride, threads=8)
    assert np.array_equal(got.cpu().numpy().view(np.uint32), want)
    # crc32_update on the same shape keeps the per-line-load kernel (RAW): registers chained on top
    st0 = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    state = torch.from_numpy(st0.view(np.int32).copy()).to(gpu)
    annety_amd.crc32_update_batch(state, d, n, length, stride)
    offs = (np.arange(n, dtype=np.uint64) * stride).astype(np.uint64)
    want_u = oracle.batch_var_mt(host, offs, np.full(n, length, np.uint32), threads=8, states=st0)
    torch.cuda.synchronize()
    assert np.array_equal(state.cpu().numpy().view(np.uint32), want_u)


def test_arena_partial_bursts(gpu):
    import torch

    import annety_amd

    rng = np.random.default_rng(5)
    for nsb in list(range(1, 41)) + [2047, 2048, 2049, 4100]:
        nbytes = nsb * 8192 + int(rng.integers(0, 8192))
        host = rng.integers(0, 256, nbytes, dtype=np.uint8)
        # zipf draws reach 1e17 and more: clip before scaling, or 64 * z wraps negative
        z = np.minimum(rng.zipf(1.3, nbytes // 500 + 1), 1 << 20)
        lens = np.minimum(20000, 64 * z + rng.integers(0, 64, nbytes // 500 + 1))
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
        keep = offs + lens <= nbytes
        offs, lens = offs[keep].astype(np.uint64), lens[keep].astype(np.uint32)
        d = torch.from_numpy(host).to(gpu)
        got = annety_amd.crc32_batch_var(d, torch.from_numpy(offs.view(np.int64)).to(gpu),
                                         torch.from_numpy(lens.view(np.int32)).to(gpu), arena=True)
        torch.cuda.synchronize()
        want = oracle.batch_var_mt(host, offs, lens, threads=8)
        assert np.array_equal(got.cpu().numpy().view(np.uint32), want), nsb
