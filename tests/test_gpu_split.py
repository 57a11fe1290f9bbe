"""Long payloads through the segment + combine path (annety_crc_set_split; crc32_split_desc/join).

Each case runs with the split forced on and forced off and must give the reference's digests
(golden fixtures) or the oracle's; the > 4 GiB payload, which only the split path accepts, is checked
through the combine identity over halves digested by the whole-payload kernels.
"""
import os

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def H(x: str) -> int:
    return int(x, 16)


class _split:
    """The split policy (annety_crc_set_split) for the duration of a block; back to auto after."""

    def __init__(self, mode: str):
        self.mode = int(mode) if mode != "" else -1  # "" = auto

    def __enter__(self):
        import annety_amd

        annety_amd.set_split(self.mode)

    def __exit__(self, *a):
        import annety_amd

        annety_amd.set_split(-1)


def _digests(out):
    import torch

    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def test_split_golden_big(golden, gpu):
    import annety_amd
    import torch

    for c in golden("big.json")["cases"]:
        b = torch.from_numpy(oracle.lcg_bytes(c["bytes"], c["seed"])).to(gpu)
        for mode in ("0", "1", ""):
            with _split(mode):
                assert int(_digests(annety_amd.crc32_batch(b, 1, c["bytes"]))[0]) == H(c["crc"]), (c, mode)


@pytest.mark.parametrize("n,length,stride", [
    (3, 2 * 65536 + 5, 2 * 65536 + 8),     # odd length, padded stride: descriptor path, short first segment
    (2, 1 << 20, 1 << 20),                 # packed multiple of the segment: uniform fixed batch
    (5, (1 << 20) + 16, (1 << 20) + 48),   # aligned but not a segment multiple
    (7, 3 * 65536 - 1, 3 * 65536 + 1),     # unaligned stride
    (1, (300 << 20) + 17, (300 << 20) + 17),  # > 256 MiB: 128 KiB segments
])
def test_split_vs_oracle(gpu, n, length, stride):
    import annety_amd
    import torch

    host = oracle.lcg_bytes((n - 1) * stride + length, n * 7919 + length)
    d = torch.from_numpy(host).to(gpu)
    want = oracle.batch_fixed_mt(host, n, length, stride, threads=16)
    for mode in ("1", "0"):
        with _split(mode):
            got = _digests(annety_amd.crc32_batch(d, n, length, stride))
        assert np.array_equal(got, want), mode


def test_split_offset_base(gpu):
    """A misaligned base pointer: every segment descriptor carries its own unaligned address."""
    import annety_amd
    import torch

    n, length = 4, 200001
    host = oracle.lcg_bytes(n * length + 3, 31)
    d = torch.from_numpy(host).to(gpu)
    want = oracle.batch_fixed(host[3:], n, length)
    with _split("1"):
        got = _digests(annety_amd.crc32_batch(d[3:], n, length))
    assert np.array_equal(got, want)


def test_split_over_4gib(gpu):
    """A 5 GiB + 12345 payload (beyond the whole-payload kernels' 32-bit lengths) equals
    combine(crc(first half), crc(second half), |second half|) with each half digested whole."""
    import annety_amd
    import torch

    total = (5 << 30) + 12345
    g = torch.Generator(device=gpu)
    g.manual_seed(5)
    d = torch.randint(0, 256, (total,), dtype=torch.uint8, device=gpu, generator=g)
    half = (5 << 29) + 7
    with _split("0"):
        a = int(_digests(annety_amd.crc32_batch(d, 1, half))[0])
        b = int(_digests(annety_amd.crc32_batch(d[half:], 1, total - half))[0])
    with _split(""):
        full = int(_digests(annety_amd.crc32_batch(d, 1, total))[0])
    assert full == annety_amd.crc32_combine(a, b, total - half)
    del d
    torch.cuda.empty_cache()
