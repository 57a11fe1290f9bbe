"""Edges of the length-sorted path's coalesced classes (crc32_kernels.hip var_class_nt: G = 32 for >= 128 lines,
G = 16 for 24..127) and of the per-line small class, against the oracle.

Every payload starts at each of the line offsets where the masks change behaviour (0, 1, 63, 64 = the half
boundary, 124, 125..127 = the init's four bytes spilling into the second line) and ends at each tail position
that matters (1..4 bytes into a line, either side of the half boundary, the full line), with line counts at the
class boundaries (23/24, 127/128) and across the end-aligned first round (every vlead 0..31 for G = 32). Digests
and update registers, in one batch per case so that the lane groups of a wave hold payloads with different
first and last rounds (the two groups of a G = 32 wave, the four of a G = 16 wave, step independently)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

LEADS = [0, 1, 63, 64, 124, 125, 126, 127]
TAILS = [1, 2, 3, 4, 63, 64, 65, 127, 128]


@pytest.fixture
def sorted_path(gpu):
    import annety_amd

    prev = annety_amd.set_var_path("sorted")
    yield gpu
    annety_amd.set_var_path(prev)


def _layout(line_counts, rng):
    """Payloads (lead, lines, tail) from the edge lists, placed at random 128-byte lines of one buffer."""
    offs, lens = [], []
    pos = 0
    for nl in line_counts:
        for lead in LEADS:
            for tail in TAILS:
                if nl == 1 and tail <= lead:
                    continue
                ln = (nl - 1) * 128 + tail - lead
                start = pos + lead
                offs.append(start)
                lens.append(ln)
                pos += nl * 128 + 128 * int(rng.integers(0, 3))
    perm = rng.permutation(len(offs))
    return np.asarray(offs, dtype=np.int64)[perm], np.asarray(lens, dtype=np.int64)[perm], pos + 256


def _check(dev, offs, lens, size, rng, ctx):
    import torch

    import annety_amd

    host = rng.integers(0, 256, size, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    o = torch.from_numpy(offs).to(dev)
    ln = torch.from_numpy(lens.astype(np.int32)).to(dev)
    got = annety_amd.crc32_batch_var(d, o, ln)
    torch.cuda.synchronize()
    assert annety_amd.last_kernels().endswith("crc32_var_sorted_kernel"), annety_amd.last_kernels()
    want = oracle.batch_var_mt(host, offs.astype(np.uint64), lens.astype(np.uint32), threads=8)
    bad = np.nonzero(got.cpu().numpy().view(np.uint32) != want)[0]
    assert bad.size == 0, (ctx, bad.size, offs[bad[:6]].tolist(), lens[bad[:6]].tolist())
    states = rng.integers(0, 2 ** 32, lens.size, dtype=np.uint64).astype(np.uint32)
    st = torch.from_numpy(states.view(np.int32).copy()).to(dev)
    annety_amd.crc32_update_batch_var(st, d, o, ln)
    torch.cuda.synchronize()
    want = oracle.batch_var_mt(host, offs.astype(np.uint64), lens.astype(np.uint32), threads=8, states=states)
    bad = np.nonzero(st.cpu().numpy().view(np.uint32) != want)[0]
    assert bad.size == 0, (ctx + " update", bad.size, offs[bad[:6]].tolist(), lens[bad[:6]].tolist())


def test_class_boundaries(sorted_path):
    rng = np.random.default_rng(41)
    offs, lens, size = _layout([1, 2, 3, 22, 23, 24, 25, 127, 128, 129], rng)
    _check(sorted_path, offs, lens, size, rng, "class boundaries")


def test_every_first_round_offset_g32(sorted_path):
    """Line counts 128..160: the end-aligned first round of a G = 32 payload has every vlead 0..31."""
    rng = np.random.default_rng(42)
    offs, lens, size = _layout(list(range(128, 161)), rng)
    _check(sorted_path, offs, lens, size, rng, "G32 vlead sweep")


def test_every_first_round_offset_g16(sorted_path):
    """Line counts 24..40: every vlead 0..15 of a G = 16 payload."""
    rng = np.random.default_rng(43)
    offs, lens, size = _layout(list(range(24, 41)), rng)
    _check(sorted_path, offs, lens, size, rng, "G16 vlead sweep")
