"""Device groups (annety_crc_group_*: single process, RCCL communicator from ncclCommInitAll) on the
GPU box's one device: the sharded device-resident batch with the chunked digest gather to the root,
and the host batch staged over the group's PCIe links - bit-exact against the oracle. (A one-device
group still builds the communicator and runs the root's send/recv schedule; the 8-device gather is
exercised by the driver's multi-GPU run of bench.py.)"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def test_group_device_shards(gpu):
    import torch

    from annety_amd import sharded

    n, L = 20000, 1024
    host = oracle.lcg_bytes(n * L, 77)
    want = oracle.batch_fixed_mt(host, n, L, threads=8)
    with sharded.DeviceGroup([0]) as g:
        assert sharded.shard_plan(n, 1) == [(0, n)]
        for chunks in (1, 3, 8):
            out = g.batch_fixed([torch.from_numpy(host).to(gpu)], L, chunks=chunks)
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy().view(np.uint32), want), chunks
        # odd shape (general kernel) through the group
        L2, n2 = 1000, 3000
        out = g.batch_fixed([torch.from_numpy(host[: n2 * 1003]).to(gpu)], L2, stride=1003, chunks=4)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), oracle.batch_fixed(host, n2, L2, 1003))


def test_group_host_batch(gpu):
    from annety_amd import sharded

    n, L = 50000, 1024
    host = oracle.lcg_bytes(n * L, 78)
    with sharded.DeviceGroup([0]) as g:
        got = g.batch_fixed_host(host, n, L)
    assert np.array_equal(got, oracle.batch_fixed_mt(host, n, L, threads=8))
