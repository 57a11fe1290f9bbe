"""A/B of the host frame walk for one LengthHeaderCodec stream (config-3 frames, 1.075 GB): walked whole
(annety_crc_set_walk_segment(2^40), the round-3-early product) against segmented speculative walks
(default 64 MiB segments), through decode_host = annety_lhc_verify_host, pageable and pinned, alternating.
Usage (GPU box, repo root): python profiles/r03/walk_ab.py"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import annety_amd  # noqa: E402
from bench import zipf_batch  # noqa: E402

lens, offs = zipf_batch(0x5EED)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(1)
data = torch.randint(0, 256, (int(offs[-1] + lens[-1]),), dtype=torch.uint8, device=dev, generator=g)
codec = annety_amd.LengthHeaderCodec(4)
stream = codec.encode_batch(data, offs.astype(np.uint64), lens.astype(np.uint32)).frames.cpu().numpy()
pin = annety_amd.PinnedHostBuffer(stream.size)
pin.array[:] = stream
payload = float(lens.astype(np.int64).sum())
print(f"stream {stream.size} B, {len(lens)} frames", flush=True)


def rate(buf, reps=5):
    r = codec.decode_host(buf)  # warm
    assert r.ok.all() and r.rt == 0 and r.consumed == stream.size and r.ok.size == len(lens)
    t0 = time.perf_counter()
    for _ in range(reps):
        codec.decode_host(buf)
    return payload / ((time.perf_counter() - t0) / reps) / 2 ** 30


for rnd in range(3):
    for seg, name in ((1 << 40, "whole"), (0, "segmented")):
        annety_amd.set_walk_segment(seg)
        print(f"round {rnd} {name:10s} pageable {rate(stream):6.2f} GiB/s  pinned {rate(pin.array):6.2f} GiB/s",
              flush=True)
annety_amd.set_walk_segment(0)
