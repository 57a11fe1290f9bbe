"""Whole payloads against 4 KiB end-aligned segments + combine, for 32 KiB - 1 MiB payloads at 0.5 - 4 GiB per
batch (packed, aligned): where does splitting pay? GPU box: python3 microbench/split_policy_sweep.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import annety_amd  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream()
sh = int(st.cuda_stream)
buf = torch.randint(0, 256, (4 << 30,), dtype=torch.uint8, device=dev)
out = torch.empty(1 << 20, dtype=torch.int32, device=dev)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for _ in range(200):
    annety_amd.crc32_batch(buf, 1 << 20, 1024, out=out, stream=sh)
for kib in (16, 32, 64, 256, 1024):
    for gib in (0.5, 1, 2, 4):
        L = kib << 10
        n = int(gib * (1 << 30)) // L
        res = []
        for mode, seg in ((0, 0), (1, 4096), (1, 8192)):
            annety_amd.set_split(mode, seg)
            ms = timeit(lambda: annety_amd.crc32_batch(buf, n, L, out=out[:n], stream=sh))
            res.append(f"{n * L / ms / 8e7:5.1f}%")
        print(f"{kib:5d} KiB x {n:7d} ({gib} GiB): whole {res[0]}  seg4K {res[1]}  seg8K {res[2]}", flush=True)
annety_amd.set_split(-1)
