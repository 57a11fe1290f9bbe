"""Fixed batches of 1 GiB at payload sizes 1 KiB .. 1 MiB (aligned, packed): rate of the fixed-batch
entry (annety_crc32_batch_fixed, split policy auto and never). GPU box: python3 microbench/fixed_size_sweep.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import annety_amd  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream()
sh = int(st.cuda_stream)
buf = torch.randint(0, 256, (1 << 30,), dtype=torch.uint8, device=dev)


def timeit(fn, reps=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


out = torch.empty(1 << 20, dtype=torch.int32, device=dev)
for _ in range(300):
    annety_amd.crc32_batch(buf, 1 << 20, 1024, out=out, stream=sh)
MODES = [(-1, 0), (0, 0), (1, 4096), (1, 8192), (1, 16384)]
for split, seg in MODES:
    annety_amd.set_split(split, seg)
    for kib in (1, 2, 4, 8, 16, 32, 64, 128, 256, 1024):
        L = kib << 10
        n = (1 << 30) // L
        ms = timeit(lambda: annety_amd.crc32_batch(buf, n, L, out=out[:n], stream=sh))
        print(f"split {split:2d} seg {seg:6d}  {kib:5d} KiB x {n:8d}: {ms:.4f} ms  {n * L / ms / 1e6:6.0f} GB/s  "
              f"{n * L / ms / 8e7:5.1f} %", flush=True)
annety_amd.set_split(-1)
