"""Launch time against batch size for the multi-round fixed kernel (64 KiB payloads) and the one-round
kernel (1 KiB payloads): fit time = a + bytes / rate, so that `a` is the per-launch ramp-up and drain.
GPU box: python3 microbench/launch_scale.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import annety_amd  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream()
sh = int(st.cuda_stream)
buf = torch.randint(0, 256, (8 << 30,), dtype=torch.uint8, device=dev)
out = torch.empty(8 << 20, dtype=torch.int32, device=dev)
annety_amd.set_split(0)


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
for L in (1024, 65536, 4096):
    xs, ys = [], []
    for gib in (0.25, 0.5, 1, 2, 4, 8):
        n = int(gib * (1 << 30)) // L
        ms = timeit(lambda: annety_amd.crc32_batch(buf, n, L, out=out[:n], stream=sh))
        xs.append(n * L)
        ys.append(ms)
        print(f"L {L:6d} {gib:5.2f} GiB: {ms:.4f} ms  {n * L / ms / 8e7:5.1f} %", flush=True)
    b, a = np.polyfit(np.array(xs, dtype=float), np.array(ys), 1)
    print(f"L {L}: fit a = {a * 1e3:.1f} us per launch, rate = {1 / b / 1e6:.0f} GB/s ({1 / b / 8e9 * 100:.1f} %)",
          flush=True)
annety_amd.set_split(-1)
