"""The sorted path's long class (crc32_var_kernel<32>) against the fixed kernel (crc32_fixed_kernel<32>) on
the same 1 GiB: 32768 payloads of 32 KiB, aligned, then the same payloads shifted by 5 bytes (unaligned),
then Zipf-like lengths 16-64 KiB packed unaligned. Sorted path forced (ANNETY_CRC_VAR_AUTO=0 before the
library loads). rocprof kernel times are the reference; event times here. GPU box: python3 microbench/var_g32_ab.py"""
import os
import sys

os.environ["ANNETY_CRC_VAR_AUTO"] = "0"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import annety_amd  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream()
sh = int(st.cuda_stream)


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


buf = torch.randint(0, 256, ((1 << 30) + 4096,), dtype=torch.uint8, device=dev)
n, L = 32768, 32768
out = torch.empty(n, dtype=torch.int32, device=dev)
for _ in range(300):
    annety_amd.crc32_batch(buf, n, L, out=out, stream=sh)  # clocks up
ms = timeit(lambda: annety_amd.crc32_batch(buf, n, L, out=out, stream=sh))
print(f"fixed G32 aligned     {ms:.4f} ms  {n * L / ms / 1e6:.0f} GB/s", flush=True)
for shift in (0, 5):
    offs = torch.from_numpy((np.arange(n, dtype=np.int64) * L + shift)).to(dev)
    lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    ms = timeit(lambda: annety_amd.crc32_batch_var(buf, offs, lens, out=out, stream=sh))
    print(f"var sorted shift {shift}    {ms:.4f} ms  {n * L / ms / 1e6:.0f} GB/s", flush=True)
rng = np.random.default_rng(1)
ln = rng.integers(16384, 65536, 1 << 20)
ln = ln[np.cumsum(ln) < (1 << 30) - 65536]
of = np.concatenate([[3], 3 + np.cumsum(ln)[:-1]])
offs = torch.from_numpy(of.astype(np.int64)).to(dev)
lens = torch.from_numpy(ln.astype(np.int32)).to(dev)
out2 = torch.empty(len(ln), dtype=torch.int32, device=dev)
ms = timeit(lambda: annety_amd.crc32_batch_var(buf, offs, lens, out=out2, stream=sh))
print(f"var sorted 16-64 KiB  {ms:.4f} ms  {int(ln.sum()) / ms / 1e6:.0f} GB/s ({len(ln)} payloads)", flush=True)
