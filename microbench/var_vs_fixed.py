"""Time the variable-length path against the fixed path on identical aligned batches, and the var
path on Zipf batches split by length class. Run on the GPU box: python3 microbench/var_vs_fixed.py"""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import annety_amd

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream()
sh = int(st.cuda_stream)

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

buf = torch.randint(0, 256, (1 << 30,), dtype=torch.uint8, device=dev)
# warm clocks
t0 = time.time()
while time.time() - t0 < 1.0:
    annety_amd.crc32_batch(buf, 1 << 20, 1024, stream=sh)
torch.cuda.synchronize()
for L in [1024, 4096, 16384, 65536, 1 << 20]:
    n = (1 << 30) // L
    offs = torch.arange(n, dtype=torch.int64, device=dev) * L
    lens = torch.full((n,), L, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    tf = timeit(lambda: annety_amd.crc32_batch(buf, n, L, out=out, stream=sh))
    tv = timeit(lambda: annety_amd.crc32_batch_var(buf, offs, lens, out=out, stream=sh))
    # unaligned by 3 bytes (var path both)
    offs3 = offs[:-1] + 3
    lens3 = lens[:-1]
    out3 = out[:-1]
    tu = timeit(lambda: annety_amd.crc32_batch_var(buf, offs3, lens3, out=out3, stream=sh))
    print(f"L={L:8d} n={n:8d}  fixed {tf:.4f} ms ({(1<<30)/tf/1e6:7.1f} GB/s)  var-aligned {tv:.4f} ms ({(1<<30)/tv/1e6:7.1f})  var-unaligned {tu:.4f} ms ({(1<<30)/tu/1e6:7.1f})", flush=True)
