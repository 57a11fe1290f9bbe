"""Probe (round 6): annety_crc32_batch_var on 2M small frames with fresh offset/length tensors on every call (the
device chooses the path) against the same batch with stable pointers (the host's records choose the arena) and the
sorted path; device time per call from HIP events, host time of the call itself. Run under rocprofv3 --kernel-trace
--stats for the per-kernel split.  Usage: python microbench/auto_fresh_probe.py [calls]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import annety_amd  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
gpu = torch.device("cuda", 0)
rng = np.random.default_rng(21)
n = 2 << 20
lens = rng.integers(16, 1025, n).astype(np.int64)
offs = (np.concatenate([[0], np.cumsum(lens + 8)[:-1]]) + 4).astype(np.int64)
d = torch.randint(0, 256, (int(offs[-1] + lens[-1]) + 260,), dtype=torch.uint8, device=gpu)
fresh = [(torch.from_numpy(offs).to(gpu), torch.from_numpy(lens.astype(np.int32)).to(gpu)) for _ in range(calls)]
out = torch.empty(n, dtype=torch.int32, device=gpu)


def run(label, pairs):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dev, host = [], []
    for o, ln in pairs:
        torch.cuda.synchronize()
        e0.record()
        t0 = time.perf_counter()
        annety_amd.crc32_batch_var(d, o, ln, out=out)
        host.append(time.perf_counter() - t0)
        e1.record()
        torch.cuda.synchronize()
        dev.append(e0.elapsed_time(e1))
    dev, host = np.array(dev[2:]) * 1e3, np.array(host[2:]) * 1e6
    print(f"{label}: device {np.median(dev):.1f} us (min {dev.min():.1f}), host call {np.median(host):.1f} us, "
          f"kernels: {annety_amd.last_kernels()}", flush=True)


run("fresh pointers (device choice)", fresh)
run("stable pointers (records)", [fresh[0]] * calls)
prev = annety_amd.set_var_path("sorted")
run("sorted path", [fresh[0]] * max(4, calls // 4))
annety_amd.set_var_path(prev)
print(annety_amd.var_path_stats(0))
