#!/usr/bin/env python3
"""Stage costs of the length-sorted path on BASELINE config 3, with the A/B build of the library
(python -m annety_amd.build --ab -> microbench/libannety_crc_ab.so, loaded through ANNETY_CRC_LIB). Each setting
runs in a child process (the library reads its switches once):
  ANNETY_CRC_W8_PROBE: 0 = the product kernel, 1 = every step unmasked, 2 = no fold, 6 = no fold on config 1's
  window (wrong digests)
  ANNETY_CRC_STITCH_PROBE (the same number, for the arena path, PROBE_PATH=auto on a dense batch): 1 = descriptors
  and stores only, 2 = + every load, 3 = + the window folds (wrong digests)
Per setting: microseconds per crc32_batch_var call (HIP events over 200 calls, median of 5 groups), alternating
settings twice. Usage: python microbench/sorted_probe.py [probes...] (default: 0 1 2)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child():
    import numpy as np
    import torch

    import annety_amd
    import bench

    dev = torch.device("cuda", 0)
    lens, offs = bench.zipf_batch(0x5EED)
    if os.environ.get("PROBE_BATCH") == "long":  # 256 payloads of 1 MiB and 20k of 4 KiB, 8 KiB gaps
        rng = np.random.default_rng(9)
        lens = rng.permutation(np.concatenate([np.full(256, 1 << 20), np.full(20000, 4096)]))
        offs = np.concatenate([[0], np.cumsum(lens + 8192)[:-1]])
    if os.environ.get("PROBE_BATCH") == "huge":  # 16 payloads of 64 MiB, packed (1 GiB)
        lens = np.full(16, 64 << 20)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    if os.environ.get("PROBE_BATCH") == "small":  # 2M payloads of 16 B - 1 KiB, packed
        rng = np.random.default_rng(7)
        lens = rng.integers(16, 1025, 2 << 20)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
    g = torch.Generator(device=dev)
    g.manual_seed(4242)
    data = torch.randint(0, 256, (int(offs[-1] + lens[-1]),), dtype=torch.uint8, device=dev, generator=g)
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    annety_amd.set_var_path(os.environ.get("PROBE_PATH", "sorted"))  # auto: the arena for a dense batch
    out = torch.empty(len(lens), dtype=torch.int32, device=dev)
    for _ in range(20):
        annety_amd.crc32_batch_var(data, d_off, d_len, out=out)
    torch.cuda.synchronize()
    per = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            annety_amd.crc32_batch_var(data, d_off, d_len, out=out)
        e1.record()
        torch.cuda.synchronize()
        per.append(e0.elapsed_time(e1) / 200 * 1e3)
    print(json.dumps({"us": sorted(per)[2], "kernels": annety_amd.last_kernels()}))


def main():
    if os.environ.get("SORTED_PROBE_CHILD"):
        return child()
    settings = sys.argv[1:] or ["0", "1", "2"]
    lib = os.environ.get("PROBE_LIB") or os.path.join(ROOT, "microbench", "libannety_crc_ab.so")
    for rep in range(2):
        for pr in settings:
            env = dict(os.environ, SORTED_PROBE_CHILD="1", ANNETY_CRC_LIB=lib, ANNETY_CRC_W8_PROBE=pr,
                       ANNETY_CRC_STITCH_PROBE=pr)
            r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True, text=True,
                               timeout=300)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            res = json.loads(line[-1]) if line else {"error": r.stderr[-500:]}
            print(f"rep {rep} probe {pr}: {res}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
