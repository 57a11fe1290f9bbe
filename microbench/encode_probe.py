#!/usr/bin/env python3
"""Stage costs of the fused LengthHeaderCodec encode (crc32_frames.hip lhc_encode_fused_kernel) on bench.py's frames
workload (2M payloads of 16 B - 1 KiB, or 408 B with ENC_FRAMES=chat, or 256K of 4000 B with ENC_FRAMES=big), with the A/B build of the library
(python -m annety_amd.build --ab -> microbench/libannety_crc_ab.so, loaded through ANNETY_CRC_LIB):
  ANNETY_CRC_ENC_PROBE: 0 = the product kernel, 1 = no copy stores, 2 = no CRC, 3 = neither (wrong frames)
Per setting: microseconds per annety_lhc_encode_batch (HIP events over 200 calls, median of 5 groups), in a child
process each, alternating twice. ENC_ALIGNED=1 puts each payload at its frame's payload offset in the source, so
that every store is 16-byte aligned. Usage: python microbench/encode_probe.py [probes...] (default: 0 1 2 3).
ENC_FRAMES=long / longmix: the long-frame path (16 x 64 MiB; 256 x 1 MiB among 200K short); ENC_CALLS = calls per
group; ENC_LIB = another build of the library (e.g. the one before a change)."""
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
    from annety_amd import _lib

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0xF4A3E5)
    n = 2 << 20
    kind = os.environ.get("ENC_FRAMES", "mixed")
    if kind == "big":  # 256K frames of 4000 B (about the same bytes)
        n = 256 << 10
        lens = np.full(n, 4000, dtype=np.int64)
    elif kind == "long":  # 16 frames of 64 MiB (the long-frame path, crc32_kernels.h EncLong)
        n = 16
        lens = np.full(n, 64 << 20, dtype=np.int64)
    elif kind == "longmix":  # 256 frames of 1 MiB among 200K of 16 B - 4 KiB
        lens = np.concatenate([rng.integers(16, 4097, 200000), np.full(256, 1 << 20)])
        lens = rng.permutation(lens).astype(np.int64)
        n = lens.size
    else:
        lens = np.full(n, 408, dtype=np.int64) if kind == "chat" else rng.integers(16, 1025, n)
    src_off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    frame_off = np.concatenate([[0], np.cumsum(lens + 8)[:-1]]).astype(np.int64)
    src_bytes = int(lens.sum())
    if os.environ.get("ENC_ALIGNED"):  # each payload at its frame's payload offset: every 16-byte store aligned
        src_off = frame_off + 4
        src_bytes = int((lens + 8).sum())
    g = torch.Generator(device=dev)
    g.manual_seed(4242)
    src = torch.randint(0, 256, (src_bytes,), dtype=torch.uint8, device=dev, generator=g)
    out = torch.empty(int((lens + 8).sum()), dtype=torch.uint8, device=dev)
    d_src_off = torch.from_numpy(src_off).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    d_foff = torch.from_numpy(frame_off).to(dev)
    lib = _lib.get()
    s = torch.cuda.current_stream().cuda_stream

    def call():
        st = lib.annety_lhc_encode_batch(src.data_ptr(), d_src_off.data_ptr(), d_len.data_ptr(), n, 4, 1 << 30,
                                         out.data_ptr(), d_foff.data_ptr(), s)
        if st:
            _lib.check(st, "annety_lhc_encode_batch")

    calls = int(os.environ.get("ENC_CALLS", "200"))
    for _ in range(min(20, calls)):
        call()
    torch.cuda.synchronize()
    per = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(calls):
            call()
        e1.record()
        torch.cuda.synchronize()
        per.append(e0.elapsed_time(e1) / calls * 1e3)
    print(json.dumps({"us": sorted(per)[2], "kernels": annety_amd.last_kernels()}))


def main():
    if os.environ.get("ENC_PROBE_CHILD"):
        return child()
    settings = sys.argv[1:] or ["0", "1", "2", "3"]
    lib = os.environ.get("ENC_LIB") or os.path.join(ROOT, "microbench", "libannety_crc_ab.so")
    for rep in range(2):
        for pr in settings:
            env = dict(os.environ, ENC_PROBE_CHILD="1", ANNETY_CRC_LIB=lib, ANNETY_CRC_ENC_PROBE=pr)
            r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, capture_output=True, text=True,
                               timeout=300)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            res = json.loads(line[-1]) if line else {"error": r.stderr[-500:]}
            print(f"rep {rep} probe {pr}: {res}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
