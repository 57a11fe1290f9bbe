"""Config-3 arena calls timed with HIP events, for A/Bs of the one-launch arena kernel's variants
(ANNETY_CRC_FUSED_VAR, ANNETY_CRC_ARENA_FUSED), with microbench/arena_fused.patch applied. Digests are not checked here: the variants other
than 0 return wrong ones. Usage: python microbench/fused_probe.py [calls]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import annety_amd  # noqa: E402
from bench import zipf_batch  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    lens, offs = zipf_batch(0x5EED)
    total = int(offs[-1] + lens[-1])
    dev = torch.device("cuda:0")
    arena = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev)
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    for _ in range(20):
        annety_amd.crc32_batch_var(arena, d_off, d_len, arena=True)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(calls):
        annety_amd.crc32_batch_var(arena, d_off, d_len, arena=True)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / calls
    print(f"fused={os.environ.get('ANNETY_CRC_ARENA_FUSED', '1')} var={os.environ.get('ANNETY_CRC_FUSED_VAR', '0')} "
          f"{ms * 1000:.1f} us per call, {(total + 16 * lens.size) / ms / 1e6:.0f} GB/s")


if __name__ == "__main__":
    main()
