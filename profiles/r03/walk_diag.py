import sys, time
import numpy as np, torch
sys.path.insert(0, ".")
import annety_amd
from bench import zipf_batch
lens, offs = zipf_batch(0x5EED)
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev); g.manual_seed(1)
data = torch.randint(0, 256, (int(offs[-1] + lens[-1]),), dtype=torch.uint8, device=dev, generator=g)
codec = annety_amd.LengthHeaderCodec(4)
stream = codec.encode_batch(data, offs.astype(np.uint64), lens.astype(np.uint32)).frames.cpu().numpy()
payload = float(lens.astype(np.int64).sum())
CAP = len(lens) + 1 if "cap" in sys.argv[2:] else None
def rate(buf, reps=5):
    codec.decode_host(buf, max_frames=CAP)
    t0 = time.perf_counter()
    for _ in range(reps): codec.decode_host(buf, max_frames=CAP)
    return payload / ((time.perf_counter() - t0) / reps) / 2 ** 30
mode = sys.argv[1]
if mode == "pin_alive":
    pin = annety_amd.PinnedHostBuffer(stream.size); pin.array[:] = stream
elif mode == "pin_closed":
    pin = annety_amd.PinnedHostBuffer(stream.size); pin.array[:] = stream; pin.close()
for i in range(4):
    print(mode, i, f"default {rate(stream):.2f}", flush=True)
    annety_amd.set_walk_segment(0)
    print(mode, i, f"explicit0 {rate(stream):.2f}", flush=True)
