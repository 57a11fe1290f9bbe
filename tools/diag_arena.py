"""Diagnostic for the arena stitch: replays test_arena_unit_boundaries' first batch several times and
prints every mismatching payload with its geometry and the lane/block that computed it."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import annety_amd
import oracle

dev = torch.device("cuda", 0)
rng = np.random.default_rng(11)
nbytes = 4 << 20
host = oracle.lcg_bytes(nbytes, 99)
d = torch.from_numpy(host).to(dev)
print("base mod 8192:", d.data_ptr() % 8192, flush=True)
n, max_len = 3000, 300
lens = rng.integers(0, max_len + 1, n)
offs = rng.integers(0, nbytes - max_len, n).astype(np.int64)
want = oracle.batch_var_mt(host, offs, lens, 8)
d_off = torch.from_numpy(offs).to(dev)
d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
blk = 512
blocks = min(256, (n + blk - 1) // blk * 2)
for rep in range(int(os.environ.get("REPS", "4"))):
    out = annety_amd.crc32_batch_var(d, d_off, d_len, arena=True)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != want)[0]
    print(f"rep {rep}: {bad.size} bad", flush=True)
    for p in bad[:3]:
        a = d.data_ptr() + int(offs[p]); L = int(lens[p]); e = a + L - 1
        print(f"  p={p} block={p % blocks} tid={p // blocks} wave={(p // blocks) // 64} off={offs[p]} len={L} "
              f"lead={a & 127} lines={(e >> 7) - (a >> 7) + 1} tailend={(e & 127) + 1} got={got[p]:08x} want={want[p]:08x}")
# same payloads alone
sel = np.arange(1536, 1920)
out = annety_amd.crc32_batch_var(d, d_off[sel], d_len[sel], arena=True)
torch.cuda.synchronize()
print("subset bad:", int((out.cpu().numpy().view(np.uint32) != want[sel]).sum()))
out = annety_amd.crc32_batch_var(d, d_off, d_len)
torch.cuda.synchronize()
print("sorted path bad:", int((out.cpu().numpy().view(np.uint32) != want).sum()))

