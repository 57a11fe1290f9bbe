"""Line-stream path stage costs (crc32_stream.hip PROBE variants, ANNETY_CRC_STREAM_PROBE) on the BASELINE
config-3 batch, beside the sorted and arena paths on the same box: time per call from HIP events after a
1 s prewarm, one process per variant (the library reads the variable once; ANNETY_CRC_STITCH_* knobs pass
through to every child). BATCH=small / long select other batches. Probe variants 1-7 return wrong
digests by design; the product variants (0, 8) and the other paths are checked against the oracle."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(which: str, reps: int = int(os.environ.get("REPS", "50"))):
    probe = int(which) if which.isdigit() else -1
    sys.path.insert(0, ROOT)
    import numpy as np
    import torch

    import annety_amd
    import bench
    import oracle

    dev = torch.device("cuda", 0)
    if os.environ.get("BATCH") == "small":  # 2M frames of 16 B - 1 KiB, packed, in shuffled order
        rng = np.random.default_rng(5)
        lens = rng.integers(16, 1025, 2 << 20).astype(np.int64)
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
        perm = rng.permutation(lens.size)
        lens, offs = lens[perm], starts[perm]
    elif os.environ.get("BATCH") == "long":  # 3000 payloads of 8 KiB - 1 MiB (up to 127 whole superblocks)
        rng = np.random.default_rng(6)
        lens = rng.integers(8 << 10, (1 << 20) + 1, 3000).astype(np.int64)
        starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
        perm = rng.permutation(lens.size)
        lens, offs = lens[perm], starts[perm]
    else:
        lens, offs = bench.zipf_batch(0x5EED)
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    data = torch.randint(0, 256, (int(lens.sum()),), dtype=torch.uint8, device=dev, generator=g)
    o = torch.from_numpy(offs).to(dev)
    ln = torch.from_numpy(lens.astype(np.int32)).to(dev)
    out = torch.zeros(lens.size, dtype=torch.int32, device=dev)
    annety_amd.set_var_path({"s": "sorted", "u": "auto"}.get(which, "stream"))
    # the C entry point directly (the Python wrapper's checks would leave the GPU idle between calls)
    from annety_amd import _lib

    if which == "a":  # the arena entry point over the packed batch
        fn = _lib.get().annety_crc32_batch_var_arena
        args = (data.data_ptr(), data.numel(), o.data_ptr(), ln.data_ptr(), lens.size, out.data_ptr(),
                torch.cuda.current_stream().cuda_stream)
    else:
        fn = _lib.get().annety_crc32_batch_var
        args = (data.data_ptr(), o.data_ptr(), ln.data_ptr(), lens.size, out.data_ptr(),
                torch.cuda.current_stream().cuda_stream)
    for _ in range(5):
        assert fn(*args) == 0
    torch.cuda.synchronize()
    ok = "-"
    if probe in (0, 8) or probe < 0:
        want = oracle.batch_var_mt(data.cpu().numpy(), offs, lens, 16)
        ok = bool(np.array_equal(out.cpu().numpy().view(np.uint32), want))
    import time

    t_end = time.time() + float(os.environ.get("PREWARM_S", "1.0"))  # clocks up (the bench's --prewarm-s)
    while time.time() < t_end:
        for _ in range(20):
            fn(*args)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn(*args)
    e1.record()
    torch.cuda.synchronize()
    print(f"{which}: {e0.elapsed_time(e1) / reps * 1000:.1f} us per call, digests ok: {ok}",
          flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        child(sys.argv[1])
    else:
        # digits: stream-kernel probe variants; s = sorted path, a = arena path, u = automatic choice
        for w in os.environ.get("PROBES", "0 s a 0 s a 1 2 4 3 7").split():
            env = dict(os.environ, ANNETY_CRC_STREAM_PROBE=w if w.isdigit() else "0")
            subprocess.run([sys.executable, __file__, w], env=env, check=True, timeout=120)
