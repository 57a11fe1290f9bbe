#!/usr/bin/env python3
"""Headline benchmark: device-resident CRC-32 (annety's "Crc32c") over 1M x 1 KiB payloads per GPU.

BASELINE.json metric: "CRC-32C GiB/s device-resident (1M x 1KiB) @1/2/4/8 MI355X; % HBM roofline".
A step = one batch launch over the GPU's payloads already resident in HBM. The default workload is
BASELINE config 1 (1M x 1 KiB per GPU); --config 2 / 3 run the other single-GPU configs (4K x 4 MiB,
Zipf-mixed lengths) as secondary lines. N GPUs = N ranks (torch.distributed.run), each with its own
shard of the same size (weak scaling, no data-path collective: payloads are independent). After the
timed region the per-shard digests are gathered to rank 0 once over RCCL (gather_ms, not in `value`).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C] [--e2e] [--no-cpu]
Prints ONE JSON line on rank 0 (contract: DESIGN.md §4).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CRC-32C GiB/s device-resident (1M×1KiB) @1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md (8.0 TB/s)
PMC_FILE = os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--prewarm-s", type=float, default=1.0,
                   help="untimed seconds of launches before warmup (the GPU ramps its clocks on sustained load)")
    p.add_argument("--config", type=int, default=1, choices=[1, 2, 3],
                   help="BASELINE config: 1 = 1M x 1 KiB (headline), 2 = 4K x 4 MiB, 3 = Zipf 64 B-64 KiB (~1 GiB)")
    p.add_argument("--var-path", choices=["arena", "sorted"], default="arena",
                   help="config 3: arena = one pass over the packed arena + per-payload stitch (annety_crc32_batch_var_arena); "
                        "sorted = the general length-bucketed path (annety_crc32_batch_var)")
    p.add_argument("--payloads", type=int, default=None, help="override payloads per GPU (fixed configs)")
    p.add_argument("--len", type=int, default=None, help="override payload bytes (fixed configs)")
    p.add_argument("--e2e", action="store_true",
                   help="also time the host-memory path (pinned staging, H2D -> kernel -> D2H) on the same batch")
    p.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample duration")
    return p.parse_args()


def zipf_batch(seed: int, target: int = 1 << 30):
    """k ~ Zipf(1.1) over ranks 1..1024, L = min(65536, 64k + r), r ~ U{0..63},
    packed back-to-back (unaligned starts), sum just under `target` bytes. Returns (lengths, offsets) int64."""
    rng = np.random.default_rng(seed)
    p = np.arange(1, 1025, dtype=np.float64) ** -1.1
    p /= p.sum()
    lens, total = [], 0
    while total < target:
        k = rng.choice(1024, size=65536, p=p) + 1
        ln = np.minimum(65536, 64 * k + rng.integers(0, 64, 65536))
        lens.append(ln)
        total += int(ln.sum())
    lens = np.concatenate(lens)
    lens = lens[: int(np.searchsorted(np.cumsum(lens), target))].astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    return lens, offs


class Workload:
    """One batch resident on the device plus everything the report needs about it."""

    def __init__(self, args, dev, rank):
        import torch

        self.torch = torch
        self.dev = dev
        gen = torch.Generator(device=dev)
        gen.manual_seed(0xC0FFEE + 7919 * rank + args.config)
        self.config = args.config
        if args.config in (1, 2):
            n = args.payloads or (1 << 20 if args.config == 1 else 4096)
            L = args.len or (1024 if args.config == 1 else 4 << 20)
            self.n, self.L = n, L
            self.data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=gen)
            self.payload_bytes = n * L
            self.algo_bytes = n * L + 4 * n  # payload reads + digest writes per launch
            self.offsets = self.lengths = None
            self.kernel = ("crc32_oneround_kernel<8>" if L == 1024 else "crc32_fixed_kernel") + \
                " (annety_amd/csrc/crc32_kernels.hip)"
            self.desc = (f"BASELINE config {args.config}: {n} x {L} B payloads contiguous in HBM per GPU, "
                         "one batch launch per step")
        else:
            lens, offs = zipf_batch(0x5EED + rank)
            total = int(lens.sum())
            self.n, self.L = len(lens), None
            self.data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=gen)
            self.offsets = torch.from_numpy(offs).to(dev)
            self.lengths = torch.from_numpy(lens.astype(np.int32)).to(dev)
            self.payload_bytes = total
            self.algo_bytes = total + 4 * self.n + 12 * self.n  # + offset/length metadata reads
            self.arena = args.var_path == "arena"
            self.kernel = ("crc32_arena_lines_kernel + crc32_arena_stitch_kernel (annety_amd/csrc/crc32_arena.hip)"
                           if self.arena else
                           "crc32_bucket_hist/scan/scatter + crc32_var_kernel<32/8/2> (annety_amd/csrc/crc32_kernels.hip)")
            self.desc = (f"BASELINE config 3: {self.n} payloads, Zipf(1.1) lengths 64 B-64 KiB packed unaligned, "
                         f"{total / 2**30:.3f} GiB per GPU")
        self.out = torch.empty(self.n, dtype=torch.int32, device=dev)

    def launch(self, stream_handle):
        import annety_amd

        if self.config in (1, 2):
            annety_amd.crc32_batch(self.data, self.n, self.L, out=self.out, stream=stream_handle)
        else:
            annety_amd.crc32_batch_var(self.data, self.offsets, self.lengths, out=self.out, stream=stream_handle,
                                       arena=True if self.arena else None)

    def host_sample(self, max_bytes=4 << 20):
        """(host bytes, offsets, lengths) of a bounded prefix of the batch, for the oracle legs."""
        if self.config in (1, 2):
            ns = max(1, min(self.n, max_bytes // self.L))
            h = self.data[: ns * self.L].cpu().numpy()
            return h, np.arange(ns, dtype=np.uint64) * self.L, np.full(ns, self.L, dtype=np.uint32)
        offs = self.offsets.cpu().numpy()
        lens = self.lengths.cpu().numpy()
        end = np.cumsum(lens)
        ns = max(1, int(np.searchsorted(end, max_bytes)))
        h = self.data[: int(end[ns - 1])].cpu().numpy()
        return h, offs[:ns].astype(np.uint64), lens[:ns].astype(np.uint32)


def cpu_baseline(h: np.ndarray, offs: np.ndarray, lens: np.ndarray, budget_s: float) -> dict:
    """Reference CPU checksum on this host's cores over a bounded sample of the same workload.
    Uses the compiled reference (oracle/_ref, kind "reference") when it travelled with the snapshot
    and the sample is a fixed-length batch, else the C restatement (kind "port")."""
    import concurrent.futures as cf

    import oracle

    threads = max(1, min(16, os.cpu_count() or 1))  # the box's CPU share for one GPU
    n = len(offs)
    L0 = int(lens[0])
    fixed = bool(np.all(lens == L0)) and bool(np.all(offs == np.arange(n, dtype=np.uint64) * L0))
    nbytes = int(lens.sum())
    if fixed and oracle.ref_available():
        lib, kind = oracle.ref_lib(), "reference"
        out = np.zeros(n, dtype=np.uint32)

        def run(th):
            lib.ref_crc32_batch_fixed_mt(h.ctypes.data, n, L0, L0, out.ctypes.data, th)
    elif fixed:
        kind = "port"

        def run(th):
            oracle.batch_fixed_mt(h, n, L0, threads=th)
    else:
        kind = "port"
        parts = np.array_split(np.arange(n), threads)

        def run(th):
            if th == 1:
                oracle.batch_var(h, offs, lens)
            else:  # ctypes releases the GIL: one oracle call per thread over its share of payloads
                with cf.ThreadPoolExecutor(th) as ex:
                    list(ex.map(lambda ix: oracle.batch_var(h, offs[ix], lens[ix]), parts))

    def rate(th, budget):
        reps, t0 = 0, time.perf_counter()
        while True:
            run(th)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= budget:
                return reps * nbytes / dt / 2 ** 30, reps

    st_rate, st_reps = rate(1, budget_s * 0.3)
    mt_rate, mt_reps = rate(threads, budget_s * 0.7)
    return {
        "value": round(mt_rate, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": kind,
        "single_thread_value": round(st_rate, 3),
        "sample": f"{n} payloads / {nbytes / 2**20:.1f} MiB prefix of the GPU workload copied to host, crc32_long "
                  f"per payload, payload-parallel over {threads} threads x {mt_reps} passes (+ 1 thread x {st_reps})",
    }


def pmc_traffic(w: Workload):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary of this workload (FETCH_SIZE x2
    gfx950 correction + WRITE_SIZE), or None if no matching profile is committed."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
        if w.config == 1 and d.get("payloads") == w.n and d.get("len") == w.L:
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def e2e_host_path(w: Workload):
    """Host-memory path: payloads in pageable host memory (as off a socket), staged through the
    engine's pinned ring, H2D -> kernel -> D2H. Fixed-length configs only."""
    import annety_amd

    if w.config not in (1, 2):
        return None
    h = w.data.cpu().numpy()
    warm_n = max(1, min(w.n, (64 << 20) // w.L))
    annety_amd.crc32_batch_host(h[: warm_n * w.L], warm_n, w.L)  # allocate/warm the pinned ring
    reps, t0 = 0, time.perf_counter()
    while reps < 3 or time.perf_counter() - t0 < 2.0:
        d = annety_amd.crc32_batch_host(h, w.n, w.L)
        reps += 1
    dt = (time.perf_counter() - t0) / reps
    w.torch.cuda.synchronize()
    ok = bool(np.array_equal(d, w.out.cpu().numpy().view(np.uint32)))
    return {"value": round(w.payload_bytes / dt / 2 ** 30, 2), "unit": "GiB/s", "ms_per_batch": round(dt * 1e3, 2),
            "bit_exact_vs_device_path": ok,
            "path": "pageable host buffer -> pinned 64 MiB x2 ring -> hipMemcpyAsync H2D -> kernel -> D2H, 2 streams"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import oracle

    w = Workload(args, dev, rank)
    stream = torch.cuda.current_stream(dev)
    sh = int(stream.cuda_stream)

    # correctness gate before timing: bit-exact vs the oracle on a prefix of this rank's batch
    w.launch(sh)
    torch.cuda.synchronize()
    hs, ho, hl = w.host_sample()
    want = oracle.batch_var(hs, ho, hl)
    got = w.out[: len(ho)].cpu().numpy().view(np.uint32)
    if not np.array_equal(got, want):
        raise SystemExit(f"rank {rank}: digests differ from the oracle on the sample")

    t_pw = time.perf_counter()
    while time.perf_counter() - t_pw < args.prewarm_s:
        for _ in range(10):
            w.launch(sh)
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        w.launch(sh)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        w.launch(sh)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # HIP events on the launch stream over the timed region
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # one-shot RCCL gather of per-shard digests to rank 0 (not part of `value`)
    gather_ms = None
    if world > 1:
        from annety_amd import sharded

        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        sharded.gather_digests(w.out, [w.n] * world, dst=0)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3

    if rank == 0:
        total_gib = w.payload_bytes * world * args.steps / 2 ** 30
        achieved = w.algo_bytes / (kern_ms / 1e3) / 1e9
        line = {
            "metric": METRIC if args.config == 1 else METRIC.replace("(1M×1KiB)", f"(config {args.config})"),
            "value": round(total_gib / elapsed, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (torch.randint bytes on device, seeded per rank)",
            "config": {
                "workload": w.desc,
                "payloads_per_gpu": w.n,
                "payload_bytes": w.L if w.L else "zipf",
                "bytes_per_gpu": w.payload_bytes,
                "parallelism": f"shard{world}" if world > 1 else "single",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pmc_traffic(w),
                "kernel": w.kernel,
                "kernel_ms_avg": round(kern_ms, 4),
                "algorithmic_bytes_per_launch": w.algo_bytes,
            },
            "cpu_baseline": None if args.no_cpu else cpu_baseline(hs, ho, hl, args.cpu_seconds),
        }
        if gather_ms is not None:
            line["gather_ms"] = round(gather_ms, 3)
        if args.e2e:
            line["e2e_host_path"] = e2e_host_path(w)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
