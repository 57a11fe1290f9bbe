#!/usr/bin/env python3
"""Headline benchmark: device-resident CRC-32 (annety's "Crc32c") over 1M x 1 KiB payloads per GPU.

BASELINE.json metric: "CRC-32C GiB/s device-resident (1M x 1KiB) @1/2/4/8 MI355X; % HBM roofline".
A step = one batch launch over the GPU's 1M x 1 KiB payloads already resident in HBM (BASELINE
config 1). N GPUs = N ranks (torch.distributed.run), each with its own 1M-payload shard (weak scaling,
no data-path collective: payloads are independent). After the timed region the per-shard digests are
gathered to rank 0 once over RCCL (reported as gather_ms, not part of `value`).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu] [--payloads P] [--len L]
Prints ONE JSON line on rank 0 (contract in the task statement / DESIGN.md §4).
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
    p.add_argument("--payloads", type=int, default=1 << 20, help="payloads per GPU (config 1: 1M)")
    p.add_argument("--len", type=int, default=1024, help="payload bytes (config 1: 1 KiB)")
    p.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample duration")
    return p.parse_args()


def cpu_baseline(host_sample: np.ndarray, n: int, length: int, budget_s: float) -> dict:
    """Reference CPU checksum on this host's cores over a bounded sample of the same workload.
    Uses the compiled reference (oracle/_ref, kind "reference") when it travelled with the snapshot,
    else the C restatement (kind "port")."""
    import oracle

    threads = max(1, min(16, os.cpu_count() or 1))  # the box's CPU share for one GPU
    if oracle.ref_available():
        lib = oracle.ref_lib()
        kind = "reference"
        out = np.zeros(n, dtype=np.uint32)

        def run(th):
            lib.ref_crc32_batch_fixed_mt(host_sample.ctypes.data, n, length, length, out.ctypes.data, th)
    else:
        kind = "port"

        def run(th):
            oracle.batch_fixed_mt(host_sample, n, length, threads=th)

    def rate(th, budget):
        reps, t0 = 0, time.perf_counter()
        while True:
            run(th)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= budget:
                return reps * n * length / dt / 2 ** 30, reps

    st_rate, st_reps = rate(1, budget_s * 0.3)
    mt_rate, mt_reps = rate(threads, budget_s * 0.7)
    return {
        "value": round(mt_rate, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": kind,
        "single_thread_value": round(st_rate, 3),
        "sample": f"{n} x {length} B payloads ({n * length / 2**20:.0f} MiB) copied from the GPU workload, "
                  f"crc32_long per payload, payload-parallel over {threads} threads x {mt_reps} passes "
                  f"(+ 1 thread x {st_reps} passes)",
    }


def pmc_traffic(n: int, length: int):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary of this workload (FETCH_SIZE x2
    gfx950 correction + WRITE_SIZE), or None if no matching profile is committed."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
        if d.get("payloads") == n and d.get("len") == length:
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


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

    import annety_amd

    n, L = args.payloads, args.len
    gen = torch.Generator(device=dev)
    gen.manual_seed(0xC0FFEE + rank)
    data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=gen)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    stream_handle = int(stream.cuda_stream)

    # correctness gate on a sample before timing (bit-exact vs the oracle)
    annety_amd.crc32_batch(data, n, L, out=out)
    torch.cuda.synchronize()
    import oracle

    ns = min(n, 4096)
    host_sample = data[: ns * L].cpu().numpy()
    want = oracle.batch_fixed_mt(host_sample, ns, L, threads=8)
    got = out[:ns].cpu().numpy().view(np.uint32)
    if not np.array_equal(got, want):
        raise SystemExit(f"rank {rank}: digests differ from the oracle on the sample")

    t_pw = time.perf_counter()
    while time.perf_counter() - t_pw < args.prewarm_s:
        for _ in range(20):
            annety_amd.crc32_batch(data, n, L, out=out, stream=stream_handle)
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        annety_amd.crc32_batch(data, n, L, out=out, stream=stream_handle)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        annety_amd.crc32_batch(data, n, L, out=out, stream=stream_handle)
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
        gathered = [torch.empty_like(out) for _ in range(world)] if rank == 0 else None
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        dist.gather(out, gathered, dst=0)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3

    if rank == 0:
        payload_bytes = n * L
        total_gib = payload_bytes * world * args.steps / 2 ** 30
        value = total_gib / elapsed
        avg_kern_s = kern_ms / 1e3
        algo_bytes = payload_bytes + 4 * n  # payload reads + digest writes per launch
        achieved = algo_bytes / avg_kern_s / 1e9
        cpu = None
        if not args.no_cpu:
            cpu = cpu_baseline(host_sample, ns, L, args.cpu_seconds)
        line = {
            "metric": METRIC,
            "value": round(value, 2),
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
                "workload": "BASELINE config 1: 1M x 1 KiB payloads contiguous in HBM per GPU, one batch launch per step",
                "payloads_per_gpu": n,
                "payload_bytes": L,
                "parallelism": f"shard{world}" if world > 1 else "single",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pmc_traffic(n, L),
                "kernel": "crc32_oneround_kernel<8> (annety_amd/csrc/crc32_kernels.hip)",
                "kernel_ms_avg": round(avg_kern_s * 1e3, 4),
                "algorithmic_bytes_per_launch": algo_bytes,
            },
            "cpu_baseline": cpu,
        }
        if gather_ms is not None:
            line["gather_ms"] = round(gather_ms, 3)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
