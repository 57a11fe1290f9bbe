#!/usr/bin/env python3
"""Headline benchmark: device-resident CRC-32 (annety's "Crc32c") over 1 KiB payloads per GPU.

BASELINE.json metric: "CRC-32C GiB/s device-resident (1M x 1KiB) @1/2/4/8 MI355X; % HBM roofline".
A step = one pass of the hot path over the GPU's batch, already resident in HBM.

  * Default, any N: BASELINE config 1 per GPU, 1M x 1 KiB resident in each GPU's HBM, one batch
    launch per step, weak scaling: the N = 1, 2, 4, 8 lines run the same per-GPU workload, so they are
    points of one curve (`config.workload` is identical at every N). At N > 1 each step's digests also
    travel to rank 0 over RCCL/xGMI (annety_amd.sharded.PipelinedGather; step s's gather overlaps step
    s+1's kernel) and that gather is inside `value`; `value_compute_only` is the same step without it.
  * --strong: the same 1M x 1 KiB TOTAL split N ways (contiguous shards), `"scaling": "strong"`
    (SURVEY.md §8e).
  * --config 4: BASELINE config 4's per-GPU shard, 8M x 1 KiB (8 GiB) per rank, checksummed in chunks
    whose digests are gathered while the next chunk computes.
  * --config 2 / 3 run the other single-GPU configs (4K x 4 MiB; Zipf 64 B-64 KiB packed, arena path)
    as secondary lines.

`python bench.py --gpus N` with N > 1 and no torchrun environment spawns the N ranks itself (one
process per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR=127.0.0.1), before anything touches the GPU;
under torch.distributed.run it uses the launcher's ranks. Prints ONE JSON line on rank 0
(contract: DESIGN.md §4).

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C] [--strong] [--e2e] [--no-cpu]
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CRC-32C GiB/s device-resident (1M×1KiB) @1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md (8.0 TB/s)
# Per-launch HBM bytes from the rocprofv3 PMC passes of this bench's own command (profiles/pmc.sh, FETCH_SIZE x2
# gfx950 correction + WRITE_SIZE), committed per config; reported as `traffic` with the file as its source
# (a PMC pass cannot run inside the timed process). Each summary is stamped with the library's source digest
# (annety_amd.build.source_digest); a summary whose digest is not the current tree's describes other kernels and is
# refused (traffic null, `traffic_refused` says why).
PMC_DIR = "profiles/r06/pmc"
PMC_FILES_VAR = {"sorted": f"{PMC_DIR}/c3s.json"}  # config 3 on another variable path
PMC_FILES_FRAMES = {("mixed", "verify"): f"{PMC_DIR}/fmv.json", ("mixed", "encode"): f"{PMC_DIR}/fme.json",
                    ("chat", "verify"): f"{PMC_DIR}/fcv.json", ("chat", "encode"): f"{PMC_DIR}/fce.json"}
PMC_FILES = {1: f"{PMC_DIR}/c1.json", 3: f"{PMC_DIR}/c3a.json", 2: f"{PMC_DIR}/c2.json", 4: f"{PMC_DIR}/c1.json"}
CPU_SAMPLE_BYTES = 1 << 30  # cpu_baseline sample: up to 1 GiB of the workload, far above the host's caches
# The reference build of oracle/_ref (oracle/Makefile): the reference's Release flags without -march=native.
REF_FLAGS = "g++ -std=c++11 -O2 -DNDEBUG (CMakeLists.txt:24,48 Release flags; -march=native dropped so the .so runs on any host)"


def parse():
    p = argparse.ArgumentParser()
    # (--config is parsed as text for "frames"; numeric configs become ints below)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--prewarm-s", type=float, default=1.0,
                   help="untimed seconds of launches before warmup (the GPU ramps its clocks on sustained load)")
    p.add_argument("--config", default="1", choices=["1", "2", "3", "4", "frames"],
                   help="BASELINE config: 1 = 1M x 1 KiB per GPU (default at every N), 2 = 4K x 4 MiB, "
                        "3 = Zipf 64 B-64 KiB (~1 GiB), 4 = 8M x 1 KiB per GPU (config 4's shard) in chunks; "
                        "frames = annety's own frame regime (secondary line): a device-resident LengthHeaderCodec "
                        "stream (4-byte lengths, checksum on), verified or encoded per step (--frames, --op)")
    p.add_argument("--frames", choices=["mixed", "chat"], default="mixed",
                   help="--config frames: mixed = payloads of 16 B-1 KiB (uniform); chat = 408 B payloads, the "
                        "chat server's frames (examples/asio/chat/server/server.cc:25-27: LengthHeaderCodec(kLengthType32, "
                        "checksum, max 408))")
    p.add_argument("--op", choices=["verify", "encode"], default="verify",
                   help="--config frames: verify = annety_lhc_verify_stream (LengthHeaderCodec::decode's checksum "
                        "check over the received stream, include/codec/LengthHeaderCodec.h:100-136); encode = "
                        "annety_lhc_encode_batch (LengthHeaderCodec::encode, :146-201)")
    p.add_argument("--frames-n", type=int, default=2 << 20, help="--config frames: frames per step (default 2M)")
    p.add_argument("--strong", action="store_true",
                   help="fixed configs: --payloads (default 1M) is the TOTAL over all ranks, split into contiguous "
                        "shards (strong scaling); default is per GPU (weak scaling)")
    p.add_argument("--var-path", choices=["arena", "auto", "sorted"], default="arena",
                   help="config 3: arena = one pass over the packed arena + per-payload stitch (annety_crc32_batch_var_arena); "
                        "auto = annety_crc32_batch_var, which picks the arena path itself from the batch's recorded extent; "
                        "sorted = the length-bucketed path only (ANNETY_CRC_VAR_PATH=sorted)")
    p.add_argument("--chunks", type=int, default=None,
                   help="N>1: chunks per shard for the pipelined gather (default 1 for config 1: step s's gather "
                        "overlaps step s+1's kernel; 2 for config 4, one-rank rehearsal 1/2/4 chunks "
                        "5755-5770/5748/5613-5616 GiB/s, profiles/r02/config4_chunks_overlap.log)")
    p.add_argument("--hw-queues", type=int, default=8,
                   help="N>1: raise GPU_MAX_HW_QUEUES to this (<= 32) so the compute and RCCL streams get queues of "
                        "their own")
    p.add_argument("--taper", type=int, default=0,
                   help="config 4: cut the last chunk into this many halving pieces (only the last piece's gather "
                        "is not hidden behind compute); 0 = equal chunks")
    p.add_argument("--no-overlap-steps", action="store_true",
                   help="config 4: wait for a step's gathers before the next step starts (default: the digests "
                        "alternate between two buffers and step s+1's chunks compute while step s's last gathers "
                        "are in flight; every gather is still inside the timed region)")
    p.add_argument("--gather-buffers", type=int, default=2,
                   help="N>1: digest buffers the steps rotate through; step s+1 computes while step s's gather is in "
                        "flight, and the compute stream waits for step s's gather only before step s+buffers reuses "
                        "its buffer (1 = wait for every step's gather before the next step)")
    p.add_argument("--dist", action="store_true",
                   help="run the N>1 code path (RCCL process group, pipelined digest gather, gather check, max over "
                        "ranks) even at one rank: a one-GPU rehearsal of the multi-GPU run")
    p.add_argument("--reserve-cus", type=int, default=None,
                   help="N>1: CUs left free of the checksum kernels for the overlapped RCCL gather "
                        "(annety_crc_reserve_cus; default 8 when gathering, else 0)")
    p.add_argument("--compute-stream", choices=["default", "own"], default="default",
                   help="launch the checksum kernels on torch's default stream or on a stream of their own")
    p.add_argument("--payloads", type=int, default=None,
                   help="override payloads per GPU (fixed configs; with --strong, the total over all ranks)")
    p.add_argument("--len", type=int, default=None, help="override payload bytes (fixed configs)")
    p.add_argument("--e2e", action="store_true",
                   help="also time the host-memory path (pinned staging, H2D -> kernel -> D2H) on the same batch")
    p.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    p.add_argument("--sample-check", action="store_true",
                   help="check only a 4 MiB prefix of the batch against the oracle before timing (default: every "
                        "digest, 1 GiB at a time)")
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU-baseline sample duration")
    a = p.parse_args()
    a.config = int(a.config) if a.config.isdigit() else a.config
    return a


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn(n: int, argv=None) -> int:
    """Start n ranks of `argv` (default: this script with the same arguments), one per GPU, the way
    torch.distributed.run would, and wait; nothing here touches the GPU. Rank 0's stdout (the JSON line)
    passes through; the exit status is the worst of the ranks'."""
    argv = argv if argv is not None else [os.path.abspath(__file__)] + sys.argv[1:]
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    # fail fast: a rank that dies leaves the others blocked in a collective, so the first non-zero exit
    # terminates the rest (the processes started here, by PID)
    while True:
        rcs = [p.poll() for p in procs]
        if all(rc is not None for rc in rcs):
            return max(rcs, key=lambda c: abs(c))
        if any(rc not in (None, 0) for rc in rcs):
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            deadline = time.time() + 10
            for p in procs:
                try:
                    p.wait(timeout=max(0.1, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return max((p.returncode for p in procs), key=lambda c: abs(c))
        time.sleep(0.2)


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

    def __init__(self, args, dev, rank, world=1):
        import torch

        self.torch = torch
        self.dev = dev
        gen = torch.Generator(device=dev)
        gen.manual_seed(0xC0FFEE + 7919 * rank + (args.config if isinstance(args.config, int) else 5))
        self.config = args.config
        self.arena = False
        if args.config in (1, 2, 4):
            default_n = {1: 1 << 20, 2: 4096, 4: 8 << 20}[args.config]
            n = args.payloads or default_n
            L = args.len or (4 << 20 if args.config == 2 else 1024)
            self.n_total = n * world  # payloads over all ranks
            if args.strong:  # n is the job's total: this rank's contiguous shard of it
                from annety_amd.sharded import shard_range

                self.n_total = n
                lo, hi = shard_range(n, rank, world)
                n = hi - lo
            self.n, self.L = n, L
            self.data = torch.randint(0, 256, (n * L,), dtype=torch.uint8, device=dev, generator=gen)
            self.payload_bytes = n * L
            self.algo_bytes = n * L + 4 * n  # payload reads + digest writes per launch
            self.offsets = self.lengths = None
            # the workload only: identical at every N for a weak-scaling run, so the driver's N = 1..8 lines
            # are one curve (the gather, when there is one, is described in the line's "gather" object)
            if args.strong:
                self.desc = (f"BASELINE config {args.config}, strong scaling: {self.n_total} x {L} B payloads in total, "
                             f"contiguous shards of {self.n_total // world}-{-(-self.n_total // world)} payloads per GPU, "
                             "one batch launch per step")
            elif args.config == 4:
                self.desc = (f"BASELINE config 4 shard: {n} x {L} B payloads contiguous in HBM per GPU "
                             "(64M x 1 KiB at 8 GPUs), checksummed in chunks per step")
            else:
                self.desc = (f"BASELINE config {args.config}: {n} x {L} B payloads contiguous in HBM per GPU, "
                             "one batch launch per step")
        elif args.config == "frames":
            self._init_frames(args, dev, rank, gen)
        else:
            lens, offs = zipf_batch(0x5EED + rank)
            total = int(lens.sum())
            self.n, self.L = len(lens), None
            self.n_total = self.n * world
            self.data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=gen)
            self.offsets = torch.from_numpy(offs).to(dev)
            self.lengths = torch.from_numpy(lens.astype(np.int32)).to(dev)
            self.payload_bytes = total
            self.algo_bytes = total + 4 * self.n + 12 * self.n  # + offset/length metadata reads
            self.arena = args.var_path == "arena"
            self.var_path = args.var_path
            self.desc = (f"BASELINE config 3: {self.n} payloads, Zipf(1.1) lengths 64 B-64 KiB packed unaligned, "
                         f"{total / 2**30:.3f} GiB per GPU, " + {"arena": "arena path", "auto": "automatic path choice",
                                                                  "sorted": "sorted path"}[args.var_path])
        # strong scaling: shards differ by at most one payload; the digest buffer is padded (zeros) to the
        # largest so that every rank's gather moves the same count
        self.n_pad = -(-self.n_total // world) if getattr(args, "strong", False) else self.n
        self.out = torch.zeros(self.n_pad, dtype=torch.int32, device=dev)
        self.kernel = None  # the kernels one step enqueues, as the library reports them (annety_crc_last_kernels)
        from annety_amd import _lib

        self._fixed = _lib.get().annety_crc32_batch_fixed
        self._data_ptr = self.data.data_ptr() if args.config != "frames" else self.src.data_ptr()

    def _init_frames(self, args, dev, rank, gen):
        """--config frames: n payloads (16 B-1 KiB uniform, or all 408 B) packed in a source buffer, and the
        LengthHeaderCodec stream of them (4-byte big-endian length = payload + 4, payload, big-endian CRC),
        built on the device by the library's encoder and checked against the oracle before timing."""
        import torch

        import annety_amd

        torch = self.torch
        rng = np.random.default_rng(0xF4A3E5 + rank)
        n = args.frames_n
        lens = (np.full(n, 408, dtype=np.int64) if args.frames == "chat" else rng.integers(16, 1025, n))
        src_off = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        total = int(lens.sum())
        self.src = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=gen)
        self.codec = annety_amd.LengthHeaderCodec(4, True, 1 << 20)
        enc = self.codec.encode_batch(self.src, src_off.astype(np.uint64), lens.astype(np.uint32))
        torch.cuda.synchronize()
        self.frame_off = enc.frame_off
        self.stream = enc.frames  # the received stream of the verify step; the encode step rewrites a copy
        self.n, self.L = n, None
        self.n_total = n
        self.lens_host, self.src_off_host = lens, src_off
        self.payload_bytes = total
        self.op = args.op
        self.frames_variant = args.frames
        self.d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
        if args.op == "verify":
            self.offsets = torch.from_numpy(enc.frame_off.astype(np.int64) + 4).to(dev)  # payloads in the stream
            self.ok = torch.zeros(n, dtype=torch.uint8, device=dev)
            # payload reads + trailer reads + offset/length reads + verdict and digest writes, per frame
            self.algo_bytes = total + n * (4 + 12 + 1 + 4)
        else:
            self.offsets = torch.from_numpy(src_off).to(dev)  # payloads in the source buffer
            self.d_foff = torch.from_numpy(enc.frame_off.astype(np.int64)).to(dev)
            self.frames_out = torch.empty_like(self.stream)
            # payload reads + frame writes (header + payload + trailer) + src/frame offset and length reads
            self.algo_bytes = 2 * total + n * (8 + 20)
        self.lengths = self.d_len
        kind = "16 B-1 KiB uniform" if args.frames == "mixed" else "408 B (the chat server's MSS)"
        self.desc = (f"annety frames ({args.frames}): {n} LengthHeaderCodec frames (4-byte lengths, checksum), payloads "
                     f"{kind}, {total / 2**30:.3f} GiB of payload, device-resident; one "
                     + ("annety_lhc_verify_stream (CRC of every payload against its trailer)" if args.op == "verify"
                        else "annety_lhc_encode_batch (header, payload copy, CRC trailer)") + " per step")

    def frames_check(self) -> dict:
        """Every frame of the step's output against the oracle: verify - every verdict 1 and every digest the
        oracle's; encode - the whole output stream byte for byte against the stream the reference's framing
        gives (header, payload, big-endian oracle CRC)."""
        import oracle

        torch = self.torch
        t0 = time.perf_counter()
        host = self.src.cpu().numpy()
        want = oracle.batch_var_mt(host, self.src_off_host.astype(np.uint64), self.lens_host.astype(np.uint32),
                                   threads=min(16, os.cpu_count() or 1))
        if self.op == "verify":
            if not bool((self.ok == 1).all()):
                raise SystemExit("frames: a verdict is not 1")
            if not np.array_equal(self.out.cpu().numpy().view(np.uint32), want):
                raise SystemExit("frames: digests differ from the oracle")
        else:
            got = self.frames_out.cpu().numpy()
            exp = np.empty_like(got)
            fo = self.frame_off.astype(np.int64)
            L = self.lens_host
            hdr = (L + 4).astype(np.uint32)
            for k in range(4):
                exp[fo + k] = (hdr >> (8 * (3 - k))) & 0xFF
                exp[fo + 4 + L + k] = (want >> (8 * (3 - k))) & 0xFF
            # payload bytes: one vectorised gather per frame position
            idx = np.repeat(fo + 4 - self.src_off_host, L) + np.arange(int(L.sum()))
            exp[idx] = host
            if not np.array_equal(got, exp):
                raise SystemExit(f"frames: encoded stream differs at byte {int(np.flatnonzero(got != exp)[0])}")
        torch.cuda.synchronize()
        return {"frames": self.n, "against": "oracle (C restatement pinned by tests/golden)",
                "seconds": round(time.perf_counter() - t0, 2)}

    def launch(self, stream_handle, lo: int = 0, hi: int | None = None):
        """Digests of payloads [lo, hi) into self.out[lo:hi] (fixed configs); the whole batch otherwise."""
        import annety_amd
        from annety_amd import _lib

        if self.config == "frames":
            lib = _lib.get()
            if self.op == "verify":
                st = lib.annety_lhc_verify_stream(self.stream.data_ptr(), self.stream.numel(), self.offsets.data_ptr(),
                                                  self.d_len.data_ptr(), self.n, self.ok.data_ptr(),
                                                  self.out.data_ptr(), stream_handle)
                name = "annety_lhc_verify_stream"
            else:
                st = lib.annety_lhc_encode_batch(self.src.data_ptr(), self.offsets.data_ptr(), self.d_len.data_ptr(),
                                                 self.n, 4, 1 << 20, self.frames_out.data_ptr(), self.d_foff.data_ptr(),
                                                 stream_handle)
                name = "annety_lhc_encode_batch"
            if st:
                _lib.check(st, name)
            if self.kernel is None:
                self.kernel = annety_amd.last_kernels()
            return self.out

        if self.config in (1, 2, 4):
            hi = self.n_pad if hi is None else hi
            top = min(hi, self.n)  # the padding past this rank's shard (strong scaling) stays zero
            if top > lo:
                # the C-ABI call itself (annety_amd.crc32_batch's checks done once in __init__): a step is
                # 0.17 ms, and per-call Python checks would eat into the launch rate on a slow host
                st = self._fixed(self._data_ptr + lo * self.L, top - lo, self.L, self.L,
                                 self.out.data_ptr() + 4 * lo, stream_handle)
                if st:
                    _lib.check(st, "annety_crc32_batch_fixed")
                if self.kernel is None:
                    self.kernel = annety_amd.last_kernels()
            return self.out[lo:hi]
        annety_amd.crc32_batch_var(self.data, self.offsets, self.lengths, out=self.out, stream=stream_handle,
                                   arena=True if self.arena else None)
        if self.kernel is None:
            self.kernel = annety_amd.last_kernels()
        return self.out

    def host_sample(self, max_bytes=4 << 20):
        """(host bytes, offsets, lengths) of a bounded prefix of the batch, for the oracle legs."""
        if self.config == "frames":  # the payloads, as the CPU codec would checksum them
            end = np.cumsum(self.lens_host)
            ns = max(1, int(np.searchsorted(end, max_bytes)))
            h = self.src[: int(end[ns - 1])].cpu().numpy()
            return h, self.src_off_host[:ns].astype(np.uint64), self.lens_host[:ns].astype(np.uint32)
        if self.config in (1, 2, 4):
            ns = max(1, min(self.n, max_bytes // self.L))
            h = self.data[: ns * self.L].cpu().numpy()
            return h, np.arange(ns, dtype=np.uint64) * self.L, np.full(ns, self.L, dtype=np.uint32)
        offs = self.offsets.cpu().numpy()
        lens = self.lengths.cpu().numpy()
        end = np.cumsum(lens)
        ns = max(1, int(np.searchsorted(end, max_bytes)))
        h = self.data[: int(end[ns - 1])].cpu().numpy()
        return h, offs[:ns].astype(np.uint64), lens[:ns].astype(np.uint32)


def full_check(w: Workload, threads: int) -> dict:
    """Every digest of the batch against the oracle (C restatement, pinned by tests/golden), 1 GiB of
    payloads at a time so host memory stays bounded (config 2: 16 GiB in 16 pieces)."""
    import oracle

    t0 = time.perf_counter()
    if w.config in (1, 2, 4):
        per = max(1, (1 << 30) // w.L)
        for lo in range(0, w.n, per):
            hi = min(w.n, lo + per)
            h = w.data[lo * w.L:hi * w.L].cpu().numpy()
            got = w.out[lo:hi].cpu().numpy().view(np.uint32)
            want = oracle.batch_fixed_mt(h, hi - lo, w.L, threads=threads)
            if not np.array_equal(got, want):
                raise SystemExit(f"digest of payload {int(np.flatnonzero(got != want)[0]) + lo} differs from the oracle")
    else:
        h = w.data.cpu().numpy()
        want = oracle.batch_var_mt(h, w.offsets.cpu().numpy().astype(np.uint64),
                                   w.lengths.cpu().numpy().astype(np.uint32), threads=threads)
        if not np.array_equal(w.out.cpu().numpy().view(np.uint32), want):
            raise SystemExit("digests differ from the oracle")
    return {"payloads": w.n, "against": "oracle (C restatement pinned by tests/golden)", "threads": threads,
            "seconds": round(time.perf_counter() - t0, 2)}


def cgroup_cpu_quota():
    """CPUs this job's cgroup may use (quota / period), or None when unlimited or unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:  # cgroup v2: "<quota> <period>" or "max <period>"
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:  # cgroup v1
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else round(q / per, 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(h: np.ndarray, offs: np.ndarray, lens: np.ndarray, budget_s: float) -> dict:
    """Reference CPU checksum on this host's cores over a bounded sample of the same workload.
    Uses the compiled reference (oracle/_ref, kind "reference") when it travelled with the snapshot
    and the sample is a fixed-length batch, else the C restatement (kind "port")."""
    import concurrent.futures as cf

    import oracle

    host_cpus = os.cpu_count() or 1
    threads = max(1, min(16, host_cpus))  # the GPU box's CPU share for one GPU (16 of the machine's cores)
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
    elif oracle.ref_available():
        lib, kind = oracle.ref_lib(), "reference"
        out = np.zeros(n, dtype=np.uint32)
        offs_c = np.ascontiguousarray(offs, dtype=np.uint64)
        lens_c = np.ascontiguousarray(lens, dtype=np.uint32)

        def run(th):  # threads balanced by bytes (oracle/ref_wrapper.cc)
            lib.ref_crc32_batch_var_mt(h.ctypes.data, offs_c.ctypes.data, lens_c.ctypes.data, n, out.ctypes.data, th)
    else:
        kind = "port"

        def run(th):
            oracle.batch_var_mt(h, offs, lens, th)

    import resource

    def rate(th, budget):
        """(GiB/s, passes, CPU-seconds the process got per wall second while running them)"""
        ru0, reps, t0 = resource.getrusage(resource.RUSAGE_SELF), 0, time.perf_counter()
        while True:
            run(th)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= budget:
                ru1 = resource.getrusage(resource.RUSAGE_SELF)
                cpu = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
                return reps * nbytes / dt / 2 ** 30, reps, cpu / dt

    st_rate, st_reps, _ = rate(1, budget_s * 0.3)
    mt_rate, mt_reps, mt_eff = rate(threads, budget_s * 0.6)
    # the reference at hardware_concurrency() threads, what annety's one-loop-per-thread
    # pool (src/EventLoopPool.cc:55-66) would use on this host. The job's CPU quota caps what these threads get:
    # effective_cpus is the CPU time they actually received per wall second (and cgroup_cpu_quota the quota itself),
    # which is why os.cpu_count() threads can run no faster than the 16-thread leg.
    all_rate, all_reps, all_eff = (rate(host_cpus, budget_s * 0.1) if host_cpus > threads
                                   else (mt_rate, mt_reps, mt_eff))
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = None
    return {
        "value": round(mt_rate, 3),
        "unit": "GiB/s",
        "cores": threads,
        "effective_cpus": round(mt_eff, 2),
        "host_cpus": host_cpus,
        "all_cores_value": round(all_rate, 3),
        "all_cores": host_cpus,
        "all_cores_effective_cpus": round(all_eff, 2),
        "cgroup_cpu_quota": cgroup_cpu_quota(),
        "affinity_cpus": affinity,
        "kind": kind,
        "compile_flags": REF_FLAGS if kind == "reference" else "gcc -O2 (oracle/Makefile, C restatement)",
        "single_thread_value": round(st_rate, 3),
        "sample": f"{n} payloads / {nbytes / 2**20:.1f} MiB prefix of the GPU workload copied to host (memory-resident, "
                  f"far above the host caches), crc32_long per payload, payload-parallel over {threads} threads x "
                  f"{mt_reps} passes (+ 1 thread x {st_reps}; + {host_cpus} threads x {all_reps} for all_cores_value)",
    }


def pmc_traffic(w: Workload, var_path: str):
    """(per-launch HBM bytes, source file, None) of this workload's kernels from the committed rocprofv3 PMC summary
    (profiles/pmc.sh + pmc.py: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), summed over the kernels of one step;
    (None, file, reason) when the summary is missing or was measured on other kernel sources than this tree's."""
    from annety_amd.build import kernel_unit, source_digest

    path = PMC_FILES.get(w.config)
    if w.config == 3 and var_path != "arena":
        path = PMC_FILES_VAR.get(var_path)
    if w.config == "frames":
        path = PMC_FILES_FRAMES.get((w.frames_variant, w.op))
    if not path or (w.config in (1, 4) and w.L != 1024):
        return None, None, "no PMC summary for this configuration"
    try:
        with open(os.path.join(ROOT, path)) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, path, "summary missing"
    # the kernels of one step: the library's own list for it (a summary also holds the setup's launches, e.g. the
    # encode that builds the frames stream of a verify step), by name without template arguments
    step = {x.split("<")[0].strip() for x in (w.kernel or "").split("+") if x.strip()}
    have = d.get("_meta", {}).get("source_digest") or {}
    for unit in sorted({kernel_unit(k) for k in step}):
        if have.get(unit) != source_digest(unit):
            return None, path, (f"stale: {unit} measured at library sources {have.get(unit)}, this tree is "
                                f"{source_digest(unit)}")
    tot = sum(v.get("hbm_bytes_per_launch", 0) for k, v in d.items()
              if k != "_meta" and ("crc32_" in k or "lhc_" in k) and (not step or k.split("<")[0].strip() in step))
    if not tot:
        return None, path, "no kernel of this step in the summary"
    if w.config == 4:  # the config-1 measurement is per 1M payloads; a config-4 step is n/1M of them
        tot = int(tot * w.n / (1 << 20))
    return tot, path, None


def e2e_host_path(w: Workload):
    """Host-memory paths (the payloads start in host memory, off a socket): the PCIe-inclusive rate,
    never `value`. Fixed configs: annety_crc32_batch_fixed_host from a pageable buffer (parallel pack into
    the pinned ring) and from a pinned (hipHostRegister'ed) one (DMA in place). Config 3: the batch as a
    LengthHeaderCodec frame stream (built on the device by encode_batch) through decode_host =
    annety_lhc_verify_host (header walk overlapped with the upload, CRCs on the device)."""
    import annety_amd

    def rate(fn, nbytes):
        fn()  # warm: staging ring, device buffers
        reps, t0 = 0, time.perf_counter()
        while reps < 3 or time.perf_counter() - t0 < 2.0:
            fn()
            reps += 1
        dt = (time.perf_counter() - t0) / reps
        return round(nbytes / dt / 2 ** 30, 2), round(dt * 1e3, 2)

    res = {"unit": "GiB/s of payload bytes", "pcie": "Gen5 x16, ~50-56 GB/s practical (63 GB/s spec)"}
    if w.config in (1, 2):
        h = w.data.cpu().numpy()
        want = w.out.cpu().numpy().view(np.uint32)
        got = {}
        res["pageable"], res["pageable_ms"] = rate(lambda: got.__setitem__("p", annety_amd.crc32_batch_host(h, w.n, w.L)),
                                                   w.payload_bytes)
        pin = annety_amd.PinnedHostBuffer(h.size)
        pin.array[:] = h
        res["pinned"], res["pinned_ms"] = rate(lambda: got.__setitem__("q", annety_amd.crc32_batch_host(pin.array, w.n, w.L)),
                                               w.payload_bytes)
        pin.close()
        res["bit_exact_vs_device_path"] = bool(np.array_equal(got["p"], want) and np.array_equal(got["q"], want))
        res["path"] = "host buffer -> pinned 64 MiB x2 ring (parallel pack) or in place -> H2D -> kernel -> D2H, 2 streams"
        return res
    if w.config == 3:
        codec = annety_amd.LengthHeaderCodec(4)
        lens = w.lengths.cpu().numpy().astype(np.uint32)
        enc = codec.encode_batch(w.data, w.offsets.cpu().numpy().astype(np.uint64), lens)
        stream = enc.frames.cpu().numpy()
        out = {}
        res["frames_pageable"], res["frames_pageable_ms"] = rate(lambda: out.__setitem__("p", codec.decode_host(stream)),
                                                                 w.payload_bytes)
        # the same with the header walk done whole, one frame after another (no segmented speculative walks)
        annety_amd.set_walk_segment(1 << 40)
        res["frames_pageable_whole_walk"], _ = rate(lambda: codec.decode_host(stream), w.payload_bytes)
        annety_amd.set_walk_segment(0)
        pin = annety_amd.PinnedHostBuffer(stream.size)
        pin.array[:] = stream
        res["frames_pinned"], res["frames_pinned_ms"] = rate(lambda: out.__setitem__("q", codec.decode_host(pin.array)),
                                                             w.payload_bytes)
        pin.close()
        # the same frames as K connections' receive buffers (one NetBuffer per TcpConnection), verified in one
        # call (annety_lhc_verify_host_iov): the K header walks run side by side
        kconn = 16
        cuts = np.linspace(0, len(lens), kconn + 1).astype(np.int64)
        fstart = np.concatenate([[0], np.cumsum(lens.astype(np.int64) + 8)])  # T = 4 + trailer 4
        conns = [stream[int(fstart[cuts[i]]):int(fstart[cuts[i + 1]])].copy() for i in range(kconn)]
        res[f"frames_iov{kconn}_pageable"], res[f"frames_iov{kconn}_pageable_ms"] = rate(
            lambda: out.__setitem__("v", codec.decode_host_iov(conns)), w.payload_bytes)
        iov_ok = all(bool(r.ok.all()) and r.rt == 0 for r in out["v"]) and sum(int(r.ok.size) for r in out["v"]) == len(lens)
        r = out["p"]
        res["frames"] = int(r.ok.size)
        res["all_frames_verified"] = bool(r.ok.all() and out["q"].ok.all() and r.rt == 0 and r.consumed == stream.size
                                          and iov_ok)
        res["stream_bytes"] = int(stream.size)
        res["path"] = ("LengthHeaderCodec stream in host memory -> header walk (host threads, segments walked side "
                       "by side from speculative entries) || staged H2D -> arena verify on the device -> per-frame "
                       "verdicts D2H")
        return res
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0 and args.gpus > 1:
        return spawn(args.gpus)  # before anything touches the GPU
    world = max(world, 1)
    multi = world > 1 or args.dist  # the distributed code path
    if args.strong and args.config not in (1, 4):
        raise SystemExit("--strong applies to the fixed 1 KiB configs (1, 4)")
    if args.chunks is None:
        args.chunks = 2 if args.config == 4 else 1
    if args.var_path in ("sorted", "auto"):
        os.environ["ANNETY_CRC_VAR_PATH"] = args.var_path  # read once by the library: before it loads
    if args.config == "frames" and multi:
        raise SystemExit("--config frames is a one-GPU secondary line")
    if multi and int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < args.hw_queues:
        # HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default); the compute stream, torch's
        # RCCL stream and RCCL's own streams then share queues, and a queue runs its packets in order. Set
        # before HIP initialises (nothing has touched the GPU yet): one-rank rehearsal 4 -> 8 queues +4-5 %.
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if multi:
        if world == 1:
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dist.init_process_group("nccl", device_id=dev)

    import oracle
    from annety_amd import sharded

    import annety_amd

    # the checksum kernels take one workgroup per CU; with the gather overlapped on another stream, a few
    # free CUs let the RCCL kernels run beside them instead of between chunks
    annety_amd.reserve_cus(args.reserve_cus if args.reserve_cus is not None else (8 if multi else 0))
    w = Workload(args, dev, rank, world)
    if args.compute_stream == "own":
        torch.cuda.set_stream(torch.cuda.Stream(dev))
    stream = torch.cuda.current_stream(dev)
    sh = int(stream.cuda_stream)
    # strong scaling: shards differ by at most one payload; every rank gathers a buffer of the largest
    nbuf = 1 if (not multi or args.no_overlap_steps) else max(1, args.gather_buffers)
    pipe = (sharded.PipelinedGather(w.n_pad, args.chunks, dst=0, device=dev, taper=args.taper, buffers=nbuf)
            if multi else None)

    # N>1: the digests alternate between two buffers, so step s+1's chunks can be computed while step s's
    # last gathers still read the other buffer; a step's handles are waited (the compute stream waits for
    # its gathers, no host block) after the next step is launched, before the buffer comes round again
    outs = [w.out] + [torch.zeros_like(w.out) for _ in range(nbuf - 1)]
    nstep = [0]

    def step(gather: bool = True):
        if pipe is None:
            w.launch(sh)
            return []
        b = nstep[0] % len(outs)
        w.out = outs[b]
        nstep[0] += 1
        return pipe.run(lambda lo, hi: w.launch(sh, lo, hi), gather=gather, buf=b)

    def produce(s: int, lo: int, hi: int):
        w.out = outs[s % len(outs)]
        return w.launch(sh, lo, hi)

    def run_steps(steps: int, gather: bool) -> None:
        if pipe is None:
            for _ in range(steps):
                w.launch(sh)
        else:
            pipe.run_steps(produce, steps, buffers=len(outs), gather=gather)

    # correctness gate before timing: bit-exact vs the oracle on a prefix of this rank's batch, and (N > 1)
    # every rank's digests delivered to rank 0 intact (checksum of checksums)
    sharded.PipelinedGather.wait(step())
    torch.cuda.synchronize()
    steady_kernels = w.kernel
    if w.config == "frames":
        checked = w.frames_check()
    else:
        hs, ho, hl = w.host_sample()
        want = oracle.batch_var(hs, ho, hl)
        got = w.out[: len(ho)].cpu().numpy().view(np.uint32)
        if not np.array_equal(got, want):
            raise SystemExit(f"rank {rank}: digests differ from the oracle on the sample")
        checked = full_check(w, threads=min(16, os.cpu_count() or 1)) if not args.sample_check else None
    gather_ok = sharded.verify_gather(pipe.recv, w.out) if pipe is not None else None
    if gather_ok is False:
        raise SystemExit(f"rank {rank}: gathered digests differ from the ranks' own")

    def timed(steps: int, gather: bool, groups: int = 1):
        """K steps bracketed by a barrier + synchronise on both sides; max over ranks. HIP events on the
        launch stream inside the same bracket give the kernel-stream time (the roofline's launch duration);
        with groups > 1, per-group events give a per-step median / min / max (not with the gather on: its
        stream waits would cut across group boundaries)."""
        ngroups = max(1, min(groups, steps)) if (pipe is None or not gather) else 1
        gsteps = [steps * (i + 1) // ngroups - steps * i // ngroups for i in range(ngroups)]
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(ngroups + 1)]
        if multi:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        evs[0].record(stream)
        for i, gs in enumerate(gsteps):
            run_steps(gs, gather)
            evs[i + 1].record(stream)
        torch.cuda.synchronize()
        if multi:
            dist.barrier()
        el = time.perf_counter() - t0
        if multi:  # max over ranks
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        kern = evs[0].elapsed_time(evs[-1]) / steps
        per = sorted(evs[i].elapsed_time(evs[i + 1]) / gs for i, gs in enumerate(gsteps))
        return el, kern, per

    t_pw = time.perf_counter()
    while time.perf_counter() - t_pw < args.prewarm_s:
        for _ in range(10 if world == 1 else 1):
            step(gather=False)
        torch.cuda.synchronize()
    run_steps(args.warmup, True)
    torch.cuda.synchronize()

    # the timed region carries two events only (an event between two launches is a marker in the queue)
    elapsed, kern_ms, _ = timed(args.steps, gather=True)
    compute_only = None
    if multi:  # the same steps without the gather: value_compute_only, and the roofline's kernel time
        compute_only, kern_ms, _ = timed(args.steps, gather=False)
    # spread: the same K steps again in a pass of its own, a HIP event after every group of >= 10 steps (an event
    # between two launches costs the stream a few us, so per-step events would time the events: VERDICT r05)
    spread_groups = max(1, min(20, args.steps // 10))
    _, _, per_group = timed(args.steps, gather=False, groups=spread_groups)

    if rank == 0:
        traffic, traffic_path, traffic_why = pmc_traffic(w, args.var_path)
        cpu = None
        if not (args.no_cpu or multi):
            cs, co, cl = w.host_sample(CPU_SAMPLE_BYTES)
            cpu = cpu_baseline(cs, co, cl, args.cpu_seconds)
            del cs
        # every rank's payload bytes (weak: n per GPU x world; strong: the fixed total)
        total_gib = (w.n_total * w.L if w.L else w.payload_bytes * world) * args.steps / 2 ** 30
        achieved = w.algo_bytes / (kern_ms / 1e3) / 1e9
        if args.config == 1:
            metric = METRIC if not args.strong else METRIC.replace("(1M×1KiB)", "(1M×1KiB total, strong scaling)")
        elif args.config == 4:
            metric = METRIC.replace("(1M×1KiB)", "(8M×1KiB per GPU, config 4)" if not args.strong
                                    else "(8M×1KiB total, config 4, strong scaling)")
        elif args.config == "frames":
            metric = METRIC.replace("(1M×1KiB)", f"(annety frames, {args.frames}, {args.op})")
        else:
            metric = METRIC.replace("(1M×1KiB)", f"(config {args.config})")
        line = {
            "metric": metric,
            "value": round(total_gib / elapsed, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (torch.randint bytes on device, seeded per rank)",
            "config": {
                "workload": w.desc,
                "payloads_per_gpu": w.n,
                "payloads_total": w.n_total,
                "payload_bytes": w.L if w.L else ("zipf" if w.config == 3 else args.frames),
                "bytes_per_gpu": w.payload_bytes,
                "parallelism": f"shard{world}" if multi else "single",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": (f"{traffic_path}: rocprofv3 PMC passes (FETCH_SIZE x2 + WRITE_SIZE) of this command, "
                                   "committed, stamped with this tree's library source digest" if traffic else None),
                "traffic_refused": None if traffic else {"file": traffic_path, "why": traffic_why},
                "kernel": steady_kernels,
                "kernel_source": "annety_crc_last_kernels() after the gate's step (the library's own launch choice)",
                # HIP events on the launch stream around the timed region's K steps
                "kernel_ms_avg": round(kern_ms, 4),
                "algorithmic_bytes_per_launch": w.algo_bytes,
            },
            # a second pass of the same K steps, right after the timed one, with a HIP event after every group of
            # steps: the kernel-stream time per step within each group (not the timed region's)
            "step_spread": {"groups": len(per_group), "steps_per_group": args.steps // len(per_group),
                            "min_ms": round(per_group[0], 4), "median_ms": round(float(np.median(per_group)), 4),
                            "max_ms": round(per_group[-1], 4)},
            "cpu_baseline": cpu,
            "checked_vs_oracle": checked,
        }
        if multi:
            line["rccl_ranks"] = dist.get_world_size()
            line["backend"] = dist.get_backend()
            line["gather"] = {"what": "every rank's digests to rank 0 (RCCL gather over xGMI), inside `value`",
                              "chunks": len(pipe.bounds), "bytes_to_rank0_per_step": 4 * w.n_pad * (world - 1),
                              "verified": bool(gather_ok), "overlapped_with_compute": True,
                              "overlapped_across_steps": len(outs) > 1}
            line["value_compute_only"] = round(total_gib / compute_only, 2)
        if args.e2e and world == 1:
            line["e2e_host_path"] = e2e_host_path(w)
        print(json.dumps(line), flush=True)
    if multi:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
