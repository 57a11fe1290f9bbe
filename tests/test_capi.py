"""C-ABI boundary checks that need no GPU: the library loads, exports exactly what
include/annety_crc.h declares, the host scalar API and the drop-in tables match the reference
fixtures, and the C++ drop-in header compiles (and, where the reference tree exists, compiles the
reference's own LengthHeaderCodec unchanged against it)."""
import ctypes
import os
import re
import subprocess
import zlib

import numpy as np
import pytest

import annety_amd
from annety_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "annety_crc.h")


def H(x: str) -> int:
    return int(x, 16)


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(annety_(?:crc|lhc|pbc)\w*)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = _lib.get()
    syms = declared_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(lib, s), s
    # the ctypes table in _lib covers the whole header (the binding INTEGRATION.md documents)
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == syms
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.lib_path()], capture_output=True, text=True).stdout
    for s in syms:
        assert re.search(rf"\bT {s}$", out, re.M), s
    # the reference's table globals, same C++ symbols as src/Crc32c.cc
    assert "_ZN6annety8internal14crc32_table256E" in out
    assert "_ZN6annety8internal13crc32_table16E" in out


def test_abi_version_and_errors():
    lib = _lib.get()
    want = int(re.search(r"#define ANNETY_CRC_ABI_VERSION (\d+)", open(HEADER).read()).group(1))
    assert lib.annety_crc_abi_version() == want
    assert lib.annety_crc_strerror(-1) == b"invalid argument"
    # argument errors are reported before any device is touched
    assert lib.annety_crc32_batch_fixed(None, 4, 16, 16, None, None) == -1
    assert lib.annety_crc32_batch_fixed(None, 0, 16, 16, None, None) == 0  # empty batch is a no-op
    assert lib.annety_crc32_batch_var(None, None, None, 3, None, None) == -1
    assert lib.annety_crc32_batch_fixed_host(None, 2, 16, 8, None) == -1  # stride < len
    assert lib.annety_crc32_batch_var_arena(None, 64, None, None, 3, None, None) == -1
    assert lib.annety_crc32_update_batch_var_arena(None, None, 64, None, None, 0, None) == 0
    assert lib.annety_lhc_verify_stream(None, 64, None, None, 2, None, None, None) == -1


def test_host_scalar_api_matches_reference(golden):
    k = golden("kat.json")
    for kat in k["kats"]:
        data = bytes.fromhex(kat["hex"])
        assert annety_amd.Crc32c.crc32_long(data) == H(kat["crc32_long"])
        assert annety_amd.Crc32c.crc32_short(data) == H(kat["crc32_short"])
    assert annety_amd.Crc32c.crc32_update(0, b"123456789") == H(k["update"]["from_zero_123456789"])
    t256, t16 = annety_amd.tables()
    assert [int(x) for x in t256] == [H(x) for x in k["table256"]]
    assert [int(x) for x in t16] == [H(x) for x in k["table16"]]


def test_host_combine(golden):
    for c in golden("combine.json")["cases"]:
        assert annety_amd.crc32_combine(H(c["crcA"]), H(c["crcB"]), c["lenB"]) == H(c["crcAB"])


def test_scalar_random_vs_zlib():
    rng = np.random.default_rng(11)
    for _ in range(200):
        a = rng.integers(0, 256, int(rng.integers(0, 5000)), dtype=np.uint8).tobytes()
        assert annety_amd.Crc32c.crc32_long(a) == zlib.crc32(a)
        assert annety_amd.Crc32c.crc32_short(a) == zlib.crc32(a)


def test_batch_path_refuses_host_tensors():
    torch = pytest.importorskip("torch")
    with pytest.raises(ValueError, match="no CPU fallback"):
        annety_amd.crc32_batch(torch.zeros(64, dtype=torch.uint8), 4, 16)


CPP_DROPIN = r"""
#define ANNETY_CRC_NO_STRINGPIECE
#include "annety/Crc32c.h"
#include <cstdio>
#include <cstring>
int main() {
  const char* s = "123456789";
  uint32_t st = 0;
  annety::Crc32c::crc32_update(&st, s, 9);
  int ok = annety::Crc32c::crc32_long(s, 9) == 0xCBF43926u && annety::Crc32c::crc32_short(s, 9) == 0xCBF43926u &&
           st == 0x2DFD2D88u && annety::internal::crc32_table256[1] == 0x77073096u &&
           annety::Crc32c::crc32_combine(annety::Crc32c::crc32_long(s, 4), annety::Crc32c::crc32_long(s + 4, 5), 5) ==
               0xCBF43926u;
  std::printf("%s\n", ok ? "OK" : "BAD");
  return ok ? 0 : 1;
}
"""


def test_cpp_dropin_header_links_and_runs(tmp_path):
    src = tmp_path / "t.cc"
    src.write_text(CPP_DROPIN)
    exe = tmp_path / "t"
    libdir = os.path.dirname(_lib.lib_path())
    subprocess.run(["g++", "-std=c++11", "-O2", "-Wall", "-Wextra", "-Werror", f"-I{ROOT}/include", str(src), "-o",
                    str(exe), f"-L{libdir}", "-lannety_crc", f"-Wl,-rpath,{libdir}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip() == "OK", r.stdout + r.stderr


CODEC_TU = r"""
// The reference's own framing codec, unchanged, compiled against the drop-in Crc32c.h.
#include "codec/LengthHeaderCodec.h"
#ifndef ANNETY_AMD_CRC32C_H
#error "the reference Crc32c.h was picked up instead of the drop-in"
#endif
int main() { return 0; }
"""


@pytest.mark.skipif(not os.path.isdir("/root/reference/include/codec"), reason="reference tree not present")
def test_reference_codec_compiles_against_dropin(tmp_path):
    # include/annety/ first on the path so "Crc32c.h" resolves to the drop-in, the rest to the reference.
    src = tmp_path / "codec.cc"
    src.write_text(CODEC_TU)
    r = subprocess.run(["g++", "-std=c++11", "-fsyntax-only", f"-I{ROOT}/include/annety", f"-I{ROOT}/include",
                        "-I/root/reference/include", "-I/root/reference/src", str(src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]


def test_shard_plan_through_cabi():
    """annety_crc_shard_plan (the C-ABI's shard arithmetic for device groups) against shard_range."""
    from annety_amd import sharded

    for n in [0, 1, 7, 1000, 1001, (64 << 20), (1 << 40) + 3]:
        for k in [1, 2, 3, 8]:
            plan = sharded.shard_plan(n, k)
            assert [(f, f + c) for f, c in plan] == [sharded.shard_range(n, r, k) for r in range(k)]
    lib = _lib.get()
    assert lib.annety_crc_shard_plan(10, 0, None, None) == -1


def test_group_errors_without_device():
    """Group creation validates arguments before touching RCCL; with no GPU it reports ENODEV."""
    import ctypes

    lib = _lib.get()
    h = ctypes.c_void_p()
    assert lib.annety_crc_group_create(None, 1, ctypes.byref(h)) == -1
    devs = (ctypes.c_int * 2)(0, 0)
    rc = lib.annety_crc_group_create(devs, 2, ctypes.byref(h))
    assert rc in (-1, -4)  # repeated device (EINVAL) or no device (ENODEV)
    assert lib.annety_crc_group_size(None) == 0
    assert lib.annety_crc_group_destroy(None) == 0
    assert lib.annety_crc32_group_batch_fixed(None, None, None, 16, 16, None, 1) == -1


def test_group_schedule_eight_devices():
    """The transfer schedule of annety_crc32_group_batch_fixed (annety_crc_group_schedule, the same
    arithmetic the send/recv loop runs) for 8 devices: every payload of the batch is computed exactly once
    and its digest lands at its global index in the root's output; pieces tile each shard in order; a
    device's piece c is the same on the sending and the receiving side."""
    from annety_amd import sharded

    lib = _lib.get()
    assert lib.annety_crc_group_schedule(None, 8, 2, None) == -1
    for n in [1, 7, 8, 1000, 1001, 64 << 20]:
        shards = sharded.shard_plan(n, 8)
        counts = [c for _, c in shards]
        for chunks in [1, 2, 3, 8, 13]:
            plan = sharded.group_schedule(counts, chunks)
            seen = np.zeros(n, dtype=np.int8) if n < (1 << 20) else None
            for k in range(8):
                pos = 0
                for c in range(chunks):
                    lo, cnt, dst = plan[c][k]
                    assert lo == pos  # pieces tile shard k in order
                    assert dst == shards[k][0] + lo  # global index = shard start + offset in the shard
                    pos += cnt
                    if seen is not None:
                        seen[dst:dst + cnt] += 1
                assert pos == counts[k]
                sizes = [plan[c][k][1] for c in range(chunks)]
                assert max(sizes) - min(sizes) <= 1  # near-equal pieces
            if seen is not None:
                assert (seen == 1).all()


def test_boundary_error_paths_without_device():
    """Error paths of the entry points added for multi-stream / multi-device callers, on a host with no
    GPU: argument checks come first, and a call that needs a device reports it instead of crashing."""
    import ctypes

    lib = _lib.get()
    assert lib.annety_crc_set_split(2, 0) == -1  # mode out of range
    assert lib.annety_crc_set_split(1, 5000) == -1  # segment not a power of two
    assert lib.annety_crc_set_split(1, 1024) == -1  # segment below 4 KiB
    assert lib.annety_crc_set_split(-1, 0) == 0
    assert lib.annety_crc_set_split_cap((1 << 18) + 1) == -1  # above kSplitSegCap
    assert lib.annety_crc_set_split_cap(0) == 0
    assert lib.annety_crc_set_split_cap(1 << 18) == 0
    v = [ctypes.c_uint64(7) for _ in range(3)]
    assert lib.annety_crc_scratch_stats(-1, *[ctypes.byref(x) for x in v]) == -4
    assert lib.annety_crc_scratch_stats(0, *[ctypes.byref(x) for x in v]) == 0
    assert [x.value for x in v] == [0, 0, 0]  # nothing ran on device 0 in this process
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        buf = (ctypes.c_uint8 * 64)()
        out = (ctypes.c_uint32 * 4)()
        # valid arguments, no device: a negative status (no HIP device), never a crash
        assert lib.annety_crc32_batch_fixed(ctypes.addressof(buf), 4, 16, 16, ctypes.addressof(out), None) < 0
        assert lib.annety_crc_stream_release(None) < 0


def test_host_register_refuses_shared_pages_without_device():
    """annety_crc_host_register's argument rules run before any HIP call: a pointer that is not
    page-aligned, zero bytes or null is refused with EINVAL, and unregistering a pointer the library did
    not pin is EINVAL too (the library never passes such a pointer to the runtime). The overlap rule is
    covered with real registrations in tests/test_gpu_parity.py and in the host self-test."""
    import ctypes
    import mmap

    lib = _lib.get()
    m = mmap.mmap(-1, 4 * mmap.PAGESIZE)
    buf = (ctypes.c_uint8 * len(m)).from_buffer(m)
    base = ctypes.addressof(buf)
    assert base % mmap.PAGESIZE == 0
    assert lib.annety_crc_host_register(base + 8, 100) == -1  # not page-aligned
    assert lib.annety_crc_host_register(base, 0) == -1
    assert lib.annety_crc_host_register(None, 100) == -1
    assert lib.annety_crc_host_unregister(base) == -1  # not pinned here
    assert lib.annety_crc_host_unregister(None) == -1
    assert lib.annety_crc_last_error_stage() in (b"", None) or isinstance(lib.annety_crc_last_error_stage(), bytes)
    assert lib.annety_crc_set_frames_pack(2) == -1
    assert lib.annety_crc_set_frames_pack(1) == 0
    del buf
    m.close()


def test_product_kernels_do_not_spill(tmp_path):
    """Every gfx950 kernel in libannety_crc.so runs without scratch (no VGPR spills): the 1024-lane stitch
    variant that returned wrong digests in round 2 was the only build that spilled (DESIGN.md §7.2;
    microbench/isa_check.py), so a change that pushes a product kernel into spilling fails here, on the
    CPU, before it reaches a GPU."""
    import shutil

    objdump = "/opt/rocm/lib/llvm/bin/llvm-objdump"
    readelf = "/opt/rocm/lib/llvm/bin/llvm-readelf"
    if not (os.path.exists(objdump) and os.path.exists(readelf)):
        pytest.skip("ROCm llvm tools not present")
    lib = tmp_path / "lib.so"
    shutil.copy(_lib.lib_path(), lib)
    subprocess.run([objdump, "--offloading", str(lib)], check=True, capture_output=True, cwd=tmp_path)
    objs = sorted(p for p in tmp_path.iterdir() if "gfx950" in p.name)
    assert objs, "no gfx950 code object in the library"
    kernels = {}
    for co in objs:
        notes = subprocess.run([readelf, "--notes", str(co)], check=True, capture_output=True, text=True).stdout
        for block in notes.split("  - .agpr_count")[1:]:
            name = re.search(r"\.name:\s+(\S+)", block).group(1)
            kernels[name] = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", block).group(1))
    assert any("crc32_arena_stitch_kernel" in k for k in kernels) and any("oneround" in k for k in kernels)
    spilling = {k: v for k, v in kernels.items() if v}
    assert not spilling, spilling


OPERATIONAL_KNOBS = {"ANNETY_CRC_SYNC_STAGES", "ANNETY_CRC_STREAM_SLOTS", "ANNETY_CRC_VAR_PATH", "ANNETY_CRC_VAR_AUTO",
                     "ANNETY_CRC_SPLIT", "ANNETY_CRC_SEG", "ANNETY_CRC_FRAMES_PACK", "ANNETY_CRC_PACK_THREADS",
                     "ANNETY_CRC_WALK_THREADS"}


def test_product_library_reads_only_operational_knobs():
    """The shipping libannety_crc.so names no A/B or probe switch (ANNETY_CRC_SORTED_CLASSES and
    ANNETY_CRC_STREAM_PROBE made the product write wrong digests): every ANNETY_CRC_* string in the binary is an
    operational knob (scratch slots, variable-path choice, split policy, staging/walk threads, stage syncs),
    none of which changes a digest. The A/B switches exist only in -DANNETY_CRC_AB builds (crc32_kernels.h)."""
    blob = open(_lib.lib_path(), "rb").read()
    names = {m.decode() for m in re.findall(rb"ANNETY_CRC_[A-Z0-9_]+", blob)}
    assert names, "no environment knob found at all: the string scan is broken"
    assert names <= OPERATIONAL_KNOBS, sorted(names - OPERATIONAL_KNOBS)
    for probe in ("SORTED_CLASSES", "STREAM_PROBE", "STITCH_MID", "STITCH_PIPE", "SORTED_NT", "LINES_NT", "FIXED_NT",
                  "SORTED_FUSED"):
        assert ("ANNETY_CRC_" + probe).encode() not in blob, probe


def test_verify_host_iov_arguments_without_device():
    """annety_lhc_verify_host_iov argument rules (before any device work): bad length type, a NULL buffer
    with a size, missing outputs; an all-empty call walks nothing and needs no device."""
    import ctypes

    lib = _lib.get()
    sizes = (ctypes.c_size_t * 2)(0, 0)
    bufs = (ctypes.c_void_p * 2)(None, None)
    nf = (ctypes.c_size_t * 2)(9, 9)
    used = (ctypes.c_size_t * 2)(9, 9)
    rt = (ctypes.c_int * 2)(9, 9)
    assert lib.annety_lhc_verify_host_iov(bufs, sizes, 2, 3, 0, None, None, None, 0, nf, used, rt) == -1
    assert lib.annety_lhc_verify_host_iov(bufs, sizes, 2, 4, 0, None, None, None, 0, nf, used, rt) == 0
    assert list(nf) == [0, 0] and list(used) == [0, 0] and list(rt) == [0, 0]
    sizes[1] = 10
    assert lib.annety_lhc_verify_host_iov(bufs, sizes, 2, 4, 0, None, None, None, 0, nf, used, rt) == -1
    assert lib.annety_lhc_verify_host_iov(bufs, sizes, 2, 4, 0, None, None, None, 5, nf, used, rt) == -1
    # the host walk alone (max_frames 0: no device): one buffer with an invalid length reports rt 1
    hdr = (ctypes.c_uint8 * 4)(0, 0, 0, 2)  # length 2 < 4
    bufs[0], sizes[0], sizes[1] = ctypes.addressof(hdr), 4, 0
    assert lib.annety_lhc_verify_host_iov(bufs, sizes, 2, 4, 0, None, None, None, 0, nf, used, rt) == 0
    assert list(nf) == [0, 0] and list(used) == [0, 0] and list(rt) == [0, 0]  # max_frames 0: nothing walked
