"""Build the native engine in-tree: annety_amd/libannety_crc.so (HIP for gfx950 + the C-ABI shim).

Used by __graft_entry__.build() and, on a GPU box whose snapshot lacks the .so, by the loader.
Pure hipcc command lines (no torch extension machinery): the product is a plain C-ABI shared library.
"""
from __future__ import annotations

import concurrent.futures
import os
import shutil
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB = os.path.join(PKG, "libannety_crc.so")
SOURCES = ["crc32_kernels.hip", "crc32_arena.hip", "crc32_frames.hip", "crc32_host.cpp", "crc32_capi.cpp",
           "crc32_group.cpp"]
HEADERS = ["crc32_kernels.h", "crc32_math.h", "crc32_device.h", "crc32_arena_lines.h", "crc32_host.h"]
ARCH = "gfx950"
ROCM_LIB = "/opt/rocm/lib"


def hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise FileNotFoundError("hipcc not found (ROCm toolchain required to build libannety_crc.so)")


def _inputs() -> list[str]:
    files = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    files.append(os.path.join(INCLUDE, "annety_crc.h"))
    return files


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(f) <= t for f in _inputs())


# The translation unit that holds each product kernel (by name prefix), for the per-unit source digests below.
KERNEL_UNITS = (("lhc_", "crc32_frames.hip"), ("crc32_arena_", "crc32_arena.hip"),
                ("crc32_extent_kernel", "crc32_arena.hip"), ("crc32_bucket_place", "crc32_arena.hip"),
                ("crc32_", "crc32_kernels.hip"))


def kernel_unit(kernel: str) -> str:
    """The .hip file that defines `kernel` (a name as rocprofv3 or annety_crc_last_kernels reports it)."""
    k = kernel.replace("void ", "").replace("annety_crc::(anonymous namespace)::", "").strip()
    for prefix, unit in KERNEL_UNITS:
        if k.startswith(prefix):
            return unit
    raise KeyError(kernel)


def source_digest(unit: str | None = None) -> str:
    """sha256 (16 hex digits) over what decides a kernel's code and launches: the kernel's translation unit (`unit`,
    a .hip file; None = every one), every header and the C-ABI shim that chooses its grids. A committed measurement
    of the kernels (profiles/pmc.py) carries the digests of the units it measured, and bench.py reports it as the
    traffic of the kernels it runs only while those digests are the tree's (stale PMC summaries)."""
    import hashlib

    files = [f for f in _inputs() if not f.endswith(".hip") or unit is None or os.path.basename(f) == unit]
    h = hashlib.sha256()
    for f in sorted(files):
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


AB_LIB = os.path.join(ROOT, "microbench", "libannety_crc_ab.so")


def build(force: bool = False, verbose: bool = False, ab: bool = False, defines: tuple = (), out: str | None = None) -> str:
    """The product library, or with ab=True the design-space build (-DANNETY_CRC_AB: the A/B and probe switches
    read from the environment, crc32_kernels.h) at microbench/libannety_crc_ab.so, loaded with ANNETY_CRC_LIB.
    `defines` (compile-time A/B macros, e.g. ANNETY_S_NT=0) need `out`, a library path of their own. Neither is
    ever the product: tests and the bench load LIB."""
    if defines and not out:
        raise ValueError("a build with extra defines needs its own output path")
    lib = out or (AB_LIB if ab else LIB)
    if not force and not ab and not out and up_to_date():
        return LIB
    tmp = os.path.join(PKG, "build", "ab" if ab else "", "x" if out else "")
    os.makedirs(tmp, exist_ok=True)
    common = ["-std=c++17", "-O3", "-fPIC", f"-I{INCLUDE}", f"-I{CSRC}", "-Wall"] + (["-DANNETY_CRC_AB"] if ab else [])
    common += [f"-D{d}" for d in defines]
    cmds, objs = [], []
    for s in SOURCES:
        src = os.path.join(CSRC, s)
        obj = os.path.join(tmp, s + ".o")
        cmd = [hipcc()] + common + ["-c", src, "-o", obj]
        if s.endswith(".hip"):
            cmd[1:1] = [f"--offload-arch={ARCH}"]
        if verbose:
            print(" ".join(cmd))
        cmds.append(cmd)
        objs.append(obj)
    # the translation units are independent: compile them side by side
    with concurrent.futures.ThreadPoolExecutor(max_workers=min(len(cmds), 8)) as ex:
        for f in [ex.submit(subprocess.run, c, check=True) for c in cmds]:
            f.result()
    out_tmp = lib + ".tmp"
    # RCCL for the device-group entry points (crc32_group.cpp); rpath so the library loads without
    # LD_LIBRARY_PATH on any box with this ROCm image
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out_tmp] + objs + [
        f"-L{ROCM_LIB}", "-lrccl", f"-Wl,-rpath,{ROCM_LIB}"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out_tmp, lib)
    if not ab and not out:
        build_native_tests(verbose)
    return lib


NATIVE_TESTS = os.path.join(ROOT, "tests", "native")


def build_native_tests(verbose: bool = False) -> None:
    """The GPU test programs that use the C++ headers directly (tests/native/*_device.cpp, run by tests/test_lhc.py),
    linked against the in-tree library through an $ORIGIN-relative rpath so they run from any checkout."""
    for src in sorted(f for f in os.listdir(NATIVE_TESTS) if f.endswith("_device.cpp")):
        exe = os.path.join(NATIVE_TESTS, src[:-4])
        cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
               f"-I{INCLUDE}", os.path.join(NATIVE_TESTS, src), "-o", exe, f"-L{PKG}", "-lannety_crc", f"-L{ROCM_LIB}",
               "-lamdhip64", "-Wl,-rpath,$ORIGIN/../../annety_amd", f"-Wl,-rpath,{ROCM_LIB}"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)


if __name__ == "__main__":
    import sys

    # python -m annety_amd.build [--ab] [-D MACRO=V ... -o path]
    args = sys.argv[1:]
    defs = tuple(args[i + 1] for i, a in enumerate(args) if a == "-D")
    out = args[args.index("-o") + 1] if "-o" in args else None
    print(build(force=True, verbose=True, ab="--ab" in args, defines=defs, out=out))
