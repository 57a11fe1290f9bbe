"""The engine's host-only parts under sanitizers (SURVEY.md §5 race detection; the reference relies on
-Wthread-safety, CMakeLists.txt:34, and runtime thread checks, src/EventLoop.cc:215-221).

`make -C annety_amd/csrc sanitize` builds crc32_host.cpp (worker pools, frame walks, encode plans, host
registrations, shard plans, the per-stream scratch slot table) with g++ twice - AddressSanitizer + UBSan and
ThreadSanitizer - and runs tests/native/host_selftest.cpp under each: concurrent callers of every part, the
walks against a sequential LengthHeaderCodec::decode walk, and the slot table's hand-over ordering over a fake
runtime. Then the Python host-side tests (frame walks, codec/encode-plan properties) run against the same
sanitized builds through ctypes (ANNETY_CRC_HOST_LIB, the sanitizer runtime preloaded). No GPU needed."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "annety_amd", "csrc")
SAN = os.path.join(CSRC, "build", "san")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None,
                                reason="needs g++ and make")

REPORTS = ("ERROR: AddressSanitizer", "WARNING: ThreadSanitizer", "runtime error:", "ERROR: LeakSanitizer")


def _clean(out: str) -> None:
    for r in REPORTS:
        assert r not in out, out[-4000:]


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-s", "-C", CSRC, "build-sanitize"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_selftest(built, kind):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(SAN, f"host_selftest_{kind}")], capture_output=True, text=True, timeout=600,
                       env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "host self-test passed" in r.stdout
    _clean(out)


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_python_host_tests_under_sanitizer(built, kind):
    """tests/test_walk.py and the host-side (CPU) tests of the codecs through the sanitized host library."""
    rt = subprocess.run(["gcc", f"-print-file-name=lib{kind}.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(rt) or not os.path.exists(rt):
        pytest.skip(f"lib{kind}.so not found")
    env = dict(os.environ, LD_PRELOAD=rt, ANNETY_CRC_HOST_LIB=os.path.join(SAN, f"libannety_host_{kind}.so"),
               ASAN_OPTIONS="detect_leaks=0", TSAN_OPTIONS="halt_on_error=1", PYTHONDONTWRITEBYTECODE="1")
    tests = [os.path.join(ROOT, "tests", t) for t in ("test_walk.py", "test_lhc.py", "test_pbc.py")]
    # tests that start compilers are left out: the preloaded sanitizer runtime would follow them into g++
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu", "-k", "not dropin and not cpp_", "-p",
                        "no:cacheprovider", *tests],
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert " passed" in r.stdout
    _clean(out)
