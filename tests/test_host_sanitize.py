"""The host-side image builders under sanitizers (CPU only).

kry_csr_create builds its SELL-64, diagonal-offset, column-blocked and
paired-row images on the host with up to 16 threads, and hands large staging
vectors to a detached thread to free (release_later). That code lives in one
plain C++ translation unit, krylov_amd/csrc/host_image.cpp, which the library
links; `make -C krylov_amd/csrc sanitize` builds it alone as two host-only
libraries, one with AddressSanitizer + UndefinedBehaviorSanitizer and one with
ThreadSanitizer. Here the plan tests of tests/test_abi.py (SELL layout, DIA,
paired-row and column-blocked plans, threaded sizes included) run against
each, loaded through KRYLOV_LIB with the sanitizer runtime preloaded into a
child interpreter; any report fails the test (halt_on_error)."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(REPO, "krylov_amd", "csrc")


def _runtime(name):
    out = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True, check=True)
    path = out.stdout.strip()
    return path if os.path.isabs(path) and os.path.exists(path) else None


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_plan_tests_under_sanitizer(kind):
    if os.environ.get("LD_PRELOAD"):
        pytest.skip("the environment already preloads a library; not stacking a sanitizer runtime on it")
    runtime = _runtime("libasan.so" if kind == "asan" else "libtsan.so")
    if runtime is None:
        pytest.skip(f"no {kind} runtime in this toolchain")
    subprocess.run(["make", "-s", "-C", CSRC, "sanitize"], check=True)
    lib = os.path.join(CSRC, "build", "san", f"libkrylov_host_{kind}.so")
    env = dict(os.environ)
    # libstdc++ preloaded beside the sanitizer runtime: ASan resolves the real
    # __cxa_throw when it starts, and the plan entry points throw (rejected
    # CSR input) from a library loaded later by ctypes
    cxx = _runtime("libstdc++.so")
    env.update({
        "KRYLOV_LIB": lib,
        "LD_PRELOAD": runtime + (" " + cxx if cxx else ""),
        "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1",
        "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1",
        "TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1",
        "PYTHONDONTWRITEBYTECODE": "1",
    })
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(HERE, "test_abi.py"), "-k", "layout or plan"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=1200)
    out = r.stdout + r.stderr
    for marker in ("AddressSanitizer", "ThreadSanitizer", "runtime error:", "LeakSanitizer"):
        assert marker not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert " passed" in r.stdout
