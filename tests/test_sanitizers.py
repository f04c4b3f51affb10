"""CPU sanitizer runs (race detection): the host code that has threads
runs under AddressSanitizer + UBSan and ThreadSanitizer here, on the CPU.

  * the oracle's OpenMP checkers (oracle/jg_oracle.c) through oracle/san_driver.c, which cross-checks
    each parallel checker against the serial restatement it is pinned to: `make -C oracle asan` (gcc) and
    `make -C oracle tsan` (clang with its libomp, whose runtime TSan understands; gcc's libgomp is not
    instrumented);
  * the device block cache behind every DevBuf (janusgraph_amd/csrc/jg_cache.h, the allocator
    jg_api.cpp runs over HIP) over a malloc backend, hammered by 8 threads (tests/san/cache_stress.cpp).

The reference's thread-safety model is `synchronized` VertexState mutators
(janusgraph-core/.../olap/computer/VertexState.java:77,85,135); these runs are the restatement's and the
library's host side of that guarantee.  GPU code is not sanitised (no GPU ASan on this pool).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/llvm/bin/clang"
SAN_ENV = {**os.environ, "OMP_NUM_THREADS": "4", "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0",
           "TSAN_OPTIONS": "ignore_noninstrumented_modules=1 halt_on_error=1 exitcode=66"}


def run(cmd, **kw):
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, **kw)
    return p.returncode, p.stdout + p.stderr


def have_clang():
    return os.path.exists(CLANG) and os.path.exists(os.path.join(os.path.dirname(CLANG), "..", "lib", "libomp.so"))


@pytest.fixture(scope="module")
def oracle_san():
    rc, out = run(["make", "-C", os.path.join(ROOT, "oracle"), "asan"] + (["tsan"] if have_clang() else []))
    assert rc == 0, out
    return os.path.join(ROOT, "oracle", "_san")


def test_oracle_asan_ubsan(oracle_san):
    rc, out = run([os.path.join(oracle_san, "oracle_asan"), "8", "12"], env=SAN_ENV)
    assert rc == 0 and "0 failures" in out, out
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out


@pytest.mark.skipif(not have_clang(), reason="clang + libomp (ROCm LLVM) not found")
def test_oracle_tsan(oracle_san):
    rc, out = run([os.path.join(oracle_san, "oracle_tsan"), "8", "11"], env=SAN_ENV)
    assert rc == 0 and "0 failures" in out, out
    assert "ThreadSanitizer" not in out, out


def build_stress(tmp_path, flags, cxx):
    exe = str(tmp_path / "cache_stress")
    rc, out = run([cxx, "-std=c++17", "-O1", "-g", "-pthread", *flags, "-I", os.path.join(ROOT, "janusgraph_amd", "csrc"),
                   os.path.join(ROOT, "tests", "san", "cache_stress.cpp"), "-o", exe])
    assert rc == 0, out
    return exe


def test_block_cache_asan(tmp_path):
    exe = build_stress(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], "g++")
    rc, out = run([exe, "8", "20000"], env=SAN_ENV)
    assert rc == 0 and " 0 bad" in out, out
    assert "AddressSanitizer" not in out and "runtime error" not in out, out


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_block_cache_tsan(tmp_path):
    cxx = CLANG + "++" if os.path.exists(CLANG + "++") else "g++"
    exe = build_stress(tmp_path, ["-fsanitize=thread"], cxx)
    rc, out = run([exe, "8", "4000"], env=SAN_ENV)
    assert rc == 0 and " 0 bad" in out, out
    assert "ThreadSanitizer" not in out, out
