"""Sanitizer builds of the native host runtime.

GPU AddressSanitizer / xnack+ code objects are not available on the MI355X pool, so
the sanitizers run on the host C++ (`csrc/host/gnnqc_host.cpp`: rolling statistics,
CRC32C): `csrc/tests/test_host_sanitize.cpp` is compiled with ASan+UBSan and with
TSan and run here on the CPU. The GPU kernels are covered by the oracle and
bitwise-determinism tests in `test_kernels_gpu.py` / `test_resilience.py`.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "tests", "test_host_sanitize.cpp")

SANITIZERS = {
    "asan_ubsan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"],
    "tsan": ["-fsanitize=thread"],
}


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
@pytest.mark.parametrize("kind", sorted(SANITIZERS))
def test_host_runtime_under_sanitizer(kind, tmp_path):
    exe = str(tmp_path / f"host_{kind}")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-msse4.2", "-pthread", *SANITIZERS[kind], SRC, "-o", exe]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               TSAN_OPTIONS="halt_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300, env=env)
    if kind == "tsan" and "FATAL: ThreadSanitizer" in r.stdout:
        pytest.skip("TSan runtime cannot map its shadow memory here: " + r.stdout.splitlines()[0])
    assert r.returncode == 0, r.stdout
    assert "self-test OK" in r.stdout
