"""Host sanitizers: the engine's host-side C/C++ (kdf.cpp key schedule, the host PN codec in
qpp_internal.h) and the oracle, built with ASan + UBSan (tests/sanitize/Makefile) and run over known answers
(RFC 9001 A.1) and randomized cross-checks.  A sanitizer report fails the test.  CPU only."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "sanitize")


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="needs hipcc (clang) to build")
def test_host_code_under_asan_ubsan(tmp_path):
    out = str(tmp_path / "host_check")
    subprocess.run(["make", "-s", "-C", HERE, f"OUT={out}"], check=True, timeout=600,
                   stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([out], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_check ok" in r.stdout
    for f in os.listdir(HERE):
        if f.endswith(".o"):
            os.remove(os.path.join(HERE, f))
