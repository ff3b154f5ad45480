"""Host sanitizers on the native runtime (SURVEY §5.2 race detection): the parameter server and
the batch loader — the concurrent C++ code — built with AddressSanitizer + UBSan and with
ThreadSanitizer and driven by a multi-threaded stress program (csrc/tests/runtime_stress.cpp).
GPU sanitizers are not available on the MI355X pool; the HIP kernels are covered by the
numerics tests and the static ISA checks instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "distributeddeeplearningspark_amd", "csrc")
SOURCES = [os.path.join(CSRC, "tests", "runtime_stress.cpp"), os.path.join(CSRC, "runtime", "param_server.cpp"),
           os.path.join(CSRC, "runtime", "loader.cpp")]

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_runtime_under_sanitizer(tmp_path, san):
    exe = str(tmp_path / "rt")
    flags = ["-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-I",
             os.path.join(CSRC, "include")]
    r = subprocess.run(["g++", *flags, *SOURCES, "-o", exe, "-lpthread"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    run = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    report = run.stdout + run.stderr
    assert run.returncode == 0, report[-4000:]
    assert "runtime stress: ok" in run.stdout
    for marker in ("ERROR: AddressSanitizer", "WARNING: ThreadSanitizer", "runtime error:"):
        assert marker not in report, report[-4000:]
