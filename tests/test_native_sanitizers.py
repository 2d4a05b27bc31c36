"""Host-side sanitizer runs of the native runtime (CPU).

The scheduler library source is compiled together with a multi-threaded stress driver
(tests/native/sched_stress.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer and
under ThreadSanitizer, then executed; any report makes the binary exit non-zero."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "cloud_server_amd", "csrc", "runtime", "scheduler.cpp"),
       os.path.join(ROOT, "tests", "native", "sched_stress.cpp")]
CXX = shutil.which("g++") or shutil.which("c++")


@pytest.mark.skipif(CXX is None, reason="no host C++ compiler")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_scheduler_under_sanitizer(tmp_path, san):
    exe = str(tmp_path / "stress")
    cmd = [CXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}",
           "-fno-sanitize-recover=all", "-pthread", *SRC, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "cannot find" in r.stderr and "san" in r.stderr:
        pytest.skip(f"sanitizer runtime for {san} not installed")
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               TSAN_OPTIONS="halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok=1" in r.stdout
