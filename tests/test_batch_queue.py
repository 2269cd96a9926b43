"""CPU test of the coalescing executor's queue (deoss_amd/csrc/batch_queue.hpp, the dm_batcher
core): tests/cpp/test_batch_queue.cpp with fake workers, built plain and with ASan/UBSan (g++) and
with TSan (ROCm's clang++: g++ 11's TSan does not intercept pthread_cond_clockwait, which
libstdc++ uses for steady-clock waits, and reports every such wait as a double lock).  Checks
exactly-once delivery and budgets under 12 callers x 4 workers, the idle launch after the base
linger, a burst held open while slots are busy, the linger counted from the oldest arrival, and
the drain on stop()."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/llvm/bin/clang++"


@pytest.mark.parametrize("name,cxx,flags", [
    ("plain", "g++", ["-O2"]),
    ("asan", "g++", ["-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer"]),
    ("tsan", CLANG, ["-O1", "-g", "-fsanitize=thread"])])
def test_batch_queue_sanitized(tmp_path, name, cxx, flags):
    if shutil.which(cxx) is None:
        pytest.skip(f"{cxx} not available")
    exe = str(tmp_path / f"test_batch_queue_{name}")
    src = os.path.join(ROOT, "tests", "cpp", "test_batch_queue.cpp")
    inc = os.path.join(ROOT, "deoss_amd", "csrc")
    subprocess.run([cxx, "-std=c++17", *flags, "-I", inc, src, "-o", exe, "-lpthread"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "PASS" in r.stdout
