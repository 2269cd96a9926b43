"""CPU test of the library's host copy pool (deoss_amd/csrc/copy_pool.hpp): tests/cpp/test_copy_pool.cpp
built plain, with ASan/UBSan and with TSan (g++, no GPU) -- concurrent jobs from 8 threads, ragged
and multi-piece items, 0 / 1 / 7 helpers, every byte and guard byte checked."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name,flags", [("plain", ["-O2"]),
                                        ("asan", ["-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer"]),
                                        ("tsan", ["-O1", "-g", "-fsanitize=thread"])])
def test_copy_pool_sanitized(tmp_path, name, flags):
    exe = str(tmp_path / f"test_copy_pool_{name}")
    src = os.path.join(ROOT, "tests", "cpp", "test_copy_pool.cpp")
    inc = os.path.join(ROOT, "deoss_amd", "csrc")
    subprocess.run(["g++", "-std=c++17", *flags, "-I", inc, src, "-o", exe, "-lpthread"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "PASS" in r.stdout
