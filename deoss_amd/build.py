"""In-tree build of libdeoss_merkle.so for gfx950 (``python -m deoss_amd.build``).

hipcc compiles the kernels and the C-ABI runtime into one shared library next to this file,
so the built .so travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "merkle_capi.hip")
HDRS = sorted(os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc"))
              if f.endswith((".hpp", ".inl", ".h"))) + [os.path.join(ROOT, "include", "deoss_merkle.h")]
OUT = os.path.join(HERE, "libdeoss_merkle.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = "gfx950"


def hipcc_cmd(out: str = OUT, extra=()) -> list:
    return [os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
            "-shared", "-Wall", "-I", os.path.join(ROOT, "include"), "-o", out, SRC,
            "-L", os.path.join(ROCM, "lib"), "-lrccl", "-Wl,-rpath," + os.path.join(ROCM, "lib"), *extra]


def up_to_date(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return False
    t = os.path.getmtime(out)
    return all(os.path.getmtime(p) <= t for p in [SRC, *HDRS])


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and up_to_date():
        return OUT
    cmd = hipcc_cmd()
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
