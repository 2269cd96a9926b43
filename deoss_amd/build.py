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


PC = os.path.join(HERE, "deoss_merkle.pc")


def write_pkg_config(path: str = PC) -> str:
    """deoss_merkle.pc for the Go bindings' `#cgo pkg-config: deoss_merkle`: the
    include and library directories of THIS checkout, so the go/ packages resolve the library
    wherever they are copied (PKG_CONFIG_PATH=<checkout>/deoss_amd)."""
    text = (f"prefix={ROOT}\n"
            "includedir=${prefix}/include\n"
            "libdir=${prefix}/deoss_amd\n\n"
            "Name: deoss_merkle\n"
            "Description: MI355X-native Merkle content hashing for DeOSS (C ABI include/deoss_merkle.h)\n"
            "Version: 0.3.0\n"
            "Cflags: -I${includedir}\n"
            "Libs: -L${libdir} -ldeoss_merkle -Wl,-rpath,${libdir}\n")
    if not os.path.exists(path) or open(path).read() != text:
        with open(path, "w") as f:
            f.write(text)
    return path


def build(force: bool = False, verbose: bool = True) -> str:
    write_pkg_config()
    if not force and up_to_date():
        return OUT
    cmd = hipcc_cmd()
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
