"""CPU checks of the C-ABI boundary: the library loads and exports exactly what the header declares.

No compute calls here (this container has no GPU); the -m gpu tests exercise every entry point.
"""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "deoss_merkle.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dm_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from deoss_amd import build as b
    b.build(verbose=False)
    from deoss_amd import load_library
    return load_library()


def test_header_matches_python_exports():
    from deoss_amd._lib import EXPORTS
    assert header_functions() == sorted(EXPORTS)


def test_library_exports_every_header_symbol(lib):
    for name in header_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "deoss_amd", "libdeoss_merkle.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (dm_[a-z0-9_]+)$", out, flags=re.M))
    assert exported == set(header_functions())
    # the product never links the CPU oracle
    assert " or_" not in out


def test_strerror_messages(lib):
    assert lib.dm_strerror(0) == b"ok"
    assert lib.dm_strerror(-1) == b"Empty data"   # common/hashtree/types.go:21
    assert lib.dm_strerror(-7) == b"no usable GPU"


def test_library_is_gfx950_code_object():
    """The fat binary embeds an amdgcn-amd-amdhsa--gfx950 code object (and nothing else)."""
    data = open(os.path.join(ROOT, "deoss_amd", "libdeoss_merkle.so"), "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", data))
    assert targets == {b"gfx950"}


def test_no_gpu_fails_loudly(lib):
    """Without a visible GPU, dm_create reports DM_ERR_NODEV (no silent CPU path)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    h = ctypes.c_void_p()
    assert lib.dm_create(ctypes.byref(h), None, 0) == -7
    from deoss_amd import DeossMerkleError, MerkleContext
    with pytest.raises(DeossMerkleError):
        MerkleContext()
    # the FullProcessing mirrors (file form and streaming form) fail the same way
    from deoss_amd.process import FullProcessing, Processor
    with pytest.raises(DeossMerkleError):
        Processor()
    info, fid, err = FullProcessing(__file__, "", "/nonexistent-savedir")
    assert info is None and fid == "" and isinstance(err, DeossMerkleError)
    # the download and batch-upload mirrors too (Go: FindFragment, FullProcessingFiles)
    from deoss_amd.process import FindFragment, FullProcessingFiles
    data, err = FindFragment(__file__, "ab" * 32)
    assert data is None and isinstance(err, DeossMerkleError)
    infos, fids, errs = FullProcessingFiles([__file__, ""], "", "/nonexistent-savedir")
    assert infos == [None, None] and fids == ["", ""]
    assert isinstance(errs[0], DeossMerkleError) and errs[1] is None
    h2 = ctypes.c_void_p()
    assert lib.dm_create_lanes(ctypes.byref(h2), None, 0, 2) == -7


def test_pkg_config_file_points_at_this_checkout(lib):
    """build() writes deoss_amd/deoss_merkle.pc for the Go packages' `#cgo pkg-config: deoss_merkle`:
    its include directory holds the header, its library directory the built library, and every
    Go package binds through it (no relative ${SRCDIR} paths that break when the files are copied
    into DeOSS)."""
    pc = os.path.join(ROOT, "deoss_amd", "deoss_merkle.pc")
    vars_ = {}
    fields = {}
    for line in open(pc):
        line = line.strip()
        if "=" in line and ":" not in line.split("=")[0]:
            k, v = line.split("=", 1)
            vars_[k] = v
        elif ":" in line:
            k, v = line.split(":", 1)
            fields[k.strip()] = v.strip()

    def expand(v):
        for _ in range(4):
            for k, x in vars_.items():
                v = v.replace("${" + k + "}", x)
        return v
    inc = expand(fields["Cflags"]).split("-I", 1)[1].split()[0]
    libdir = expand(fields["Libs"]).split("-L", 1)[1].split()[0]
    assert os.path.exists(os.path.join(inc, "deoss_merkle.h"))
    assert os.path.exists(os.path.join(libdir, "libdeoss_merkle.so"))
    assert "-ldeoss_merkle" in fields["Libs"]
    for pkg in ("hashtree/types_hip.go", "process/process_hip.go", "reedsolomon/reedsolomon_hip.go"):
        src = open(os.path.join(ROOT, "go", pkg)).read()
        assert "#cgo pkg-config: deoss_merkle" in src and "${SRCDIR}" not in src, pkg
