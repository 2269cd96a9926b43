"""Zero-copy host paths: in auto mode, objects in pinned host memory are hashed in
place by K1Q over PCIe whenever the leaf count is in the latency regime.  No copy to HBM is made.
These tests run every host entry point on pinned memory against the CPU oracle:
- dm_root_buffer, dm_root_chunks and dm_root_batch;
- aligned, misaligned and odd chunk sizes;
- empty chunks, and chunks spread over two pinned allocations;
- memory registered with hipHostRegister, whose device address can differ from the host address;
- the many-leaf (copy) regime next to the zero-copy one.
"""
import ctypes
import mmap

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def auto_ctx(ctx):
    ctx.set_leaf_kernel("auto")
    yield ctx


def _pinned(nbytes, torch):
    return torch.empty(nbytes + 64, dtype=torch.uint8, pin_memory=True)


def _fill(oracle_lib, addr, nbytes, seed):
    oracle_lib.fill_splitmix_ptr(addr, 0, (nbytes + 7) // 8 * 8, seed)


@pytest.mark.parametrize("length,chunk,offset", [
    (300 * (1 << 20) - 12345, 1 << 20, 0),       # 300 leaves, ragged tail
    (3 * (40 << 20) + 7, 40 << 20, 1),           # few long leaves, misaligned base
    ((50 << 20) + 3, 1000003, 16),               # chunk not a multiple of 16 (unaligned kernel)
    (777, 1 << 20, 5),                           # one short leaf
    (20000 * 4096 - 1, 4096, 0),                 # 20,000 leaves: wide regime (copy path)
])
def test_zero_copy_root_buffer(auto_ctx, oracle_lib, length, chunk, offset):
    import torch
    host = _pinned(length + offset, torch)
    addr = host.data_ptr() + offset
    _fill(oracle_lib, addr, length, length ^ chunk)
    want_leaves, want = oracle_lib.root_buffer_ptr(addr, length, chunk, 8, True)
    leaves, root = auto_ctx.root_buffer_ptr(addr, length, chunk, want_leaves=True)
    assert root == want
    assert leaves == want_leaves


def test_zero_copy_root_chunks_two_allocations(auto_ctx, oracle_lib):
    """Chunks alternating between two pinned allocations, some empty, at odd offsets."""
    import torch
    a, b = _pinned(64 << 20, torch), _pinned(64 << 20, torch)
    _fill(oracle_lib, a.data_ptr(), 64 << 20, 1)
    _fill(oracle_lib, b.data_ptr(), 64 << 20, 2)
    ptrs, lens = [], []
    pos = [0, 0]
    sizes = [5 << 20, 0, 3 << 20, 1, (2 << 20) + 13, 0, 4096, 7 << 20, 999999]
    for i, n in enumerate(sizes):
        src = (a, b)[i % 2]
        ptrs.append(src.data_ptr() + pos[i % 2] + (i % 3))
        lens.append(n)
        pos[i % 2] += n + 64
    n = len(sizes)
    P = (ctypes.c_void_p * n)(*ptrs)
    L = (ctypes.c_uint64 * n)(*lens)
    leaf = ctypes.create_string_buffer(32 * n)
    root = ctypes.create_string_buffer(32)
    auto_ctx._check(auto_ctx._L.dm_root_chunks(auto_ctx._h, P, L, n, leaf, root), "dm_root_chunks")
    chunks = [ctypes.string_at(p, m) if m else b"" for p, m in zip(ptrs, lens)]
    from oracle import py_root_chunks
    want_leaves, want = py_root_chunks(chunks)
    assert root.raw == want
    assert leaf.raw == b"".join(want_leaves)


def test_zero_copy_root_batch_multi_leaf(auto_ctx, oracle_lib):
    """Objects of several leaves each (chunk 1 MiB), ragged, from one pinned allocation."""
    import torch
    lens = [(3 << 20) + 5, 1, 1 << 20, (5 << 20) - 1, 4097, 2 << 20]
    offs = [sum((m + 4095) // 4096 * 4096 + 3 for m in lens[:i]) for i in range(len(lens))]
    host = _pinned(offs[-1] + lens[-1] + 64, torch)
    for i, m in enumerate(lens):
        _fill(oracle_lib, host.data_ptr() + offs[i], m, 70 + i)
    n = len(lens)
    P = (ctypes.c_void_p * n)(*[host.data_ptr() + o for o in offs])
    L = (ctypes.c_uint64 * n)(*lens)
    out = ctypes.create_string_buffer(32 * n)
    auto_ctx._check(auto_ctx._L.dm_root_batch(auto_ctx._h, P, L, n, 1 << 20, out), "dm_root_batch")
    for i in range(n):
        assert out.raw[32 * i:32 * i + 32] == oracle_lib.root_buffer_ptr(host.data_ptr() + offs[i], lens[i], 1 << 20)[1], i


def test_zero_copy_registered_memory(auto_ctx, oracle_lib):
    """hipHostRegister'd memory: pinned, with the device address taken from hipHostGetDevicePointer."""
    hip = ctypes.CDLL("libamdhip64.so")
    size = 96 << 20
    m = mmap.mmap(-1, size)
    addr = ctypes.addressof(ctypes.c_char.from_buffer(m))
    _fill(oracle_lib, addr, size, 99)
    assert hip.hipHostRegister(ctypes.c_void_p(addr), ctypes.c_size_t(size), ctypes.c_uint(0)) == 0
    try:
        length, chunk = size - 1000, 3 << 20
        want_leaves, want = oracle_lib.root_buffer_ptr(addr + 8, length, chunk, 8, True)
        leaves, root = auto_ctx.root_buffer_ptr(addr + 8, length, chunk, want_leaves=True)
        assert root == want and leaves == want_leaves
    finally:
        assert hip.hipHostUnregister(ctypes.c_void_p(addr)) == 0
        del m


def test_pageable_memory_still_copies(auto_ctx, oracle_lib):
    """A pageable buffer in the same regime goes through the pinned ring (no device view)."""
    buf = np.frombuffer(oracle_lib.splitmix_bytes((20 << 20) + 3, 17), dtype=np.uint8)
    leaves, root = auto_ctx.root_buffer_ptr(buf.ctypes.data, buf.size, 1 << 20, want_leaves=True)
    want_leaves, want = oracle_lib.root_buffer_ptr(buf.ctypes.data, buf.size, 1 << 20, 4, True)
    assert root == want and leaves == want_leaves


def test_zero_copy_allocation_above_4GiB(auto_ctx, oracle_lib):
    """A pinned allocation of more than 4 GiB, whose HIP range-size query comes back truncated
    (the extent then comes from hipMemPtrGetInfo / the last byte): a window near its end."""
    import torch
    size = (4 << 30) + 4096
    host = torch.empty(size, dtype=torch.uint8, pin_memory=True)
    off, length, chunk = size - (96 << 20) - 3, (96 << 20) - 61, 5 << 20
    addr = host.data_ptr() + off
    _fill(oracle_lib, addr, length, 4242)
    want_leaves, want = oracle_lib.root_buffer_ptr(addr, length, chunk, 8, True)
    leaves, root = auto_ctx.root_buffer_ptr(addr, length, chunk, want_leaves=True)
    assert root == want and leaves == want_leaves


def test_zero_copy_files_striped(auto_ctx, oracle_lib, tmp_path):
    """NewHashTree over files larger than one stripe budget in auto mode: every stripe is hashed
    straight out of the pinned staging slot it was read into (ragged sizes, an empty file)."""
    sizes = [(17 << 20) + 5, 16 << 20, 0, (16 << 20) - 3, 1] + [(15 << 20) + 4096 * i for i in range(14)]
    paths, blobs = [], []
    for i, n in enumerate(sizes):
        data = oracle_lib.splitmix_bytes(n, 900 + i) if n else b""
        p = tmp_path / f"seg{i:02d}"
        p.write_bytes(data)
        paths.append(str(p))
        blobs.append(data)
    assert sum(sizes) > (256 << 20)
    leaves, root = auto_ctx.new_hash_tree(paths)
    from oracle import py_root_chunks
    want_leaves, want = py_root_chunks(blobs)
    assert root == want
    assert leaves == want_leaves


def test_pinned_buffer_api(auto_ctx, oracle_lib):
    """dm_host_alloc / dm_host_free (PinnedBuffer): an object written into it hashes in place."""
    from deoss_amd import DeossMerkleError, PinnedBuffer
    n = (24 << 20) + 99
    pb = PinnedBuffer(n)
    arr = pb.array()
    arr[:] = np.frombuffer(oracle_lib.splitmix_bytes(n, 31), dtype=np.uint8)
    leaves, root = auto_ctx.root_buffer_ptr(pb.ptr, n, 1 << 20, want_leaves=True)
    want_leaves, want = oracle_lib.root_buffer_ptr(pb.ptr, n, 1 << 20, 4, True)
    assert root == want and leaves == want_leaves
    pb.free()
    with pytest.raises(DeossMerkleError):
        PinnedBuffer(0)
