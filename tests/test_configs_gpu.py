"""BASELINE configs[2], configs[4] and one GPU's share of configs[3] at their full workloads, every
root checked against the CPU oracle (until round 4 these shapes ran only in
bench.py).  The oracle is the checker only; every result comes from libdeoss_merkle.so.

  configs[2]  4,096 x 4 MiB objects resident in HBM, one root each (dm_root_batch_device_async):
              many independent trees of one 4 MiB leaf (chunk 32 MiB), root = SHA256(h || h).
  configs[4]  one GPU's share of 100,000 x 1 MiB host objects: 12,500 x 1 MiB in pinned and in
              pageable host memory through dm_root_batch (the upload regime: host buffers in,
              roots out).
  configs[3]  one GPU's share of the 1 TiB object: 4,096 x 32 MiB leaves (128 GiB) generated in
              HBM at the share's byte offset, reduced 12 levels by dm_subtree_device_async (the
              block root that rank sends in the RCCL all-gather), against the oracle's root of
              the same leaf range regenerated leaf by leaf (or_root_synthetic_at); and the whole
              1 TiB object share by share on one GPU against the full-size fixture.
  configs[1]  the 8 GiB object made ragged at full size (257 / 256 / 255 leaves with short last
              leaves): merkletree's odd-count duplication at the headline's scale, leaves and root.

Reference path: /root/reference/common/hashtree/types.go:19-39 (NewHashTree: one merkletree per
object, types.go:38), hashtree.go:23-30 (leaf = SHA-256 of the chunk)."""
import hashlib
import os

import pytest

pytestmark = pytest.mark.gpu

SEED = 0xDE0550000          # configs k use seed 0xDE0550000 + k
MiB, GiB = 1 << 20, 1 << 30
CHUNK = 32 * MiB


def _torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _threads():
    """The job's CPU share (16 on the GPU box; os.cpu_count() there is the whole machine)."""
    for v in ("OMP_NUM_THREADS", "MAX_JOBS"):
        x = os.environ.get(v, "")
        if x.isdigit() and int(x) > 0:
            return int(x)
    return min(16, os.cpu_count() or 1)


def _need_hbm(torch, nbytes):
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    assert free >= nbytes, f"{free} B of HBM free, the workload needs {nbytes} B"


def test_configs2_4096x4MiB_device_batch(ctx, oracle_lib):
    from concurrent.futures import ThreadPoolExecutor
    torch = _torch()
    nobj, obj = 4096, 4 * MiB
    seed0 = SEED + 2
    _need_hbm(torch, nobj * obj + 4 * GiB)
    buf = torch.empty(nobj * obj, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for j in range(nobj):                                     # object j: splitmix64 stream seed0 + j
        ctx.fill_synthetic_async(buf.data_ptr() + j * obj, 0, obj, seed0 + j, s)
    roots = torch.zeros(32 * nobj, dtype=torch.uint8, device="cuda")
    ctx.root_batch_device_async([buf.data_ptr() + j * obj for j in range(nobj)], [obj] * nobj, CHUNK,
                                roots.data_ptr(), s)
    torch.cuda.synchronize()
    got = bytes(roots.cpu().numpy())
    host = torch.empty(nobj * obj, dtype=torch.uint8, pin_memory=True)
    host.copy_(buf)
    del buf
    torch.cuda.empty_cache()
    hv = host.numpy()
    for j in (0, 1777, nobj - 1):                             # the device generator == the oracle's
        assert bytes(hv[j * obj:(j + 1) * obj]) == oracle_lib.splitmix_bytes(obj, seed0 + j), j
    base = host.data_ptr()
    with ThreadPoolExecutor(_threads()) as ex:
        wants = list(ex.map(lambda j: oracle_lib.root_buffer_ptr(base + j * obj, obj, CHUNK)[1], range(nobj)))
    bad = [j for j in range(nobj) if got[32 * j:32 * j + 32] != wants[j]]
    assert not bad, f"{len(bad)} of {nobj} roots differ, first {bad[:5]}"
    # one object, one leaf: root = SHA256(leaf || leaf) (merkletree v0.2.0's single-leaf rule)
    leaf = hashlib.sha256(bytes(hv[:obj])).digest()
    assert got[:32] == hashlib.sha256(leaf + leaf).digest()


@pytest.mark.parametrize("pinned", [True, False])
def test_configs4_share_12500x1MiB_host_batch(ctx, oracle_lib, pinned):
    """Pinned bodies are read in place by K1Q over PCIe (zero-copy); pageable ones stream through
    the pinned ring with H2D copies overlapped with hashing (configs[4]'s "overlapped H2D")."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    torch = _torch()
    nobj, obj = 12500, MiB                                    # 100,000 / 8 GPUs
    seed0 = SEED + 4
    host = torch.empty(nobj * obj, dtype=torch.uint8, pin_memory=pinned)
    base = host.data_ptr()
    with ThreadPoolExecutor(_threads()) as ex:
        list(ex.map(lambda j: oracle_lib.fill_splitmix_ptr(base + j * obj, 0, obj, seed0 + j), range(nobj)))
    P = (ctypes.c_void_p * nobj)(*[base + j * obj for j in range(nobj)])
    L = (ctypes.c_uint64 * nobj)(*([obj] * nobj))
    out = ctypes.create_string_buffer(32 * nobj)
    ctx._check(ctx._L.dm_root_batch(ctx._h, P, L, nobj, CHUNK, out), "dm_root_batch")
    got = out.raw
    with ThreadPoolExecutor(_threads()) as ex:
        wants = list(ex.map(lambda j: oracle_lib.root_buffer_ptr(base + j * obj, obj, CHUNK)[1], range(nobj)))
    bad = [j for j in range(nobj) if got[32 * j:32 * j + 32] != wants[j]]
    assert not bad, f"{len(bad)} of {nobj} roots differ, first {bad[:5]}"


def test_configs3_share_4096x32MiB_subtree(ctx, oracle_lib):
    """Rank 5 of 8's share of the 1 TiB object: bytes [5 x 128 GiB, 6 x 128 GiB), 4,096 leaves.
    12 levels reduce it to the one block root that rank contributes (2^12 leaves per block), which
    is the merkletree root of those 4,096 leaves (a power of two: no odd-node duplication)."""
    torch = _torch()
    share, rank = 128 * GiB, 5
    off = rank * share
    seed = SEED + 3
    _need_hbm(torch, share + 4 * GiB)
    buf = torch.empty(share + 64, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    ctx.fill_synthetic_async(buf.data_ptr(), off, share, seed, s)
    nodes = torch.zeros(64, dtype=torch.uint8, device="cuda")
    n = ctx.subtree_device_async(buf.data_ptr(), share, CHUNK, 12, nodes.data_ptr(), s)
    torch.cuda.synchronize()
    assert n == 1
    got = bytes(nodes[:32].cpu().numpy())
    probe = bytes(buf[CHUNK - 64:CHUNK + 64].cpu().numpy())   # the generator at the share's offset
    assert probe == oracle_lib.splitmix_bytes(128, seed, off=off + CHUNK - 64)
    del buf
    torch.cuda.empty_cache()
    _, want = oracle_lib.root_synthetic(share, CHUNK, seed, nthreads=_threads(), base=off)
    assert got == want


def test_configs3_full_object_shard_by_shard_on_one_gpu(ctx):
    """The whole 1 TiB configs[3] object on ONE MI355X, as the 8-GPU run computes it, one rank's
    share after another: each 128 GiB share generated in HBM at its byte offset (bench.py's seed,
    the bytes the N = 8 line's configs[3] hashes), 4,096 leaves reduced 12 levels to that rank's
    block root (dm_subtree_device_async), then the 8 block roots finished to the root
    (dm_finish_device_async, what rank 0 does after the RCCL all-gather).  Every block root and
    the root equal the oracle's full-size fixture (tests/golden/config3_root.json, 32,768 leaves
    regenerated leaf by leaf by tests/golden/make_config3_root.py)."""
    import json
    torch = _torch()
    with open(os.path.join(os.path.dirname(__file__), "golden", "config3_root.json")) as f:
        fx = json.load(f)
    share, ranks = 128 * GiB, 8
    assert fx["len"] == ranks * share and fx["chunk"] == CHUNK
    _need_hbm(torch, share + 4 * GiB)
    buf = torch.empty(share + 64, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    nodes = torch.zeros(ranks * 32, dtype=torch.uint8, device="cuda")
    try:
        for r in range(ranks):
            ctx.fill_synthetic_async(buf.data_ptr(), r * share, share, fx["seed"], s)
            n = ctx.subtree_device_async(buf.data_ptr(), share, CHUNK, 12, nodes.data_ptr() + 32 * r, s)
            assert n == 1
        root = torch.zeros(32, dtype=torch.uint8, device="cuda")
        ctx.finish_device_async(nodes.data_ptr(), ranks, False, root.data_ptr(), s)
        torch.cuda.synchronize()
        got = bytes(nodes.cpu().numpy())
        assert [got[32 * r:32 * r + 32].hex() for r in range(ranks)] == fx["shard_roots_k12"]
        assert bytes(root.cpu().numpy()).hex() == fx["root"]
    finally:
        del buf
        torch.cuda.empty_cache()


@pytest.mark.parametrize("length", [8 * GiB + 8, 8 * GiB - 8, 8 * GiB - CHUNK + 4096])
def test_configs1_ragged_full_size(ctx, oracle_lib, length):
    """configs[1]'s 8 GiB object, made ragged at full size: 257 leaves whose last is one 8-byte
    block (the odd leaf duplicated at level 0, then a lone node self-paired up 8 levels), 256
    leaves whose last is 8 bytes short (multi-block leaf ending inside a block), and 255 leaves
    with a 4 KiB last leaf (odd counts at several levels).  Device-generated bytes; the oracle
    regenerates them leaf by leaf (or_root_synthetic); leaf digests checked too."""
    torch = _torch()
    seed = SEED + 1
    _need_hbm(torch, length + 4 * GiB)
    buf = torch.empty(length + 64, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    ctx.fill_synthetic_async(buf.data_ptr(), 0, length, seed, s)
    n = (length + CHUNK - 1) // CHUNK
    root = torch.zeros(32, dtype=torch.uint8, device="cuda")
    lv = torch.zeros(32 * n, dtype=torch.uint8, device="cuda")
    ctx.root_device_async(buf.data_ptr(), length, CHUNK, root.data_ptr(), lv.data_ptr(), s)
    torch.cuda.synchronize()
    got, got_leaves = bytes(root.cpu().numpy()), bytes(lv.cpu().numpy())
    del buf
    torch.cuda.empty_cache()
    leaves, want = oracle_lib.root_synthetic(length, CHUNK, seed, nthreads=_threads(), want_leaves=True)
    assert got_leaves == leaves
    assert got == want, (length, got.hex(), want.hex())


def test_new_hash_tree_257_segment_files(ctx, oracle_lib):
    """The reference's own entry point at the headline's scale, odd: NewHashTree(chunkPath) over
    257 files of 32 MiB (8 GiB + 32 MiB, DeOSS's segment files; types.go:19-39) through
    dm_new_hash_tree (page cache -> pinned stripes -> K1Q, zero-copy), every leaf digest and the
    root against the oracle's regeneration of the same bytes (file i = bytes [i, i + 1) x 32 MiB of
    one splitmix64 stream, so the files' concatenation is one synthetic object)."""
    import shutil
    import tempfile
    import numpy as np
    nfiles, seed = 257, SEED + 1
    need = nfiles * CHUNK + (2 << 30)
    base = "/dev/shm" if os.path.isdir("/dev/shm") and shutil.disk_usage("/dev/shm").free > need else None
    d = tempfile.mkdtemp(prefix="deoss_nht_", dir=base)
    try:
        buf = np.empty(CHUNK, dtype=np.uint8)
        paths = []
        for i in range(nfiles):
            oracle_lib.fill_splitmix_ptr(buf.ctypes.data, i * CHUNK, CHUNK, seed)
            p = os.path.join(d, f"seg{i:04d}")
            buf.tofile(p)
            paths.append(p)
        leaves, root = ctx.new_hash_tree(paths)
        want_leaves, want = oracle_lib.root_synthetic(nfiles * CHUNK, CHUNK, seed, nthreads=_threads(),
                                                      want_leaves=True)
        assert b"".join(leaves) == want_leaves
        assert root == want
    finally:
        shutil.rmtree(d, ignore_errors=True)


def test_stream_upload_full_size_odd(ctx, oracle_lib):
    """Hash while the body arrives (dm_stream) at the headline's scale: an 8 GiB +
    32 MiB + 8 B body (258 leaves of 32 MiB, the last 8 bytes) written in pieces of random sizes
    (1 B .. 8 MiB, as a handler's reads of c.Request.Body return), across the stream's 1 GiB device
    segments and batched leaf launches; every leaf digest and the root against the oracle."""
    import random
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    length, seed = 8 * GiB + CHUNK + 8, SEED + 1
    host = np.empty(length, dtype=np.uint8)
    step = 256 * MiB
    with ThreadPoolExecutor(_threads()) as ex:
        list(ex.map(lambda o: oracle_lib.fill_splitmix_ptr(host.ctypes.data + o, o, min(step, length - o), seed),
                    range(0, length, step)))
    rnd = random.Random(11)
    st = ctx.open_stream(CHUNK)
    pos = 0
    while pos < length:
        n = min(length - pos, rnd.choice([1, 7, 4096, 65536, 1 << 20, 3 << 20, 8 << 20]))
        st.write((host.ctypes.data + pos, n))
        pos += n
    leaves, root = st.close(want_leaves=True)
    want_leaves, want = oracle_lib.root_synthetic(length, CHUNK, seed, nthreads=_threads(), want_leaves=True)
    assert leaves == want_leaves
    assert root == want
