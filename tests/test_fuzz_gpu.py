"""Seeded random campaign over the hashing entry points, every leaf kernel, checked against the oracle.

Each case draws an object length (biased to SHA-256 padding edges: 55/56/63/64/119/120 bytes mod
64, whole and ragged chunks, one-leaf objects, 0-byte leaves in chunk lists), a chunk size (multiples of 64 and not, 16 B up to
4 MiB), a leaf kernel (auto / K1 / K1L / K1P / K1Q) and an entry point:
  device      dm_root_device_async at a random byte offset 0..15 (aligned and unaligned loads), leaves too
  pageable    dm_root_buffer from ordinary host memory (striped H2D through the pinned ring)
  pinned      dm_root_buffer from pinned host memory (zero-copy reads)
  chunks      dm_root_chunks over chunks of random lengths (table mode, 0-byte leaves allowed)
  batch       dm_root_batch over several objects, one root each
  stream      dm_stream in random pieces (chunk rounded to a multiple of 16)
Every root (and every leaf digest where the entry point returns them) must equal the C oracle's
restatement of common/hashtree (types.go:19-39, hashtree.go:23-30) and merkletree v0.2.0.  Bit-exact.
"""
import random

import pytest

MODES = ["auto", "wide", "latency", "pair", "quad"]
EDGES = [0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128]


def _len_for(rnd, chunk):
    """An object length near an interesting boundary for this chunk size (at most ~6 MiB)."""
    leaves = rnd.choice([1, 1, 2, 3, 7, 8, 9, 31, 64, 65, 257])
    while leaves * chunk > (6 << 20) and leaves > 1:
        leaves //= 2
    kind = rnd.random()
    if kind < 0.3:
        n = leaves * chunk                                        # whole chunks
    elif kind < 0.7:
        n = (leaves - 1) * chunk + rnd.choice(EDGES[1:] + [chunk - 1, chunk // 2 + 9])
    else:
        n = rnd.randrange(1, leaves * chunk + 1)                  # anywhere
    return max(1, min(n, leaves * chunk))


def _cases(seed, count):
    rnd = random.Random(seed)
    chunk_choices = [16, 64, 100, 448, 1000, 4096, 4095, 4097, 65536, 65600, 1 << 20, (1 << 20) + 48, 3 << 20,
                     4 << 20]
    out = []
    for i in range(count):
        chunk = rnd.choice(chunk_choices)
        entry = rnd.choice(["device", "device", "pageable", "pinned", "chunks", "batch", "stream"])
        out.append({"i": i, "chunk": chunk, "entry": entry, "mode": rnd.choice(MODES),
                    "len": _len_for(rnd, chunk), "seed": rnd.randrange(1 << 30), "off": rnd.randrange(16),
                    "rnd": rnd.randrange(1 << 30)})
    return out


def _check_case(ctx, orc, torch, c):
    chunk, n, entry = c["chunk"], c["len"], c["entry"]
    rnd = random.Random(c["rnd"])
    data = orc.splitmix_bytes(n, c["seed"])
    if entry == "device":
        import numpy as np
        off = c["off"]
        t = torch.zeros(n + 64 + off, dtype=torch.uint8, device="cuda")
        t[off:off + n] = torch.from_numpy(np.frombuffer(data, dtype=np.uint8).copy()).cuda()
        nl = (n + chunk - 1) // chunk
        r = torch.zeros(32, dtype=torch.uint8, device="cuda")
        lv = torch.zeros(nl * 32, dtype=torch.uint8, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        ctx.root_device_async(t.data_ptr() + off, n, chunk, r.data_ptr(), lv.data_ptr(), s)
        torch.cuda.synchronize()
        want_l, want = orc.root_buffer(data, chunk)
        return bytes(lv.cpu().numpy()) == want_l and bytes(r.cpu().numpy()) == want
    if entry == "pageable":
        leaves, root = ctx.root_buffer(data, chunk, want_leaves=True)
        want_l, want = orc.root_buffer(data, chunk)
        return leaves == want_l and root == want
    if entry == "pinned":
        from deoss_amd import PinnedBuffer
        pin = PinnedBuffer(max(n, 1))
        try:
            import numpy as np
            pin.array()[:n] = np.frombuffer(data, dtype=np.uint8)
            leaves, root = ctx.root_buffer_ptr(pin.ptr, n, chunk, want_leaves=True)
        finally:
            pin.free()
        want_l, want = orc.root_buffer(data, chunk)
        return leaves == want_l and root == want
    if entry == "chunks":
        pieces = []
        count = rnd.choice([1, 2, 3, 5, 8, 17, 33])
        for k in range(count):
            m = rnd.choice([0, 1, 55, 56, 64, 119, 4096, chunk, rnd.randrange(0, 2 * chunk + 2)])
            pieces.append(orc.splitmix_bytes(m, c["seed"] + k) if m else b"")
        leaves, root = ctx.root_chunks(pieces)
        want_l, want = orc.root_chunks(pieces)
        return leaves == want_l and root == want
    if entry == "batch":
        objs = [data] + [orc.splitmix_bytes(rnd.randrange(1, max(2, min(n, 1 << 20) + 1)), c["seed"] + k + 1)
                         for k in range(rnd.choice([1, 2, 6, 15]))]
        roots = ctx.root_batch(objs, chunk)
        return roots == [orc.root_buffer(o, chunk)[1] for o in objs]
    if entry == "stream":
        chunk = max(16, chunk // 16 * 16)
        st = ctx.open_stream(chunk)
        pos = 0
        while pos < n:
            m = min(n - pos, rnd.choice([1, 15, 16, 64, 1000, 65536, 1 << 20]))
            st.write(data[pos:pos + m])
            pos += m
        leaves, root = st.close(want_leaves=True)
        want_l, want = orc.root_buffer(data, chunk)
        return leaves == want_l and root == want
    raise AssertionError(entry)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [20251018, 5, 77])
def test_random_entry_points_modes_and_lengths(ctx, oracle_lib, seed):
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    cases = _cases(seed, 200)
    bad = []
    try:
        for c in cases:
            ctx.set_leaf_kernel(c["mode"])
            if not _check_case(ctx, oracle_lib, torch, c):
                bad.append({k: c[k] for k in ("i", "entry", "mode", "chunk", "len", "off")})
    finally:
        ctx.set_leaf_kernel("auto")
    assert not bad, bad


def test_campaign_shape():
    """The campaign covers every entry point and leaf kernel, padding edges and one-leaf objects
    (checked on the CPU: the draw is seeded)."""
    cases = _cases(20251018, 200) + _cases(5, 200) + _cases(77, 200)
    assert {c["entry"] for c in cases} == {"device", "pageable", "pinned", "chunks", "batch", "stream"}
    assert {c["mode"] for c in cases} == set(MODES)
    assert any(c["len"] % 64 in (55, 56) for c in cases) and any(c["len"] <= c["chunk"] for c in cases)
    assert any(c["off"] % 16 for c in cases if c["entry"] == "device")
    assert max(c["len"] for c in cases) <= 8 << 20
