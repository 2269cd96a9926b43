"""GPU parity of FullProcessing (dm_process_*) and Merkle proofs (dm_tree_*, dm_merkle_paths*,
dm_verify_paths*) against the CPU restatements.

Bit-exact against oracle/process_oracle.c and the fixtures in tests/golden/process_golden.json
(FullProcessing composition parity-unpinned against the SDK itself: see test_process_oracle.py),
at full segment size (32 MiB segments, 4 + 8 fragments of 8 MiB) through the device-resident form,
and through the Python mirror of FullProcessing(file, cipher, savedir) writing fragment files.
Proofs: every fixture path, tree levels for n = 1..300, batched verification of valid and
tampered proofs, and the hashtree mirror's GetMerklePath / VerifyContent / VerifyTree.
"""
from __future__ import annotations

import hashlib
import json
import os
import random

import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "process_golden.json")


def _torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


@pytest.fixture(scope="module")
def pg():
    with open(GOLDEN) as f:
        return json.load(f)


def _processor(ctx, k=4, m=8, segment=32 << 20):
    from deoss_amd.process import Processor
    return Processor(ctx, k, m, segment)


# ---- FullProcessing ----------------------------------------------------------------------------

def test_process_golden_host(ctx, pg):
    from oracle import splitmix64_bytes
    for c in pg["process"]:
        p = _processor(ctx, c["data"], c["parity"], c["segment"])
        buf = splitmix64_bytes(c["len"], c["seed"])
        seg, frag, fid, frags = p.process_buffer(buf, want_frags=True)
        total = c["data"] + c["parity"]
        nseg = len(c["segment_hashes"])
        assert [seg[32 * i:32 * i + 32].hex() for i in range(nseg)] == c["segment_hashes"]
        assert [[frag[32 * (s * total + j):32 * (s * total + j + 1)].hex() for j in range(total)]
                for s in range(nseg)] == c["fragment_hashes"]
        assert fid.hex() == c["fid"]
        fsz = c["segment"] // c["data"]
        for t in range(nseg * total):   # fragment bytes hash to their names
            assert hashlib.sha256(frags[t * fsz:(t + 1) * fsz]).digest() == frag[32 * t:32 * t + 32]
        p.close()


@pytest.mark.parametrize("nbytes", [1, (32 << 20) - 1, 32 << 20, (32 << 20) + 17, 9 * (32 << 20) + 12345])
def test_process_device_full_segments(ctx, oracle_lib, nbytes):
    """32 MiB segments, 4 + 8 fragments of 8 MiB, device-resident; stale bytes in the padding
    region must be zeroed by the call."""
    torch = _torch()
    p = _processor(ctx)
    seg, k, m = 32 << 20, 4, 8
    nseg = -(-nbytes // seg)
    obj = torch.full((nseg * seg,), 0xA5, dtype=torch.uint8, device="cuda")
    p.ctx.fill_synthetic_async(obj.data_ptr(), 0, nbytes // 8 * 8, 0xDE0552000 + nbytes)
    torch.cuda.synchronize()
    host = obj[:nbytes].cpu().numpy().tobytes()
    parity = torch.empty(nseg * m * (seg // k), dtype=torch.uint8, device="cuda")
    segh = torch.empty(nseg * 32, dtype=torch.uint8, device="cuda")
    fragh = torch.empty(nseg * (k + m) * 32, dtype=torch.uint8, device="cuda")
    fid = torch.empty(32, dtype=torch.uint8, device="cuda")
    p.process_device_async(obj.data_ptr(), nbytes, parity.data_ptr(), segh.data_ptr(), fragh.data_ptr(),
                           fid.data_ptr())
    torch.cuda.synchronize()
    want_seg, want_frag, want_fid, _ = oracle_lib.full_processing(host, seg, k, m, nthreads=8)
    assert segh.cpu().numpy().tobytes() == want_seg
    assert fragh.cpu().numpy().tobytes() == want_frag
    assert fid.cpu().numpy().tobytes() == want_fid
    if nseg * seg > nbytes:
        assert int(obj[nbytes:].sum().item()) == 0
    p.close()


def test_process_errors(ctx):
    from deoss_amd import DeossMerkleError
    p = _processor(ctx, 4, 8, 64)
    with pytest.raises(DeossMerkleError, match="Empty data"):
        p.process_buffer(b"")
    q = _processor(ctx, 4, 8, 100)   # not a multiple of 16 x 4
    with pytest.raises(DeossMerkleError, match="segment size"):
        q.process_buffer(b"x" * 10)
    p.close()
    q.close()


@pytest.mark.parametrize("path,slot,window", [("windows", None, None), ("one_call", None, None),
                                              ("one_call_nostripes", None, None), ("one_call", 8192, 3 * 4096),
                                              ("one_call", 3 * 4096, 4 * 4096), ("one_call", 8192, 6 * 4096),
                                              ("one_call", 2 * 4096, 40 * 4096)])
def test_full_processing_files(ctx, oracle_lib, tmp_path, monkeypatch, path, slot, window):
    """FullProcessing(file, "", savedir): fragment (and segment) files named by their SHA-256 with
    the right bytes, fid = oracle fid.  "windows": the window path (several dm_process_buffer
    calls; the fid then comes from the tree over all segment digests).  "one_call":
    dm_full_processing, also with small pinned slots (slot reuse, parity sets split over slots)
    and small windows (several GPU passes, fid over all segments); no temporary file survives."""
    import deoss_amd.process as proc
    from oracle import splitmix64_bytes
    monkeypatch.setattr(proc, "WINDOW_SEGMENTS", 3)
    if path == "one_call_nostripes":
        monkeypatch.setenv("DEOSS_FP_STRIPES", "0")
        path = "one_call"
    if slot:
        monkeypatch.setenv("DEOSS_FP_SLOT_BYTES", str(slot))
        monkeypatch.setenv("DEOSS_FP_WINDOW_BYTES", str(window))
    p = _processor(ctx, 4, 8, 4096)
    run = p.FullProcessingWindows if path == "windows" else p.FullProcessing
    data = splitmix64_bytes(10 * 4096 + 999, 0xDE0552100)
    f = tmp_path / "object.bin"
    f.write_bytes(data)
    savedir = tmp_path / "cache" / "deeper"
    info, fid, err = run(str(f), "", str(savedir))
    assert err is None
    seg_b, frag_b, want_fid, frags = oracle_lib.full_processing(data, 4096, 4, 8, want_frags=True)
    assert fid == want_fid.hex()
    assert len(info) == 11
    for s, si in enumerate(info):
        assert os.path.basename(si.SegmentHash) == seg_b[32 * s:32 * s + 32].hex()
        padded = data[s * 4096:(s + 1) * 4096]
        assert open(si.SegmentHash, "rb").read() == padded + bytes(4096 - len(padded))
        assert len(si.FragmentHash) == 12
        for j, fp in enumerate(si.FragmentHash):
            t = s * 12 + j
            assert os.path.basename(fp) == frag_b[32 * t:32 * t + 32].hex()
            assert open(fp, "rb").read() == frags[t * 1024:(t + 1) * 1024]
    assert not [n for n in os.listdir(savedir) if n.startswith(".")]
    # errors keep the Go shape: (nil, "", err)
    assert run(str(f), "key", str(savedir))[2] is not None
    empty = tmp_path / "empty.bin"
    empty.write_bytes(b"")
    assert str(run(str(empty), "", str(savedir))[2]) == "Empty data"
    missing = run(str(tmp_path / "missing"), "", str(savedir))[2]
    assert missing is not None
    if path == "one_call":
        assert str(missing) == f"open {tmp_path / 'missing'}: no such file or directory"
        blocker = tmp_path / "not_a_dir"
        blocker.write_bytes(b"x")
        assert run(str(f), "", str(blocker / "sub"))[2] is not None   # savedir under a regular file
    p.close()


@pytest.mark.parametrize("nbytes,stripes", [(1, "1"), (9 * (32 << 20) + 12345, "1"), (9 * (32 << 20) + 12345, "0"),
                                            (4 * (32 << 20), "1"), (5 * (32 << 20) - 64, "1")])
def test_full_processing_one_call_full_segments(ctx, oracle_lib, tmp_path, monkeypatch, nbytes, stripes):
    """dm_full_processing at chain.SegmentSize (32 MiB segments, 4 + 8 fragments of 8 MiB): digests
    and fid = the oracle's, every file on disk hashes to its name.  stripes "1": windows of >= 4
    segments are read in stripes with the segment and data-fragment chains running from the first
    stripe (round 3); "0": the read-then-launch order."""
    from oracle import splitmix64_bytes
    monkeypatch.setenv("DEOSS_FP_STRIPES", stripes)
    p = _processor(ctx)
    data = splitmix64_bytes(nbytes, 0xDE0552200 + nbytes)
    f = tmp_path / "object.bin"
    f.write_bytes(data)
    savedir = tmp_path / "cache"
    segd, fragd, fid = p.full_processing_file(str(f), str(savedir))
    want_seg, want_frag, want_fid, _ = oracle_lib.full_processing(data, 32 << 20, 4, 8, nthreads=8)
    assert (segd, fragd, fid) == (want_seg, want_frag, want_fid)
    names = sorted(os.listdir(savedir))
    assert names == sorted({fragd[32 * t:32 * t + 32].hex() for t in range(len(fragd) // 32)} |
                           {segd[32 * s:32 * s + 32].hex() for s in range(len(segd) // 32)})
    for n in names[:6] + names[-3:]:
        assert hashlib.sha256(open(savedir / n, "rb").read()).hexdigest() == n
    last = segd[-32:].hex()   # the zero-padded last segment's file
    assert hashlib.sha256(open(savedir / last, "rb").read()).hexdigest() == last
    p.close()


@pytest.mark.parametrize("window,slot", [(None, None), (3 * 4096, None), (4096, None), (5 * 4096, 2 * 4096),
                                         (None, 4096)])
def test_fragment_lookup(ctx, oracle_lib, tmp_path, monkeypatch, window, slot):
    """dm_fragment_lookup (the download handler's one fragment, node/fileHandler.go:962-979): every
    probed name is found at the oracle's (segment, index) with the oracle's bytes -- first, middle
    parity, the zero-padded last segment's last fragment --, across window boundaries (one window,
    3-, 5- and 1-segment windows) and pinned-slot reuse (1- and 2-segment slots, 3 slots cycling);
    a repeated segment resolves to its first copy; an unknown name is None; file errors keep Go's
    text; nothing is written next to the file."""
    from oracle import splitmix64_bytes
    if window:
        monkeypatch.setenv("DEOSS_FL_WINDOW_BYTES", str(window))
    if slot:
        monkeypatch.setenv("DEOSS_FP_SLOT_BYTES", str(slot))
    p = _processor(ctx, 4, 8, 4096)
    data = splitmix64_bytes(10 * 4096 + 999, 0xDE0554000)
    data = data[:4096] + data[:4096] + data[4096:]   # segments 0 and 1 identical
    f = tmp_path / "object.bin"
    f.write_bytes(data)
    nseg = (len(data) + 4095) // 4096
    _, frag_b, _, frags = oracle_lib.full_processing(data, 4096, 4, 8, want_frags=True)
    for s, j in [(0, 0), (1, 3), (5, 9), (6, 4), (nseg - 1, 11), (nseg - 1, 0)]:
        t = s * 12 + j
        name = frag_b[32 * t:32 * t + 32].hex()
        got = p.fragment_lookup(str(f), name)
        want_s = 0 if s == 1 else s   # segment 1 repeats segment 0: the first copy wins
        assert got == (want_s, j, frags[t * 1024:(t + 1) * 1024]), (s, j)
        assert p.fragment_lookup(str(f), name, want_bytes=False) == (want_s, j, None)
    assert p.fragment_lookup(str(f), "ab" * 32) is None
    assert sorted(os.listdir(tmp_path)) == ["object.bin"]
    with pytest.raises(Exception, match="no such file or directory"):
        p.fragment_lookup(str(tmp_path / "missing"), "ab" * 32)
    empty = tmp_path / "empty.bin"
    empty.write_bytes(b"")
    with pytest.raises(Exception, match="Empty data"):
        p.fragment_lookup(str(empty), "ab" * 32)
    p.close()


def test_fragment_lookup_full_segments(ctx, oracle_lib, tmp_path, monkeypatch):
    """chain.SegmentSize (32 MiB segments, 8 MiB fragments), 2-segment windows: the last segment's
    last parity fragment and a data fragment of the second window, vs the oracle."""
    from oracle import splitmix64_bytes
    monkeypatch.setenv("DEOSS_FL_WINDOW_BYTES", str(64 << 20))
    p = _processor(ctx)
    data = splitmix64_bytes(5 * (32 << 20) + 12345, 0xDE0554100)
    f = tmp_path / "object.bin"
    f.write_bytes(data)
    _, frag_b, _, frags = oracle_lib.full_processing(data, 32 << 20, 4, 8, want_frags=True, nthreads=8)
    fr = 8 << 20
    for s, j in [(5, 11), (2, 1)]:
        t = s * 12 + j
        assert p.fragment_lookup(str(f), frag_b[32 * t:32 * t + 32].hex()) == (s, j, frags[t * fr:(t + 1) * fr])
    p.close()
    import deoss_amd.process as proc   # the Go-shaped mirror (go/process FindFragment)
    t = 3 * 12 + 7
    assert proc.FindFragment(str(f), frag_b[32 * t:32 * t + 32].hex()) == (frags[t * fr:(t + 1) * fr], None)
    assert proc.FindFragment(str(f), "cd" * 32) == (None, None)
    # names are lower-case hex (node/fileHandler.go:968 compares strings): other spellings find nothing
    assert proc.FindFragment(str(f), "zz") == (None, None)
    assert proc.FindFragment(str(f), frag_b[32 * t:32 * t + 32].hex().upper()) == (None, None)


def test_full_processing_files_batch_upload(oracle_lib, tmp_path):
    """process.FullProcessingFiles (PUT /files, node/filesHandler.go:197-207): 12 files of 1 B ..
    40 MiB (+ one skipped entry and one missing file), all at once: each result equals that
    file's oracle FullProcessing, files on disk hash to their names, errors stay per file."""
    import deoss_amd.process as proc
    from oracle import splitmix64_bytes
    sizes = [1, 4096, 100000, (1 << 20) + 3, 5 << 20, (32 << 20) - 1, 32 << 20, (40 << 20) + 7,
             777, 65536, 3 << 20, 12345]
    paths = []
    for i, n in enumerate(sizes):
        pth = tmp_path / f"f{i}.bin"
        pth.write_bytes(splitmix64_bytes(n, 0xDE0555000 + i))
        paths.append(str(pth))
    paths.insert(3, "")
    paths.append(str(tmp_path / "missing.bin"))
    savedir = str(tmp_path / "cache")
    infos, fids, errs = proc.FullProcessingFiles(paths, "", savedir)
    assert len(infos) == len(fids) == len(errs) == len(paths)
    assert (infos[3], fids[3], errs[3]) == (None, "", None)
    assert errs[-1] is not None and fids[-1] == ""
    for i, pth in enumerate(paths[:-1]):
        if not pth:
            continue
        data = open(pth, "rb").read()
        seg_b, frag_b, fid, _ = oracle_lib.full_processing(data, 32 << 20, 4, 8, nthreads=4)
        assert errs[i] is None and fids[i] == fid.hex(), pth
        nseg = len(seg_b) // 32
        assert [os.path.basename(x.SegmentHash) for x in infos[i]] == [seg_b[32 * s:32 * s + 32].hex() for s in range(nseg)]
        last = infos[i][-1].FragmentHash[-1]
        assert hashlib.sha256(open(last, "rb").read()).hexdigest() == os.path.basename(last)


def test_process_lanes_concurrent(oracle_lib, tmp_path):
    """rs calls on call lanes: one coder on a 3-lane context, 9 threads mixing FullProcessing from
    files (own savedirs), dm_process_buffer, Encode and Reconstruct, each with its lane's own rs
    staging; then two 5-segment files at chain.SegmentSize through dm_full_processing at once
    (striped windows, pooled kits per lane).  Everything vs the oracle."""
    import threading
    from deoss_amd import MerkleContext
    from deoss_amd.process import Processor
    from deoss_amd.reedsolomon import Encoder
    from oracle import splitmix64_bytes
    ctx = MerkleContext(lanes=3)
    p = Processor(ctx, 4, 8, 4096)
    enc = Encoder(ctx, 4, 8)
    errors = []

    def worker(t):
        try:
            for i in range(3):
                data = splitmix64_bytes(7 * 4096 + 131 * (3 * t + i) + 1, 0xDE0553000 + 3 * t + i)
                want_seg, want_frag, want_fid, want_frags = oracle_lib.full_processing(data, 4096, 4, 8, want_frags=True)
                kind = (t + i) % 3
                if kind == 0:
                    f = tmp_path / f"obj_{t}_{i}.bin"
                    f.write_bytes(data)
                    got = p.full_processing_file(str(f), str(tmp_path / f"cache_{t}_{i}"))
                    ok = got == (want_seg, want_frag, want_fid)
                elif kind == 1:
                    seg, frag, fid, frags = p.process_buffer(data)
                    ok = (seg, frag, fid, frags) == (want_seg, want_frag, want_fid, want_frags)
                else:
                    shards = enc.Split(data[:4096 * 2])
                    full = enc.Encode(shards)
                    rebuilt = enc.Reconstruct([None if j in (0, 5, 9, 11) else s for j, s in enumerate(full)])
                    ok = rebuilt == full and enc.Verify(full)
                if not ok:
                    errors.append((t, i, kind))
        except Exception as e:   # reported below
            errors.append((t, repr(e)))

    try:
        th = [threading.Thread(target=worker, args=(t,)) for t in range(9)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert errors == []
        big = Processor(ctx)
        datas = [splitmix64_bytes(5 * (32 << 20) - 77 * (j + 1), 0xDE0553100 + j) for j in range(2)]
        outs = [None, None]

        def fp(j):
            f = tmp_path / f"big_{j}.bin"
            f.write_bytes(datas[j])
            outs[j] = big.full_processing_file(str(f), str(tmp_path / f"bigcache_{j}"))

        th = [threading.Thread(target=fp, args=(j,)) for j in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        for j in range(2):
            want = oracle_lib.full_processing(datas[j], 32 << 20, 4, 8, nthreads=8)[:3]
            assert outs[j] == want, j
        big.close()
    finally:
        enc.close()
        p.close()
        ctx.close()


def _pieces(data, rng, most):
    pos = 0
    while pos < len(data):
        n = min(len(data) - pos, rng.randint(1, most))
        yield data[pos:pos + n]
        pos += n


@pytest.mark.parametrize("slot,batch", [(None, None), (8192, 2), (3 * 4096, 1)])
def test_processing_stream_small(ctx, oracle_lib, tmp_path, monkeypatch, slot, batch):
    """dm_pstream: the body in random pieces -> the same digests, fid and files as the oracle;
    small slots / batches (test hooks) make every chunk its own RS launch and batches of 1-2 chunks
    hash concurrently on the two lanes; no temporary file survives."""
    from oracle import splitmix64_bytes
    if slot:
        monkeypatch.setenv("DEOSS_FP_SLOT_BYTES", str(slot))
        monkeypatch.setenv("DEOSS_PS_BATCH_CHUNKS", str(batch))
    p = _processor(ctx, 4, 8, 4096)
    rng = random.Random(slot or 1)
    for n in (1, 4096, 4097, 23 * 4096 + 555):
        data = splitmix64_bytes(n, 0xDE0552300 + n)
        savedir = tmp_path / f"cache{n}"
        st = p.NewProcessingStream(str(savedir))
        for piece in _pieces(data, rng, 9000):
            st.write(piece)
        info, fid = st.close()
        seg_b, frag_b, want_fid, frags = oracle_lib.full_processing(data, 4096, 4, 8, want_frags=True)
        assert fid == want_fid.hex()
        assert st.segment_digests == seg_b and st.fragment_digests == frag_b
        assert len(info) == -(-n // 4096)
        for s_i, si in enumerate(info):
            padded = data[s_i * 4096:(s_i + 1) * 4096]
            assert open(si.SegmentHash, "rb").read() == padded + bytes(4096 - len(padded))
            for j, fp in enumerate(si.FragmentHash):
                t = s_i * 12 + j
                assert open(fp, "rb").read() == frags[t * 1024:(t + 1) * 1024]
        assert not [x for x in os.listdir(savedir) if x.startswith(".")]
    p.close()


@pytest.mark.parametrize("cap_bufs", [0, 1, 3])
def test_processing_stream_device_cap(ctx, oracle_lib, tmp_path, monkeypatch, cap_bufs):
    """a pstream's HBM must not grow with the body.  Chunk buffers (2 MiB each
    here: 2 segments of 4 KiB + parity, rounded up) are reused once their parity is out and their
    leaf launch has finished; at DEOSS_PS_DEVICE_CAP write blocks (launching the pending batch
    early).  A body of 100 chunks through a cap of 0 (= one buffer), 1 and 3 buffers: peak device
    bytes stay within the cap and the results equal the oracle's."""
    from oracle import splitmix64_bytes
    monkeypatch.setenv("DEOSS_FP_SLOT_BYTES", "8192")
    monkeypatch.setenv("DEOSS_PS_DEVICE_CAP", str(max(1, cap_bufs * (2 << 20))))   # 1 B: below one buffer
    p = _processor(ctx, 4, 8, 4096)
    n = 200 * 4096 - 77
    data = splitmix64_bytes(n, 0xDE0552350 + cap_bufs)
    st = p.NewProcessingStream(str(tmp_path / "cap"))
    for piece in _pieces(data, random.Random(cap_bufs), 20000):
        st.write(piece)
        cur, peak = st.stats()
        assert cur <= max(cap_bufs, 1) * (2 << 20) and peak <= max(cap_bufs, 1) * (2 << 20)
    info, fid = st.close()
    assert 0 < st.peak_device_bytes <= max(cap_bufs, 1) * (2 << 20)
    seg_b, frag_b, want_fid, _ = oracle_lib.full_processing(data, 4096, 4, 8)
    assert fid == want_fid.hex()
    assert st.segment_digests == seg_b and st.fragment_digests == frag_b
    assert len(info) == 200
    assert not [x for x in os.listdir(tmp_path / "cap") if x.startswith(".")]
    p.close()


def test_processing_stream_full_segments_and_errors(ctx, oracle_lib, tmp_path):
    """32 MiB segments through dm_pstream in 1 B .. 3 MiB pieces = dm_full_processing on the same
    file = the oracle; two streams at once on one coder; empty and aborted streams leave nothing."""
    import threading
    from deoss_amd import DeossMerkleError
    from oracle import splitmix64_bytes
    p = _processor(ctx)
    n = 9 * (32 << 20) + 12345
    data = splitmix64_bytes(n, 0xDE0552400)
    want_seg, want_frag, want_fid, _ = oracle_lib.full_processing(data, 32 << 20, 4, 8, nthreads=8)
    results = {}

    def upload(tag, seed):
        st = p.NewProcessingStream(str(tmp_path / tag))
        for piece in _pieces(data, random.Random(seed), 3 << 20):
            st.write(piece)
        info, fid = st.close()
        results[tag] = (st.segment_digests, st.fragment_digests, fid, len(info))

    th = [threading.Thread(target=upload, args=(f"u{i}", i)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for tag in ("u0", "u1"):
        assert results[tag] == (want_seg, want_frag, want_fid.hex(), 10)
        names = set(os.listdir(tmp_path / tag))   # equal contents share a name (zero fragments)
        want_names = {want_frag[i:i + 32].hex() for i in range(0, len(want_frag), 32)} | \
                     {want_seg[i:i + 32].hex() for i in range(0, len(want_seg), 32)}
        assert names == want_names
    f = tmp_path / "obj.bin"
    f.write_bytes(data)
    assert p.full_processing_file(str(f), str(tmp_path / "file_form"))[2] == want_fid
    empty = p.NewProcessingStream(str(tmp_path / "empty"))
    with pytest.raises(DeossMerkleError, match="Empty data"):
        empty.close()
    aborted = p.NewProcessingStream(str(tmp_path / "aborted"))
    aborted.write(data[:200 << 20])
    aborted.abort()
    assert os.listdir(tmp_path / "aborted") == []
    p.close()


# ---- Merkle proofs -----------------------------------------------------------------------------

def test_proof_golden_paths(ctx, pg):
    for case in pg["proofs"]:
        leaves = b"".join(bytes.fromhex(h) for h in case["leaves"])
        # GetMerklePath(content) answers for the first leaf holding that content (it scans Leafs)
        first = [case["leaves"].index(case["leaves"][p["leaf"]]) for p in case["paths"]]
        got = ctx.merkle_paths(leaves, first)
        assert ctx.tree_root(leaves).hex() == case["root"]
        for (path, bits), p in zip(got, case["paths"]):
            assert [x.hex() for x in path] == p["path"] and bits == p["index"]


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 17, 100, 255, 256, 257, 300, 513, 1025])
def test_tree_levels_match_oracle(ctx, n):
    from oracle import py_level
    rng = random.Random(n)
    leaves = [rng.randbytes(32) for _ in range(n)]
    got = ctx.tree_levels(b"".join(leaves))
    want, lev = [], leaves
    while True:
        lev = py_level(lev)
        want += lev
        if len(lev) == 1:
            break
    assert got == b"".join(want)
    assert ctx.tree_node_count(n) == len(want)


def test_verify_paths_valid_and_tampered(ctx):
    from oracle import py_root_chunks
    rng = random.Random(7)
    chunks = [rng.randbytes(rng.randrange(0, 3000)) for _ in range(333)]
    leaves, root = py_root_chunks(chunks)
    paths = ctx.merkle_paths(b"".join(leaves), list(range(333)))
    contents = list(chunks)
    ok = ctx.verify_paths(contents, [p for p, _ in paths], [b for _, b in paths], [root])
    assert all(ok)
    contents[5] = contents[5] + b"x"
    bad_paths = [list(p) for p, _ in paths]
    bad_paths[9][3] = bytes(32)
    bad_bits = [list(b) for _, b in paths]
    bad_bits[11][0] ^= 1
    bad_bits[12][1] = 2
    ok = ctx.verify_paths(contents, bad_paths, bad_bits, [root])
    assert [i for i, v in enumerate(ok) if not v] == [5, 9, 11, 12]
    # per-proof roots
    ok = ctx.verify_paths(chunks[:3], [p for p, _ in paths[:3]], [b for _, b in paths[:3]],
                          [root, bytes(32), root])
    assert ok == [True, False, True]


def test_proofs_device_large(ctx, oracle_lib):
    """2^17 + 3 leaves of 4 KiB on the device: levels, every path, every proof verified."""
    torch = _torch()
    n, chunk = (1 << 17) + 3, 4096
    obj = torch.empty(n * chunk, dtype=torch.uint8, device="cuda")
    ctx.fill_synthetic_async(obj.data_ptr(), 0, n * chunk, 0xDE0552200)
    leaves = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    root = torch.empty(32, dtype=torch.uint8, device="cuda")
    ctx.root_device_async(obj.data_ptr(), n * chunk, chunk, root.data_ptr(), leaves.data_ptr())
    nodes = torch.empty(ctx.tree_node_count(n) * 32, dtype=torch.uint8, device="cuda")
    ctx.tree_levels_device_async(leaves.data_ptr(), n, nodes.data_ptr())
    depth = ctx.tree_depth(n)
    idx = torch.arange(n, dtype=torch.int64, device="cuda")
    paths = torch.empty(n * depth * 32, dtype=torch.uint8, device="cuda")
    bits = torch.empty(n * depth, dtype=torch.uint8, device="cuda")
    ctx.merkle_paths_device_async(leaves.data_ptr(), nodes.data_ptr(), n, idx.data_ptr(), n, paths.data_ptr(),
                                  bits.data_ptr())
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    base = obj.data_ptr()
    ctx.verify_paths_device_async([base + i * chunk for i in range(n)], [chunk] * n, n, paths.data_ptr(),
                                  bits.data_ptr(), depth, root.data_ptr(), 0, ok.data_ptr())
    torch.cuda.synchronize()
    assert int(ok.sum().item()) == n
    assert nodes[-32:].cpu().numpy().tobytes() == root.cpu().numpy().tobytes()
    host = obj.cpu().numpy().tobytes()
    _, want_root = oracle_lib.root_buffer(host, chunk, nthreads=8)
    assert root.cpu().numpy().tobytes() == want_root
    # one tampered byte fails exactly its own proof
    obj[77 * chunk + 5] ^= 1
    ok.zero_()
    ctx.verify_paths_device_async([base + i * chunk for i in range(n)], [chunk] * n, n, paths.data_ptr(),
                                  bits.data_ptr(), depth, root.data_ptr(), 0, ok.data_ptr())
    torch.cuda.synchronize()
    bad = torch.nonzero(ok == 0).flatten().cpu().tolist()
    assert bad == [77]
    # uniform-layout form (no per-content table) gives the same answers
    ok.fill_(7)
    ctx.verify_object_device_async(obj.data_ptr(), n * chunk, chunk, paths.data_ptr(), bits.data_ptr(), depth,
                                   root.data_ptr(), 0, ok.data_ptr())
    torch.cuda.synchronize()
    assert torch.nonzero(ok != 1).flatten().cpu().tolist() == [77]


@pytest.mark.parametrize("n,chunk,tail", [(1, 64, 0), (2, 64, 1), (3, 4096, 100), (1000, 1000, 7)])
def test_verify_object_ragged(ctx, n, chunk, tail):
    """Uniform form with a short last chunk and odd leaf counts, per-proof roots."""
    torch = _torch()
    from oracle import py_get_merkle_path, py_root_chunks
    length = (n - 1) * chunk + (tail or chunk)
    obj = torch.empty(length + 64, dtype=torch.uint8, device="cuda")
    ctx.fill_synthetic_async(obj.data_ptr(), 0, (length + 7) // 8 * 8, 0xDE0552300 + n)
    host = obj[:length].cpu().numpy().tobytes()
    chunks = [host[i * chunk:(i + 1) * chunk] for i in range(n)]
    leaves, root = py_root_chunks(chunks)
    depth = ctx.tree_depth(n)
    pb, bb = b"", b""
    for i in range(n):
        p, b = py_get_merkle_path(chunks, chunks[i])
        pb += b"".join(p)
        bb += bytes(b)
    paths = torch.frombuffer(bytearray(pb), dtype=torch.uint8).cuda()
    bits = torch.frombuffer(bytearray(bb), dtype=torch.uint8).cuda()
    roots = torch.frombuffer(bytearray(root * n), dtype=torch.uint8).cuda()
    ok = torch.zeros(n, dtype=torch.uint8, device="cuda")
    ctx.verify_object_device_async(obj.data_ptr(), length, chunk, paths.data_ptr(), bits.data_ptr(), depth,
                                   roots.data_ptr(), 32, ok.data_ptr())
    torch.cuda.synchronize()
    assert int(ok.sum().item()) == n


def test_hashtree_mirror_proof_api(ctx, tmp_path):
    from deoss_amd import HashTreeContent, NewHashTree
    from oracle import py_fold_path, py_get_merkle_path
    contents = [b"content_one", b"content_two", b"content_three", b"content_two", b"content_five"]
    paths = []
    for i, c in enumerate(contents):
        p = tmp_path / f"c{i}"
        p.write_bytes(c)
        paths.append(str(p))
    tree, err = NewHashTree(paths, ctx=ctx, keep_content=True)
    assert err is None
    for c in contents:
        path, index, err = tree.GetMerklePath(HashTreeContent(c))
        assert err is None
        assert (path, index) == py_get_merkle_path(contents, c)
        assert py_fold_path(hashlib.sha256(c).digest(), path, index) == tree.MerkleRoot()
        ok, err = tree.VerifyContent(HashTreeContent(c))
        assert ok and err is None
    assert tree.GetMerklePath(HashTreeContent(b"absent")) == (None, None, None)
    assert tree.VerifyContent(HashTreeContent(b"absent")) == (False, None)
    assert tree.VerifyTree() == (True, None)
    tree.Leafs[2].C.x = b"tampered"
    assert tree.VerifyTree() == (False, None)


# ---- batched FullProcessing and the coalescing executor -------------------------------------------

def test_process_batch_matches_oracle(ctx, oracle_lib):
    from oracle import splitmix64_bytes
    p = _processor(ctx, 4, 8, 4096)
    rng = random.Random(11)
    bufs = [splitmix64_bytes(rng.choice([1, 63, 4096, 4097, 9000, 3 * 4096, 50000]), 0xDE0552400 + i)
            for i in range(23)]
    got = p.process_batch(bufs, want_frags=True)
    for b, (seg, frag, fid, frags) in zip(bufs, got):
        ws, wf, wfid, wfr = oracle_lib.full_processing(b, 4096, 4, 8, want_frags=True)
        assert (seg, frag, fid, frags) == (ws, wf, wfid, wfr)
    from deoss_amd import DeossMerkleError
    with pytest.raises(DeossMerkleError, match="Empty data"):
        p.process_batch([b"abc", b""])
    p.close()


def test_batcher_root_concurrent(oracle_lib):
    """64 threads x 4 blocking requests of random size: every root equals the oracle's, and the
    requests were coalesced into fewer launches."""
    import threading
    from deoss_amd.batcher import ROOT, Batcher
    from oracle import splitmix64_bytes
    chunk = 64 << 10
    b = Batcher(ROOT, chunk, device=None, slots=2, linger_us=200)   # every visible GPU
    errors, results = [], {}

    def worker(t):
        rng = random.Random(t)
        try:
            for r in range(4):
                n = rng.choice([1, 100, chunk - 1, chunk, chunk + 1, 3 << 20, (1 << 20) + 7])
                data = splitmix64_bytes(n, 0xDE0552500 + 16 * t + r)
                leaves, root = b.root(data, want_leaves=True)
                results[(t, r)] = (data, leaves, root)
        except Exception as e:   # surfaced below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(64)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    assert len(results) == 256
    for data, leaves, root in results.values():
        wl, wr = oracle_lib.root_buffer(data, chunk)
        assert (leaves, root) == (wl, wr)
    nreq, nbatch, maxb = b.stats()
    assert nreq == 256 and nbatch < nreq and maxb > 1
    b.close()


def test_batcher_process_concurrent(oracle_lib):
    import threading
    from deoss_amd.batcher import PROCESS, Batcher
    from oracle import splitmix64_bytes
    b = Batcher(PROCESS, 4096, 4, 8, device=[0, 0], slots=2, linger_us=100)   # 2 'GPUs' x 2 slots
    errors, results = [], []

    def worker(t):
        try:
            for r in range(3):
                data = splitmix64_bytes(1 + (t * 7919 + r * 104729) % 20000, 0xDE0552600 + 8 * t + r)
                results.append((data, b.process(data, want_frags=True)))
        except Exception as e:
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(24)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    for data, got in results:
        assert got == oracle_lib.full_processing(data, 4096, 4, 8, want_frags=True)
    nreq, nbatch, _ = b.stats()
    assert nreq == 72 and nbatch < nreq
    from deoss_amd import DeossMerkleError
    with pytest.raises(DeossMerkleError, match="Empty data"):
        b.process(b"")
    with pytest.raises(DeossMerkleError):
        b.root(b"x")          # wrong mode
    b.close()


def test_cpp_process_mirror(tmp_path):
    """Compile and run tests/cpp/test_process.cpp: the C++ mirror of the Go process shim
    (include/deoss_process.hpp: FullProcessing over a file, the streaming Writer, Go's errors)."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "test_process")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(root, "include"),
                    os.path.join(root, "tests", "cpp", "test_process.cpp"),
                    "-L", os.path.join(root, "deoss_amd"), "-ldeoss_merkle",
                    "-L", os.path.join(root, "oracle"), "-loracle_merkle",   # the checker's restatement only
                    "-Wl,-rpath," + os.path.join(root, "deoss_amd") + ":" + os.path.join(root, "oracle"),
                    "-lpthread", "-o", exe], check=True)
    r = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "PASS" in r.stdout, r.stdout + r.stderr


def test_processing_stream_write_failure(ctx, tmp_path, monkeypatch):
    """A savedir the process cannot write: the failure surfaces as DM_ERR_IO with the OS message
    from a write or from close, the stream stays failed (nothing more reaches the GPU) and no
    temporary is left.  Needs a non-root user (root writes through mode 0555)."""
    import ctypes
    from deoss_amd import DeossMerkleError
    from oracle import splitmix64_bytes
    if os.geteuid() == 0:
        pytest.skip("root ignores directory permissions")
    monkeypatch.setenv("DEOSS_FP_SLOT_BYTES", "8192")
    p = _processor(ctx, 4, 8, 4096)
    ro = tmp_path / "ro"
    ro.mkdir()
    ro.chmod(0o555)
    data = splitmix64_bytes(40 * 4096, 0xDE0552600)
    L = p.ctx._L
    h = ctypes.c_void_p()
    assert L.dm_pstream_open(p.enc._h, 4096, os.fsencode(str(ro)), 1, ctypes.byref(h)) == 0
    rcs = [L.dm_pstream_write(h, data[i:i + 4096], 4096) for i in range(0, len(data), 4096)]
    failed = [rc for rc in rcs if rc != 0]
    if failed:   # sticky: every write after the first failure returns the same code
        first = rcs.index(failed[0])
        assert all(rc == failed[0] for rc in rcs[first:])
    seg = ctypes.create_string_buffer(32 * 64)
    frag = ctypes.create_string_buffer(32 * 64 * 12)
    fid = ctypes.create_string_buffer(32)
    n = ctypes.c_uint64()
    rc = L.dm_pstream_close(h, seg, frag, 64, ctypes.byref(n), fid)
    assert rc == -6 and "permission denied" in (L.dm_last_error(None) or b"").decode()
    assert os.listdir(ro) == []
    ro.chmod(0o755)
    # the mirror raises on the same failure and the Processor keeps working
    ro.chmod(0o555)
    with pytest.raises(DeossMerkleError, match="permission denied"):
        st = p.NewProcessingStream(str(ro))
        for i in range(0, len(data), 4096):
            st.write(data[i:i + 4096])
        st.close()
    ro.chmod(0o755)
    st = p.NewProcessingStream(str(tmp_path / "ok"))
    st.write(data)
    assert len(st.close()[0]) == 40
    p.close()


def test_skip_segment_files(ctx, oracle_lib, tmp_path, monkeypatch):
    """DEOSS_SKIP_SEGMENT_FILES=1 (Go, C++ and Python shims alike): only fragment files are written,
    digests and fid unchanged; file form and streaming form."""
    from oracle import splitmix64_bytes
    monkeypatch.setenv("DEOSS_SKIP_SEGMENT_FILES", "1")
    p = _processor(ctx, 4, 8, 4096)
    data = splitmix64_bytes(5 * 4096 + 77, 0xDE0552700)
    f = tmp_path / "obj.bin"
    f.write_bytes(data)
    seg_b, frag_b, want_fid, _ = oracle_lib.full_processing(data, 4096, 4, 8)
    frag_names = {frag_b[i:i + 32].hex() for i in range(0, len(frag_b), 32)}
    segd, fragd, fid = p.full_processing_file(str(f), str(tmp_path / "a"))
    assert (segd, fragd, fid) == (seg_b, frag_b, want_fid)
    assert set(os.listdir(tmp_path / "a")) == frag_names
    st = p.NewProcessingStream(str(tmp_path / "b"))
    st.write(data)
    assert st.close()[1] == want_fid.hex()
    assert set(os.listdir(tmp_path / "b")) == frag_names
    p.close()


def test_process_device_bench_scale_cross_paths(ctx, oracle_lib):
    """FullProcessing at the bench workload's scale (`bench.py --workload process`: 8 GiB in HBM =
    256 segments -> 3,328 names + fid), every output cross-checked against independent GPU paths
    (size-independent properties): segment names and fid == the uniform-chunk Merkle tree of the
    object at 32 MiB (K1Q, the headline path); data-fragment names == its leaves at 8 MiB; parity ==
    a standalone rs encode of the object; parity names == the leaves of that parity at 8 MiB.
    Segments 0 and 255 are also checked against the CPU restatement."""
    torch = _torch()
    p = _processor(ctx)
    seg, k, m = 32 << 20, 4, 8
    frag = seg // k
    nseg = 256
    nbytes = nseg * seg
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    assert torch.cuda.mem_get_info()[0] >= 5 * nbytes + (4 << 30)
    obj = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    p.ctx.fill_synthetic_async(obj.data_ptr(), 0, nbytes, 0xDE0559)
    parity = torch.empty(nseg * m * frag, dtype=torch.uint8, device="cuda")
    segh = torch.empty(nseg * 32, dtype=torch.uint8, device="cuda")
    fragh = torch.empty(nseg * (k + m) * 32, dtype=torch.uint8, device="cuda")
    fid = torch.empty(32, dtype=torch.uint8, device="cuda")
    p.process_device_async(obj.data_ptr(), nbytes, parity.data_ptr(), segh.data_ptr(), fragh.data_ptr(),
                           fid.data_ptr())
    torch.cuda.synchronize()
    fh = fragh.view(nseg, k + m, 32)

    def tree(ptr, length, chunk):
        n = length // chunk
        r = torch.zeros(32, dtype=torch.uint8, device="cuda")
        lv = torch.zeros(n * 32, dtype=torch.uint8, device="cuda")
        p.ctx.root_device_async(ptr, length, chunk, r.data_ptr(), lv.data_ptr(), 0)
        torch.cuda.synchronize()
        return r, lv.view(n, 32)

    r32, l32 = tree(obj.data_ptr(), nbytes, seg)
    assert torch.equal(l32, segh.view(nseg, 32)) and torch.equal(r32, fid)
    _, l8 = tree(obj.data_ptr(), nbytes, frag)
    assert torch.equal(l8.view(nseg, k, 32), fh[:, :k])
    par2 = torch.empty_like(parity)
    p.enc.encode_device_async(obj.data_ptr(), seg, par2.data_ptr(), m * frag, frag, nseg, 0)
    torch.cuda.synchronize()
    assert torch.equal(par2, parity)
    del par2
    _, lp = tree(parity.data_ptr(), nseg * m * frag, frag)
    assert torch.equal(lp.view(nseg, m, 32), fh[:, k:])
    for s in (0, nseg - 1):
        host = obj[s * seg:(s + 1) * seg].cpu().numpy().tobytes()
        want_seg, want_frag, _, _ = oracle_lib.full_processing(host, seg, k, m, nthreads=8)
        assert segh[s * 32:(s + 1) * 32].cpu().numpy().tobytes() == want_seg
        assert fh[s].cpu().numpy().tobytes() == want_frag
    p.close()
