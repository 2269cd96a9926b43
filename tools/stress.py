"""Concurrency stress of the library, every result checked (a diagnosis tool; not product code).

T threads for S seconds, each looping over random operations on a shared context, a shared
batcher and contexts of their own that they create and destroy mid-run:
  pageable / pinned dm_root_buffer, dm_root_chunks, dm_root_batch, a streamed upload in random
  pieces, a device-resident root on the thread's own torch stream, a batcher root, FullProcessing
  (1 MiB segments) on the shared context, from a file, while the body arrives and through a
  PROCESS batcher, a fragment found by name, NewHashTree over chunk files, Reed-Solomon 4 + 8, a
  short-lived
  context (create, one call, destroy), a context destroyed while another thread's calls run on
  the shared one.
Objects come from a fixed pool whose roots the oracle computed up front, so a check is a lookup.
Prints one JSON line: operations per kind, failures (first few with their error), wall time.
usage: python tools/stress.py [threads=24] [seconds=60]
"""
from __future__ import annotations

import json
import os
import random
import shutil
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    S = float(sys.argv[2]) if len(sys.argv) > 2 else 60.0
    import numpy as np
    import torch
    from oracle import Oracle
    from deoss_amd import MerkleContext, PinnedBuffer
    from deoss_amd.batcher import PROCESS as B_PROCESS, ROOT as B_ROOT, Batcher
    from deoss_amd.process import Processor
    assert torch.cuda.is_available()
    orc = Oracle()
    rnd = random.Random(1)
    CH = [4096, 65536, 1 << 20]
    SEG = 1 << 20
    pool = []
    for i in range(24):   # objects of 1 B .. 24 MiB, roots per chunk size up front
        n = rnd.choice([1, 63, 64, 4097, 100_000, 1 << 20, (3 << 20) + 5, 9 << 20, (24 << 20) - 3])
        data = orc.splitmix_bytes(n, 500 + i)
        want = {c: orc.root_buffer(data, c, nthreads=8)[1] for c in CH}
        _, fr, want["fid"], _ = orc.full_processing(data, SEG, nthreads=8)   # FullProcessing at 1 MiB segments
        want["frags"] = fr
        pool.append((data, want))
    big = max(len(d) for d, _ in pool)
    pin = PinnedBuffer(big * 2)
    pin_lock = threading.Lock()
    shared = MerkleContext()
    batcher = Batcher(B_ROOT, 65536, linger_us=500)
    pbatcher = Batcher(B_PROCESS, SEG, linger_us=500)
    proc = Processor(shared, 4, 8, SEG)
    from deoss_amd.reedsolomon import New as rs_new
    rse = rs_new(shared, 4, 8)
    counts, fails = {}, []
    mu = threading.Lock()
    stop_at = time.perf_counter() + S

    def note(kind, ok, err=None):
        with mu:
            counts[kind] = counts.get(kind, 0) + 1
            if not ok and len(fails) < 20:
                fails.append({"op": kind, "error": err})
            elif not ok:
                fails.append(None)

    def worker(t):
        r = random.Random(100 + t)
        tmp = tempfile.mkdtemp(prefix=f"stress{t}_")
        stream = torch.cuda.Stream()
        own = None
        while time.perf_counter() < stop_at:
            data, roots = r.choice(pool)
            c = r.choice(CH)
            want = roots[c]
            op = r.choice(["pageable", "pinned", "chunks", "batch", "stream", "device", "batcher", "short_ctx",
                           "own_ctx", "process", "process_batcher", "files", "fullproc_file", "pstream", "lookup",
                           "rs"])
            try:
                if op == "pageable":
                    got = shared.root_buffer(data, c, want_leaves=False)[1]
                elif op == "pinned":
                    with pin_lock:   # one writer of the pinned region at a time; the hash reads it
                        pin.array()[:len(data)] = np.frombuffer(data, dtype=np.uint8)
                        got = shared.root_buffer_ptr(pin.ptr, len(data), c)[1]
                elif op == "chunks":
                    got = shared.root_chunks([data[o:o + c] for o in range(0, len(data), c)])[1]
                elif op == "batch":
                    d2, r2 = r.choice(pool)
                    rs = shared.root_batch([data, d2], c)
                    got = rs[0] if rs[1] == r2[c] else b"mismatch"
                elif op == "stream":
                    st = shared.open_stream(c)
                    pos = 0
                    while pos < len(data):
                        k = r.choice([1, 1000, 65536, 1 << 20])
                        st.write(data[pos:pos + k])
                        pos += k
                    got = st.close()[1]
                elif op == "device":
                    with torch.cuda.stream(stream):
                        buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda", non_blocking=False)
                        out = torch.zeros(32, dtype=torch.uint8, device="cuda")
                        shared.root_device_async(buf.data_ptr(), len(data), c, out.data_ptr(), 0, stream.cuda_stream)
                        stream.synchronize()
                        got = bytes(out.cpu().numpy())
                elif op == "batcher":
                    c = 65536
                    want = roots[c]
                    got = batcher.root(data)[1]
                elif op == "process":   # FullProcessing on the shared context (RS + leaf launch + fid)
                    want = roots["fid"]
                    got = proc.process_buffer(data, want_frags=False)[2]
                elif op == "process_batcher":
                    want = roots["fid"]
                    got = pbatcher.process(data)[2]
                elif op == "files":      # NewHashTree over chunk files
                    c = 1 << 20
                    want = roots[c]
                    paths = []
                    for j, o in enumerate(range(0, len(data), c)):
                        paths.append(os.path.join(tmp, f"c{j}"))
                        with open(paths[-1], "wb") as f:
                            f.write(data[o:o + c])
                    got = shared.new_hash_tree(paths)[1]
                elif op in ("fullproc_file", "lookup"):
                    want = roots["fid"] if op == "fullproc_file" else True
                    src = os.path.join(tmp, "obj")
                    with open(src, "wb") as f:
                        f.write(data)
                    if op == "fullproc_file":
                        got = proc.full_processing_file(src, tmp, segment_files=False)[2]
                        for name in os.listdir(tmp):
                            if len(name) == 64:
                                os.unlink(os.path.join(tmp, name))
                    else:   # the download path: one fragment found by name, nothing written
                        frs = roots["frags"]
                        t_ = r.randrange(len(frs) // 32)
                        hit = proc.fragment_lookup(src, frs[32 * t_:32 * t_ + 32].hex(), want_bytes=False)
                        h_ = hit[0] * 12 + hit[1] if hit is not None else -1   # equal names: the first match
                        got = h_ >= 0 and frs[32 * h_:32 * h_ + 32] == frs[32 * t_:32 * t_ + 32]
                elif op == "pstream":    # FullProcessing while the body arrives
                    want = roots["fid"]
                    ps = proc.NewProcessingStream(tmp, segment_files=False)
                    pos = 0
                    while pos < len(data):
                        k = r.choice([1000, 65536, 1 << 20, 3 << 20])
                        ps.write(data[pos:pos + k])
                        pos += k
                    got = ps.close()[1]
                    got = bytes.fromhex(got)
                    for name in os.listdir(tmp):
                        if len(name) == 64:
                            os.unlink(os.path.join(tmp, name))
                elif op == "rs":         # Reed-Solomon 4 + 8 of four random-length shards
                    sz = r.choice([16, 4096, 65536, 1 << 20])
                    shards = [data[:sz].ljust(sz, b"\0")] + [orc.splitmix_bytes(sz, 77 + j) for j in range(3)]
                    want = orc.rs_encode(shards, 8)
                    got = rse.Encode(shards + [bytes(sz)] * 8)[4:]
                elif op == "short_ctx":
                    with MerkleContext(lanes=1) as x:
                        got = x.root_buffer(data, c, want_leaves=False)[1]
                else:   # own_ctx: keep one for a while, drop it at random
                    if own is None:
                        own = MerkleContext(lanes=r.choice([1, 2]))
                    got = own.root_buffer(data, c, want_leaves=False)[1]
                    if r.random() < 0.3:
                        own.close()
                        own = None
                note(op, got == want, None if got == want else "wrong root")
            except Exception as e:   # counted and reported, the run goes on
                note(op, False, f"{type(e).__name__}: {e}")
        if own is not None:
            own.close()
        shutil.rmtree(tmp, ignore_errors=True)

    t0 = time.perf_counter()
    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    last = time.perf_counter()
    while any(x.is_alive() for x in th):
        time.sleep(1)
        if time.perf_counter() - last > 20:
            last = time.perf_counter()
            with mu:
                print(f"[stress] {round(last - t0)} s, {sum(counts.values())} ops, {len(fails)} failures",
                      file=sys.stderr, flush=True)
    for x in th:
        x.join()
    wall = time.perf_counter() - t0
    batcher.close()
    pbatcher.close()
    proc.close()
    rse.close()
    shared.close()
    pin.free()
    print(json.dumps({"threads": T, "seconds": round(wall, 1), "ops": sum(counts.values()), "by_op": counts,
                      "failures": len(fails), "first_failures": [f for f in fails if f][:10]}), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
