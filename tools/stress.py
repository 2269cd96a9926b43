"""Concurrency stress of the library, every result checked (a diagnosis tool; not product code).

T threads for S seconds, each looping over random operations on a shared context, a shared
batcher and contexts of their own that they create and destroy mid-run:
  pageable / pinned dm_root_buffer, dm_root_chunks, dm_root_batch, a streamed upload in random
  pieces, a device-resident root on the thread's own torch stream, a batcher root, FullProcessing
  (1 MiB segments) on the shared context and through a PROCESS batcher, a short-lived
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
import sys
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
        want["fid"] = orc.full_processing(data, SEG, nthreads=8)[2]     # FullProcessing at 1 MiB segments
        pool.append((data, want))
    big = max(len(d) for d, _ in pool)
    pin = PinnedBuffer(big * 2)
    pin_lock = threading.Lock()
    shared = MerkleContext()
    batcher = Batcher(B_ROOT, 65536, linger_us=500)
    pbatcher = Batcher(B_PROCESS, SEG, linger_us=500)
    proc = Processor(shared, 4, 8, SEG)
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
        stream = torch.cuda.Stream()
        own = None
        while time.perf_counter() < stop_at:
            data, roots = r.choice(pool)
            c = r.choice(CH)
            want = roots[c]
            op = r.choice(["pageable", "pinned", "chunks", "batch", "stream", "device", "batcher", "short_ctx",
                           "own_ctx", "process", "process_batcher"])
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
    shared.close()
    pin.free()
    print(json.dumps({"threads": T, "seconds": round(wall, 1), "ops": sum(counts.values()), "by_op": counts,
                      "failures": len(fails), "first_failures": [f for f in fails if f][:10]}), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
