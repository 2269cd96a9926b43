"""Per-upload fixed cost of the streaming entry points (dm_stream_*, dm_pstream_*): open, write one
small body, close -- on an idle GPU and while another context keeps the same GPU busy with 32 MiB
leaf chains (~0.5 s each), which is what concurrent handlers see.

Prints one JSON line: median / p90 milliseconds per phase for each case.
usage: python tools/stream_latency.py [--reps 15] [--body-kib 1024]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--body-kib", type=int, default=1024)
    args = ap.parse_args()
    import torch
    from deoss_amd import MerkleContext
    from deoss_amd.process import Processor
    torch.cuda.init()
    body = os.urandom(args.body_kib << 10)
    ctx = MerkleContext()
    busy_ctx = MerkleContext()
    proc = Processor(ctx, 4, 8, 32 << 20)
    obj = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    busy_ctx.fill_synthetic_async(obj.data_ptr(), 0, 1 << 30, 7)
    torch.cuda.synchronize()
    stop = threading.Event()

    def keep_busy():   # 32 leaves of 32 MiB: one ~0.5 s chain per call, back to back
        while not stop.is_set():
            busy_ctx.root_device(obj.data_ptr(), 1 << 30, 32 << 20)

    def one_stream():
        t0 = time.perf_counter()
        st = ctx.open_stream(32 << 20)
        t1 = time.perf_counter()
        st.write(body)
        t2 = time.perf_counter()
        st.close()
        t3 = time.perf_counter()
        return (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3

    def one_pstream(d):
        t0 = time.perf_counter()
        st = proc.NewProcessingStream(d)
        t1 = time.perf_counter()
        st.write(body)
        t2 = time.perf_counter()
        st.close()
        t3 = time.perf_counter()
        return (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3

    def summarize(rows):
        out = {}
        for i, name in enumerate(("open", "write", "close")):
            xs = sorted(r[i] for r in rows)
            out[name] = {"median_ms": round(statistics.median(xs), 3), "p90_ms": round(xs[int(0.9 * (len(xs) - 1))], 3)}
        return out

    res = {"body_bytes": len(body), "reps": args.reps}
    with tempfile.TemporaryDirectory(dir="/dev/shm") as d:
        for case in ("idle", "busy"):
            th = None
            if case == "busy":
                stop.clear()
                th = threading.Thread(target=keep_busy)
                th.start()
                time.sleep(0.2)
            one_stream()
            one_pstream(d)   # warm
            res[f"stream_{case}"] = summarize([one_stream() for _ in range(args.reps)])
            res[f"pstream_{case}"] = summarize([one_pstream(d) for _ in range(args.reps)])
            if th:
                stop.set()
                th.join()
    res["library"] = os.environ.get("DEOSS_MERKLE_LIB", "deoss_amd/libdeoss_merkle.so")
    print(json.dumps(res), flush=True)
    proc.close()
    ctx.close()
    busy_ctx.close()


if __name__ == "__main__":
    main()
