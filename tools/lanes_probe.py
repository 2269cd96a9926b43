"""Concurrent large calls on ONE GPU: do they overlap?  T threads each hash the same object (host
memory through dm_root_buffer, or device memory through dm_root_device_async on the thread's own
stream) on one context with V call lanes (dm_create_lanes: each lane its own streams, scratch and
lock).  With V = 1 every call holds the GPU's one lane and the calls run back to back; with V >= T
each call gets its own lane and the leaf chains of different calls can share the chip (an 8 GiB object at 32 MiB
chunks uses 32 of the 256 CUs).  Prints one JSON line per (workload, V, T) with the wall time of
all T calls and whether every root matched the single-call root.

usage: python tools/lanes_probe.py [--threads 1,2,4] [--lanes 1,2,4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="1,2,4")
    ap.add_argument("--lanes", default="1,2,4")
    ap.add_argument("--workloads", default="device8g,pinned8g,pageable2g,pinned1m")
    ap.add_argument("--fp-gib", type=float, default=1.0, help="FullProcessing file size (0: skip)")
    args = ap.parse_args()
    import torch
    from deoss_amd import MerkleContext
    torch.cuda.init()
    gib = 1 << 30
    shapes = {   # name -> (bytes, chunk, pinned); pinned None: device-resident (each thread its own stream)
        "device8g": (8 * gib, 32 << 20, None),
        "pinned8g": (8 * gib, 32 << 20, True),
        "pageable2g": (2 * gib, 32 << 20, False),
        "pinned1m": (1 * gib, 1 << 20, True),
    }
    threads = [int(x) for x in args.threads.split(",")]
    lanes = [int(x) for x in args.lanes.split(",")]
    for name in filter(None, args.workloads.split(",")):
        length, chunk, pinned = shapes[name]
        dev = torch.empty(length, dtype=torch.uint8, device="cuda")
        with MerkleContext() as c0:
            c0.fill_synthetic_async(dev.data_ptr(), 0, length, 0xC0FFEE, 0)
            torch.cuda.synchronize()
            if pinned is None:
                host = dev
                r0 = torch.zeros(32, dtype=torch.uint8, device="cuda")
                c0.root_device_async(dev.data_ptr(), length, chunk, r0.data_ptr(), 0, 0)
                torch.cuda.synchronize()
                want = bytes(r0.cpu().numpy())
            else:
                host = torch.empty(length, dtype=torch.uint8, pin_memory=pinned)
                host.copy_(dev)
                del dev
                torch.cuda.empty_cache()
                want = c0.root_buffer_ptr(host.data_ptr(), length, chunk)[1]
        streams = [torch.cuda.Stream() for _ in range(max(threads))]
        roots_dev = torch.zeros(32 * max(threads), dtype=torch.uint8, device="cuda")

        def one_call(c, i):
            if pinned is not None:
                return c.root_buffer_ptr(host.data_ptr(), length, chunk)[1]
            c.root_device_async(host.data_ptr(), length, chunk, roots_dev.data_ptr() + 32 * i, 0,
                                streams[i].cuda_stream)
            streams[i].synchronize()
            return bytes(roots_dev[32 * i:32 * i + 32].cpu().numpy())
        for V in lanes:
            ctx = MerkleContext(lanes=V)
            with ctx:
                one_call(ctx, 0)   # warm lane 0
                for T in threads:
                    roots = [None] * T
                    ms = [0.0] * T
                    go = threading.Barrier(T + 1)

                    def work(i):
                        go.wait()
                        t0 = time.perf_counter()
                        roots[i] = one_call(ctx, i)
                        ms[i] = (time.perf_counter() - t0) * 1e3

                    for _rep in range(2):   # the first round grows every lane's scratch
                        th = [threading.Thread(target=work, args=(i,)) for i in range(T)]
                        for t in th:
                            t.start()
                        go.wait()
                        t0 = time.perf_counter()
                        for t in th:
                            t.join()
                        wall = (time.perf_counter() - t0) * 1e3
                    print(json.dumps({"workload": name, "bytes": length, "chunk": chunk, "pinned": pinned,
                                      "lanes": V, "threads": T, "wall_ms": round(wall, 1),
                                      "per_call_ms": [round(x, 1) for x in ms],
                                      "GiBps": round(T * length / gib / (wall / 1e3), 3),
                                      "roots_match": all(r == want for r in roots)}), flush=True)
        del host
    if args.fp_gib:
        full_processing(args, torch, threads, lanes)


def full_processing(args, torch, threads, lanes):
    """T threads each run dm_full_processing on their own file (own savedir) through one coder on
    a context of V lanes: with V = 1 the calls queue on the coder's one lane."""
    import shutil
    import tempfile
    from deoss_amd import MerkleContext
    from deoss_amd.process import Processor
    length = int(args.fp_gib * (1 << 30))
    tmp = tempfile.mkdtemp(prefix="lanes_fp_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        T = max(threads)
        with MerkleContext() as c0:
            dev = torch.empty(length, dtype=torch.uint8, device="cuda")
            for i in range(T):
                c0.fill_synthetic_async(dev.data_ptr(), 0, length, 0xF00 + i, 0)
                torch.cuda.synchronize()
                with open(os.path.join(tmp, f"in_{i}"), "wb") as f:
                    f.write(dev.cpu().numpy().tobytes())
            del dev
            torch.cuda.empty_cache()
        want = None
        for V in lanes:
            ctx = MerkleContext(lanes=V)
            p = Processor(ctx)
            p.full_processing_file(os.path.join(tmp, "in_0"), os.path.join(tmp, "warm"))
            ref = p.full_processing_file(os.path.join(tmp, "in_0"), os.path.join(tmp, "warm"))[2]
            want = want or ref
            for Tn in threads:
                fids = [None] * Tn
                go = threading.Barrier(Tn + 1)

                def work(i):
                    go.wait()
                    fids[i] = p.full_processing_file(os.path.join(tmp, f"in_{i}"), os.path.join(tmp, f"out_{V}_{Tn}_{i}"))[2]

                th = [threading.Thread(target=work, args=(i,)) for i in range(Tn)]
                for t in th:
                    t.start()
                go.wait()
                t0 = time.perf_counter()
                for t in th:
                    t.join()
                wall = (time.perf_counter() - t0) * 1e3
                for i in range(Tn):
                    shutil.rmtree(os.path.join(tmp, f"out_{V}_{Tn}_{i}"), ignore_errors=True)
                print(json.dumps({"workload": "full_processing_file", "bytes": length, "lanes": V, "threads": Tn,
                                  "wall_ms": round(wall, 1),
                                  "GiBps": round(Tn * length / (1 << 30) / (wall / 1e3), 3),
                                  "fid0_matches": fids[0] == want}), flush=True)
            p.close()
            ctx.close()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
