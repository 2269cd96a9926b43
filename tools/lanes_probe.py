"""Concurrent large calls on ONE GPU: do they overlap?  T threads each hash the same host object
through dm_root_buffer on one context whose device list is the box's GPU V times
(DEOSS_VIRTUAL_DEVICES=V: V call lanes, each with its own streams, scratch and lock).  With V = 1
every call holds the device's one lane and the calls run back to back; with V >= T each call gets
its own lane and the leaf chains of different calls can share the chip (an 8 GiB object at 32 MiB
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
    ap.add_argument("--workloads", default="pinned8g,pageable2g,pinned1m")
    args = ap.parse_args()
    import torch
    from deoss_amd import MerkleContext
    torch.cuda.init()
    gib = 1 << 30
    shapes = {   # name -> (bytes, chunk, pinned)
        "pinned8g": (8 * gib, 32 << 20, True),
        "pageable2g": (2 * gib, 32 << 20, False),
        "pinned1m": (1 * gib, 1 << 20, True),
    }
    threads = [int(x) for x in args.threads.split(",")]
    lanes = [int(x) for x in args.lanes.split(",")]
    for name in args.workloads.split(","):
        length, chunk, pinned = shapes[name]
        host = torch.empty(length, dtype=torch.uint8, pin_memory=pinned)
        dev = torch.empty(length, dtype=torch.uint8, device="cuda")
        with MerkleContext() as c0:
            c0.fill_synthetic_async(dev.data_ptr(), 0, length, 0xC0FFEE, 0)
            torch.cuda.synchronize()
            host.copy_(dev)
            del dev
            torch.cuda.empty_cache()
            want = c0.root_buffer_ptr(host.data_ptr(), length, chunk)[1]
        for V in lanes:
            if V > 1:
                os.environ["DEOSS_VIRTUAL_DEVICES"] = str(V)
            try:
                ctx = MerkleContext()
            finally:
                os.environ.pop("DEOSS_VIRTUAL_DEVICES", None)
            with ctx:
                ctx.root_buffer_ptr(host.data_ptr(), length, chunk)   # warm lane 0
                for T in threads:
                    roots = [None] * T
                    ms = [0.0] * T
                    go = threading.Barrier(T + 1)

                    def work(i):
                        go.wait()
                        t0 = time.perf_counter()
                        roots[i] = ctx.root_buffer_ptr(host.data_ptr(), length, chunk)[1]
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


if __name__ == "__main__":
    main()
