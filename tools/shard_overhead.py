"""Fixed cost of a sharded in-process call (dm_plan's shard_overhead_ms): the same small pinned
object through dm_root_buffer on a 1-device context and on G virtual devices with sharding forced
(DEOSS_VIRTUAL_DEVICES + DEOSS_FORCE_SHARDED: a host thread per device, per-device leaf pass and
k-level reduce, the gather of subtree roots, compaction, final levels on device 0).  On one GPU the
gather is a D2D copy instead of RCCL, so the RCCL all-gather's own latency is not in this number.

usage: python tools/shard_overhead.py [--reps 50]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import torch
    from deoss_amd import MerkleContext
    torch.cuda.init()
    length, chunk = 1 << 20, 4096      # 256 leaves: tiny chains, so the fixed costs dominate
    host = torch.randint(0, 255, (length,), dtype=torch.uint8).pin_memory()

    def timed(ctx):
        ctx.root_buffer_ptr(host.data_ptr(), length, chunk)   # warm
        ts = []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            ctx.root_buffer_ptr(host.data_ptr(), length, chunk)
            ts.append((time.perf_counter() - t0) * 1e3)
        return statistics.median(ts)

    res = {"object_bytes": length, "chunk": chunk, "reps": args.reps}
    with MerkleContext() as one:
        res["one_device_ms"] = round(timed(one), 4)
    for G in (2, 4, 8):
        os.environ["DEOSS_VIRTUAL_DEVICES"] = str(G)
        os.environ["DEOSS_FORCE_SHARDED"] = "1"
        try:
            ctx = MerkleContext()
        finally:
            del os.environ["DEOSS_VIRTUAL_DEVICES"], os.environ["DEOSS_FORCE_SHARDED"]
        with ctx:
            ms = timed(ctx)
        res[f"sharded_{G}_ms"] = round(ms, 4)
        res[f"overhead_{G}_ms"] = round(ms - res["one_device_ms"], 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
