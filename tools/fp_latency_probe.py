"""Where one small FullProcessing call's time goes (per-request latency).

Times dm_process_buffer on a 1 MiB and a 64 MiB upload with and without the fragments copied
back, with the library's HIP-event timing on (leaf kernel and whole call), and the batch form
(dm_process_batch) of 1 and 16 requests.  usage: python tools/fp_latency_probe.py
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
from deoss_amd import MerkleContext  # noqa: E402
from deoss_amd.process import Processor  # noqa: E402
from oracle import Oracle  # noqa: E402

SEG = 32 << 20


def main():
    orc = Oracle()
    res = {}
    with MerkleContext() as ctx:
        proc = Processor(ctx, 4, 8, SEG)
        for nbytes in (1 << 20, 64 << 20):
            a = np.empty(nbytes, dtype=np.uint8)
            orc.fill_splitmix_ptr(a.ctypes.data, 0, nbytes, 99)
            src = (ctypes.c_char * nbytes).from_address(a.ctypes.data)
            for frags in (True, False):
                proc.process_buffer(src, want_frags=frags)
                ctx.set_timing(True)
                walls = []
                for _ in range(5):
                    t = time.perf_counter()
                    proc.process_buffer(src, want_frags=frags)
                    walls.append((time.perf_counter() - t) * 1e3)
                n, k1, call, mx = ctx.timing_summary()
                ctx.set_timing(False)
                res[f"{nbytes >> 20}MiB_frags{int(frags)}"] = {
                    "wall_ms": [round(x, 1) for x in walls], "leaf_kernel_ms": round(k1 / max(n, 1), 2),
                    "k1_to_call_end_ms": round(call / max(n, 1), 2), "timed": n}
        a = np.empty(16 << 20, dtype=np.uint8)
        orc.fill_splitmix_ptr(a.ctypes.data, 0, a.size, 7)
        for nreq in (1, 16):
            bufs = [bytes(a[i << 20:(i + 1) << 20]) for i in range(nreq)]
            proc.process_batch(bufs)
            ctx.set_timing(True)
            t = time.perf_counter()
            proc.process_batch(bufs)
            w = (time.perf_counter() - t) * 1e3
            n, k1, call, mx = ctx.timing_summary()
            ctx.set_timing(False)
            res[f"batch_{nreq}x1MiB"] = {"wall_ms": round(w, 1), "leaf_kernel_ms": round(k1 / max(n, 1), 2),
                                         "k1_to_call_end_ms": round(call / max(n, 1), 2)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
