"""Sum rocprofv3 FETCH_SIZE / WRITE_SIZE passes of one-step extra workloads into per-step traffic.

Usage: python tools/pmc_extras.py <gpurun_out/<tag>_pmc> <profiles/extras_traffic.json> [tag]

Input: <dir>/<name>/{FETCH_SIZE,WRITE_SIZE}/**/*counter_collection.csv from tools/profile_extras.sh
(each pass one `bench.py --workload ... --warmup 0 --steps 1` run).  Per workload, every kernel
dispatch except the synthetic-data fill (fill_splitmix_kernel), the read probe and torch's own
buffer kernels (at::native, zeroing result tensors) is one step's
work; memory-side bytes = FETCH_SIZE * 1024 * 2 + WRITE_SIZE * 1024 (gfx950 corrections of
/opt/skills/guides/MI355X_MICROARCH.md "HBM": FETCH_SIZE is half the bytes of a 16 B/lane streaming
read, WRITE_SIZE exact for 16 B/lane stores; other access widths are uncalibrated).  The counters
are L2 memory-side requests, so reads of pinned host memory (the zero-copy K1Q paths) are counted
too: for those workloads the bytes crossed PCIe, not HBM.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys

SKIP = ("fill_splitmix_kernel", "read_probe_kernel", "at::native::")   # setup: data, torch buffers


def short(name: str) -> str:
    n = name.split("(")[0].replace("void ", "").strip()
    n = n.split("<")[0]
    return n.split("::")[-1]


def dispatches(path_glob):
    rows = []
    for path in sorted(glob.glob(path_glob, recursive=True)):
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((int(r.get("Dispatch_Id", 0) or 0), r["Kernel_Name"], int(r["Grid_Size"]),
                             float(r["Counter_Value"])))
    rows.sort()
    return rows


def main():
    src, dst = sys.argv[1], sys.argv[2]
    res = {"round": sys.argv[3] if len(sys.argv) > 3 else None,
           "source": f"{src}/<name>/{{FETCH_SIZE,WRITE_SIZE}} (rocprofv3 --pmc, separate passes, one step each)",
           "correction": "bytes = FETCH_SIZE*1024*2 + WRITE_SIZE*1024 (gfx950, 16 B/lane)",
           "scope": "every kernel of one step (warmup 0, steps 1) except the synthetic-data fill",
           "workloads": {}}
    for d in sorted(glob.glob(os.path.join(src, "*"))):
        name = os.path.basename(d)
        fr = dispatches(os.path.join(d, "FETCH_SIZE", "**", "*counter_collection.csv"))
        wr = dispatches(os.path.join(d, "WRITE_SIZE", "**", "*counter_collection.csv"))
        if not fr or not wr:
            continue
        fsum, wsum = {}, {}
        for _, k, g, v in fr:
            if not any(x in k for x in SKIP):
                fsum.setdefault(short(k), [0, 0.0])
                fsum[short(k)][0] += 1
                fsum[short(k)][1] += v * 1024 * 2
        for _, k, g, v in wr:
            if not any(x in k for x in SKIP):
                wsum.setdefault(short(k), [0, 0.0])
                wsum[short(k)][0] += 1
                wsum[short(k)][1] += v * 1024
        kernels = {}
        for k in sorted(set(fsum) | set(wsum)):
            kernels[k] = {"launches": max(fsum.get(k, [0])[0], wsum.get(k, [0])[0]),
                          "read_bytes": fsum.get(k, [0, 0.0])[1], "write_bytes": wsum.get(k, [0, 0.0])[1]}
        total = sum(v["read_bytes"] + v["write_bytes"] for v in kernels.values())
        args = open(os.path.join(d, "args.txt")).read().strip() if os.path.exists(os.path.join(d, "args.txt")) else ""
        res["workloads"][name] = {"bench_args": args, "traffic_bytes_per_step": total, "kernels": kernels}
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v["traffic_bytes_per_step"] for k, v in res["workloads"].items()}, indent=1))


if __name__ == "__main__":
    main()
