"""Per-step memory-side traffic of the extra workloads from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

Usage: python tools/pmc_extras.py <gpurun_out/<tag>_pmc | profiles/r04/extras_pmc> <out.json> [tag]

Input (tools/profile_extras.sh): <dir>/<name>/s<K>/{FETCH_SIZE,WRITE_SIZE}/**/*counter_collection.csv,
one `bench.py --workload ... --warmup 0 --steps K` run per pass, K = 1 and 2.  One step's traffic
is the MARGINAL step, PMC(K=2) - PMC(K=1), per kernel: the setup (synthetic data, pinned copies of
it) and the parity check after the timed region (the device result and, for some workloads, the
whole object copied back to the host) cancel, and the step counted is a warm one.  A workload with
only one pass (the round-4 layout <dir>/<name>/{FETCH_SIZE,WRITE_SIZE}) falls back to every
dispatch of that run except the synthetic-data fill, the read probe and torch's own kernels, and
says so ("method").  Bytes = FETCH_SIZE * 1024 * 2 + WRITE_SIZE * 1024 (gfx950 corrections of
/opt/skills/guides/MI355X_MICROARCH.md "HBM": FETCH_SIZE is half the bytes of a 16 B/lane streaming
read, WRITE_SIZE exact for 16 B/lane stores; other access widths are uncalibrated).  The counters
are L2 memory-side requests, so reads of pinned host memory (the zero-copy K1Q paths) count too.
"""
from __future__ import annotations

import csv
import glob
import gzip
import json
import os
import sys

SKIP = ("fill_splitmix_kernel", "read_probe_kernel", "at::native::")   # single-pass fallback only


def short(name: str) -> str:
    n = name.split("(")[0].replace("void ", "").strip()
    n = n.split("<")[0]
    return n.split("::")[-1]


def dispatches(path_glob):
    rows = []
    for path in sorted(glob.glob(path_glob, recursive=True) + glob.glob(path_glob + ".gz", recursive=True)):
        with (gzip.open(path, "rt") if path.endswith(".gz") else open(path)) as f:
            for r in csv.DictReader(f):
                rows.append((int(r.get("Dispatch_Id", 0) or 0), r["Kernel_Name"], int(r["Grid_Size"]),
                             float(r["Counter_Value"])))
    rows.sort()
    return rows


def per_kernel(d, skip):
    """{kernel: [launches, read_bytes, write_bytes]} of one run's two passes, or None."""
    fr = dispatches(os.path.join(d, "FETCH_SIZE", "**", "*counter_collection.csv"))
    wr = dispatches(os.path.join(d, "WRITE_SIZE", "**", "*counter_collection.csv"))
    if not fr and not wr:      # the archived layout: <d>/{FETCH_SIZE,WRITE_SIZE}_counter_collection.csv.gz
        fr = dispatches(os.path.join(d, "FETCH_SIZE_counter_collection.csv"))
        wr = dispatches(os.path.join(d, "WRITE_SIZE_counter_collection.csv"))
    if not fr or not wr:
        return None
    out = {}
    for rows, col, scale in ((fr, 1, 2048.0), (wr, 2, 1024.0)):
        n = {}
        for _, k, g, v in rows:
            if skip and any(x in k for x in skip):
                continue
            e = out.setdefault(short(k), [0, 0.0, 0.0])
            e[col] += v * scale
            n[short(k)] = n.get(short(k), 0) + 1
        for k, c in n.items():
            out[k][0] = max(out[k][0], c)
    return out


def total(ks):
    return sum(v[1] + v[2] for v in ks.values())


def main():
    src, dst = sys.argv[1], sys.argv[2]
    res = {"round": sys.argv[3] if len(sys.argv) > 3 else None,
           "source": f"{src}/<name>/s{{1,2}}/{{FETCH_SIZE,WRITE_SIZE}} (rocprofv3 --pmc, separate passes)",
           "correction": "bytes = FETCH_SIZE*1024*2 + WRITE_SIZE*1024 (gfx950, 16 B/lane)",
           "scope": "the marginal step: PMC(--steps 2) - PMC(--steps 1), per kernel, every kernel counted "
                    "(setup and the post-run parity check cancel)",
           "workloads": {}}
    for d in sorted(glob.glob(os.path.join(src, "*"))):
        name = os.path.basename(d)
        if not os.path.isdir(d):
            continue
        args_p = os.path.join(d, "args.txt")
        args = open(args_p).read().strip() if os.path.exists(args_p) else ""
        s1, s2 = per_kernel(os.path.join(d, "s1"), None), per_kernel(os.path.join(d, "s2"), None)
        if s1 is not None and s2 is not None:
            kernels = {}
            for k in sorted(set(s1) | set(s2)):
                a, b = s1.get(k, [0, 0.0, 0.0]), s2.get(k, [0, 0.0, 0.0])
                if b[0] - a[0] == 0 and abs((b[1] + b[2]) - (a[1] + a[2])) < 1 << 20:
                    continue            # not launched by the step (setup / check only)
                kernels[k] = {"launches": b[0] - a[0], "read_bytes": b[1] - a[1], "write_bytes": b[2] - a[2]}
            res["workloads"][name] = {
                "bench_args": args, "method": "marginal step (steps 2 - steps 1)",
                "traffic_bytes_per_step": sum(v["read_bytes"] + v["write_bytes"] for v in kernels.values()),
                "setup_and_check_bytes": total(s1) - (total(s2) - total(s1)), "kernels": kernels}
            continue
        one = per_kernel(d, SKIP)
        if one is None:
            continue
        kernels = {k: {"launches": v[0], "read_bytes": v[1], "write_bytes": v[2]} for k, v in sorted(one.items())}
        res["workloads"][name] = {"bench_args": args, "method": "single run (steps 1), setup kernels skipped by name",
                                  "traffic_bytes_per_step": total(one), "kernels": kernels}
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    with open(dst, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v["traffic_bytes_per_step"] for k, v in res["workloads"].items()}, indent=1))


if __name__ == "__main__":
    main()
