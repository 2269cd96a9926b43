"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE counter CSVs into per-launch HBM bytes for K1.

Usage: python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> [out.json]

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md §HBM (gfx950):
  * FETCH_SIZE is in KiB and reports exactly 1/2 of the bytes of a wide (16 B per lane) read
    stream -> bytes = FETCH_SIZE * 1024 * 2.  K1 reads with global_load_dwordx4 (16 B per lane).
    Cross-check in the same run: at 32 MiB chunks K1 reads 8 GiB and FETCH_SIZE is 4.00 GiB.
  * WRITE_SIZE is in KiB and exact for 16-B-per-lane stores (fill kernel: 8 GiB -> 8388608 KiB).
Launches are matched by dispatch order (both passes run the same command).
"""
from __future__ import annotations

import csv
import json
import os
import sys

KERNEL = "leaf_kernel"


def kind(name: str) -> str:
    if "leaf_kernel_quad" in name:
        return "quad"
    if "leaf_kernel_pair" in name:
        return "pair"
    if "leaf_kernel_lat" in name:
        return "latency"
    return "wide"


def rows(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if KERNEL in r["Kernel_Name"]:
                out.append((f'{kind(r["Kernel_Name"])}:{int(r["Grid_Size"])}', float(r["Counter_Value"])))
    return out


def main():
    fetch, write = sys.argv[1], sys.argv[2]
    out_path = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                                  "k1_traffic.json")
    fr, wr = rows(fetch), rows(write)
    by = {}
    for (g, f), (g2, w) in zip(fr, wr):
        assert g == g2, "dispatch order mismatch between the two passes"
        hbm = f * 1024 * 2 + w * 1024
        by.setdefault(str(g), []).append({"fetch_kib_raw": f, "write_kib": w, "hbm_bytes": hbm})
    summary = {}
    for g, lst in by.items():
        summary[g] = {"launches": len(lst), "hbm_bytes_per_launch": sum(x["hbm_bytes"] for x in lst) / len(lst),
                      "fetch_kib_raw_per_launch": sum(x["fetch_kib_raw"] for x in lst) / len(lst),
                      "write_kib_per_launch": sum(x["write_kib"] for x in lst) / len(lst)}
    res = {"source": f"{os.path.basename(fetch)} + {os.path.basename(write)} (rocprofv3 --pmc, separate passes)",
           "kernel": KERNEL, "correction": "bytes = FETCH_SIZE*1024*2 + WRITE_SIZE*1024 (gfx950, 16 B/lane)",
           "by_kernel_grid": summary}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
