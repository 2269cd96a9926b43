"""Shared constants and host helpers of bench.py and bench_workloads.py (no torch, no GPU):
the peaks the rooflines use, the synthetic-data seed, progress lines, the job's CPU share, what
each workload's parity is pinned by."""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_SLOT_PEAK = 256 * 128 * 2.4e9   # 256 CU x 4 SIMD-32 x 2.4 GHz: full-rate int32 lane-slots/s
MAX_CLOCK_HZ = 2.4e9                  # MI355X_MICROARCH.md chip parameters
ISSUE_CYCLES_ONE_WAVE = 4             # one wave alone issues a VALU instruction every 4 cycles (same guide)
SEED = 0xDE0550002               # configs[1] seed (0xDE0550000 + k)
PHASE = ["start"]   # what the run is doing now (stderr progress lines, heartbeat)


def progress(phase: str) -> None:
    """One stderr line per phase (stdout carries only the JSON line), and the heartbeat's label.
    Only rank 0 prints (the other ranks run the same phases)."""
    PHASE[0] = phase
    if os.environ.get("RANK", "0") in ("", "0"):
        print(f"[bench] {time.strftime('%H:%M:%S')} {phase}", file=sys.stderr, flush=True)


def start_heartbeat(period_s: float = 50.0) -> None:
    """A daemon thread that prints the current phase to stderr every period_s: a long default run
    (N = 1: headline, extras, latency) never goes silent for minutes."""
    import threading

    def beat():
        while True:
            time.sleep(period_s)
            if os.environ.get("RANK", "0") in ("", "0"):
                print(f"[bench] {time.strftime('%H:%M:%S')} ... {PHASE[0]}", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()


def env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def host_cpu_facts() -> dict:
    """What the CPU baseline ran on: model, sockets, physical cores, logical CPUs, this process's
    affinity, the cgroup CPU quota and the share the job may use ("report nproc and
    the model").  The GPU box shows the whole machine in os.cpu_count() but allots 16 CPUs per GPU
    (OMP_NUM_THREADS / MAX_JOBS are set to that share there), so worker pools use `share`."""
    model, phys, sockets = None, set(), set()
    try:
        cur = {}
        with open("/proc/cpuinfo") as f:
            for line in list(f) + ["\n"]:
                if not line.strip():
                    if "physical id" in cur:
                        sockets.add(cur["physical id"])
                        phys.add((cur["physical id"], cur.get("core id", cur.get("processor"))))
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                cur[k.strip()] = v.strip()
                if k.strip() == "model name" and model is None:
                    model = v.strip()
    except OSError:
        pass
    logical = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = logical
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(p)
    except (OSError, ValueError):
        pass
    share = affinity
    if quota:
        share = min(share, max(1, int(quota)))
    for var in ("OMP_NUM_THREADS", "MAX_JOBS"):
        v = os.environ.get(var)
        if v and v.isdigit() and int(v) > 0:
            share = min(share, int(v))
            break
    return {"model": model, "sockets": len(sockets) or None, "physical_cores": len(phys) or None,
            "logical_cpus": logical, "affinity_cpus": affinity, "cgroup_cpu_quota": quota, "share": share,
            "share_basis": "min(affinity, cgroup quota, OMP_NUM_THREADS/MAX_JOBS): the CPUs this job may use"}


def cpu_share() -> int:
    """Worker threads for CPU checkers and the parallel baseline: this job's CPU share."""
    return max(1, host_cpu_facts()["share"])


# What each workload's parity is pinned by (state it in every parity block).
PIN_MERKLE = ("reference KAT common/hashtree/hashtree_test.go:20-82 (4 even leaves, each under one block) + NIST "
              "FIPS 180-4; odd leaf counts, n = 1, multi-block and empty leaves are pinned by two restatements of "
              "merkletree v0.2.0 only (module not vendored, go.mod:10)")
PIN_RS = ("klauspost/reedsolomon v1.12.4 TestOneEncode, restated from upstream (module not vendored, go.mod:65); "
          "everything else restatement-pinned")
PIN_PROCESS = ("cess-go-sdk FullProcessing composition: parity-unpinned against the SDK (not vendored, go.mod:8); "
               "its parts are pinned: SHA-256 (NIST), the tree (hashtree_test.go KAT), RS (restated TestOneEncode)")
PIN_PROOFS = "merkletree v0.2.0 GetMerklePath index rule restated (module not vendored); restatement-pinned"


def pinning_for(workload: str, mode: str = "root") -> str:
    if workload in ("process", "fullprocessing", "process_upload") or (workload == "concurrent" and mode == "process"):
        return PIN_PROCESS
    if workload == "rs":
        return PIN_RS
    if workload == "proofs":
        return PIN_PROOFS
    return PIN_MERKLE


def blocks_for(length: int, chunk: int) -> int:
    """Compression blocks of the whole tree: sum ceil((len+9)/64) + 2 x nodes."""
    n = (length + chunk - 1) // chunk
    last = length - (n - 1) * chunk
    leaf_blocks = (n - 1) * ((chunk + 9 + 63) // 64) + (last + 9 + 63) // 64
    nodes, m, levels = 0, n, 0
    while levels == 0 or m > 1:
        m = (m + 1) // 2
        nodes += m
        levels += 1
    return leaf_blocks + 2 * nodes


def _host_mem_available() -> int:
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    return int(line.split()[1]) * 1024
    except (OSError, ValueError, IndexError):
        pass
    return 0


def _fill_host(orc, addr, nbytes, seed, threads):
    """splitmix64 bytes [0, nbytes) of stream `seed` into host memory at addr, `threads` at once."""
    from concurrent.futures import ThreadPoolExecutor
    piece = 256 << 20
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(lambda o: orc.fill_splitmix_ptr(addr + o, o, min(piece, nbytes - o), seed),
                    range(0, nbytes, piece)))


def _pcts(xs):
    """p50 / p99 / min / max (ms) of a list of seconds; p99 by nearest rank (= max below 100 samples)."""
    v = sorted(xs)
    pick = lambda q: v[min(len(v) - 1, max(0, int(-(-q * len(v) // 1)) - 1))]   # noqa: E731
    return {"p50_ms": round(pick(0.50) * 1e3, 3), "p99_ms": round(pick(0.99) * 1e3, 3),
            "min_ms": round(v[0] * 1e3, 3), "max_ms": round(v[-1] * 1e3, 3), "samples": len(v)}
PCIE_PEAK_GBS = 64.0   # PCIe 5.0 x16, one direction, raw (about 55 GB/s measured)


def golden_case(name):
    with open(os.path.join(ROOT, "tests", "golden", "merkle_golden.json")) as f:
        return next(c for c in json.load(f)["cases"] if c["name"] == name)


def root_fixture(length, chunk, seed=SEED):
    """The committed full-size root of the splitmix64 object [0, length) of stream `seed` at `chunk`
    -- tests/golden/merkle_golden.json (configs[0], configs[1]), config3_root.json (configs[3],
    1 TiB) and scale_roots.json (the N > 1 weak objects, the 4 KiB strong leg), each made leaf by
    leaf by the C oracle -- as {"root", "name", "file"}, or None when none is committed.  The N > 1
    legs check their roots against it instead of re-hashing up to 1 TiB on the host inside the
    driver's time limit."""
    gold = os.path.join(ROOT, "tests", "golden")
    found = []
    try:
        with open(os.path.join(gold, "merkle_golden.json")) as f:
            found += [(c, "merkle_golden.json") for c in json.load(f)["cases"]
                      if c.get("kind") == "buffer" and c.get("full_size")]
    except (OSError, ValueError, KeyError):
        pass
    try:
        with open(os.path.join(gold, "config3_root.json")) as f:
            found.append((json.load(f), "config3_root.json"))
    except (OSError, ValueError):
        pass
    try:
        with open(os.path.join(gold, "scale_roots.json")) as f:
            d = json.load(f)
        found += [(dict(r, seed=d["seed"]), "scale_roots.json") for r in d["roots"]]
    except (OSError, ValueError, KeyError):
        pass
    for c, fname in found:
        if c.get("len") == length and c.get("chunk") == chunk and c.get("seed") == seed:
            return {"root": c["root"], "name": c.get("name"), "file": f"tests/golden/{fname}"}
    return None
