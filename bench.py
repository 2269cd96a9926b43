"""Benchmark: device-resident GiB/s hashed to a Merkle root (BASELINE.json metric), 1..8 MI355X.

One step = one full Merkle root (leaf SHA-256 + tree reduce) over this rank's share of one
synthetic object already resident in HBM.  Weak scaling: every rank holds `--object-gib`
(default 8 GiB = BASELINE configs[1]); at N GPUs the object is N x 8 GiB, sharded by aligned
chunk ranges, with one RCCL all-gather of subtree roots before rank 0's final levels.

Rank 0 prints ONE JSON line on stdout, last, at most LINE_MAX_BYTES (compact_line): the headline,
the K1 roofline (HIP events on the launch stream over the timed region), the CPU baseline (the
oracle's faithful serial restatement of common/hashtree timed on this host over the same bytes),
full-size parity (GPU root == CPU root), the host-buffer end-to-end rate, the strong-scaling leg at
N > 1, and one short entry per extra config; `ok` is false if any check failed.  The full record
(every extra's nested roofline / traffic / CPU legs, latency tables, the in-process leg) goes to the
detail file the line names (--detail-out; default gpurun_out/bench_detail_n<N>.json).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

# Shared helpers and the workloads measured beside the headline; tests and tools reach some of
# them as bench.<name> (re-exports: _pcts, PCIE_PEAK_GBS, EXTRA_ROOF, extras_traffic, extra_roofline,
# cpu_fp_baseline, cpu_root_baseline).
from bench_common import (  # noqa: F401
    ROOT, HBM_PEAK_GBS, VALU_SLOT_PEAK, MAX_CLOCK_HZ, ISSUE_CYCLES_ONE_WAVE, SEED, progress,
    start_heartbeat, env_int, host_cpu_facts, cpu_share, PIN_MERKLE, pinning_for, blocks_for, _pcts,
    PCIE_PEAK_GBS, root_fixture)
from bench_workloads import (  # noqa: F401
    latency_block, in_process_configs, _summary, EXTRA_ROOF, extras_traffic, extra_roofline,
    cpu_fp_baseline, cpu_root_baseline, run_files, run_plumbing, run_upload, run_rs, run_process,
    run_fullprocessing, run_process_upload, run_proofs, run_concurrent, run_batch)


LEAF_GRID = {"wide": (256, 256), "latency": (64, 128), "pair": (32, 128), "quad": (8, 128)}   # leaves, threads per WG


def load_traffic(kind: str, n_leaves: int, alg_bytes: int = 0):
    """PMC HBM bytes per leaf-kernel launch of this kernel and launch shape, from the committed
    rocprofv3 passes (profiles/k1_traffic.json, made by tools/pmc_traffic.py from the same
    bench command).  A launch shape that was not profiled (an N > 1 rank's share, say) takes the
    same kernel's traffic-over-algorithmic ratio at the nearest profiled grid times this launch's
    algorithmic bytes, and says so in the source."""
    path = os.path.join(ROOT, "profiles", "k1_traffic.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    per_wg, threads = LEAF_GRID[kind]
    grid = (n_leaves + per_wg - 1) // per_wg * threads
    key = f"{kind}:{grid}"
    e = d.get("by_kernel_grid", {}).get(key)
    if e:
        return e["hbm_bytes_per_launch"], f"profiles/k1_traffic.json[{key}] <- " + (e.get("round_files") or
                                                                                  d.get("source", ""))
    same = [(abs(int(k.split(":")[1]) - grid), k, v) for k, v in d.get("by_kernel_grid", {}).items()
            if k.split(":")[0] == kind]
    if not same or not alg_bytes:
        return None, None
    _, k2, v = min(same)
    leaves2 = int(k2.split(":")[1]) // threads * per_wg
    alg2 = (8 << 30) + 32 * leaves2          # every profiled grid hashed the 8 GiB headline object
    ratio = v["hbm_bytes_per_launch"] / alg2
    return round(ratio * alg_bytes), (f"profiles/k1_traffic.json[{k2}] ratio {ratio:.5f} x this launch's algorithmic "
                                      f"bytes ({key} not profiled)")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--object-gib", type=float, default=8.0, help="object bytes per GPU (GiB), weak scaling")
    ap.add_argument("--total-gib", type=float, default=0.0,
                    help="object bytes across all ranks (GiB); 1024 at --gpus 8 = BASELINE configs[3] "
                         "(1 TiB, 128 GiB per rank); 0 = --object-gib per GPU")
    ap.add_argument("--multi-configs", action="store_true",
                    help="rehearsal: run the 8-GPU extras (configs[3], configs[4]) at any N > 1")
    ap.add_argument("--cfg3-total-gib", type=float, default=1024.0, help=argparse.SUPPRESS)
    ap.add_argument("--cfg4-objects", type=int, default=100000, help=argparse.SUPPRESS)
    ap.add_argument("--prefix-gib", type=float, default=64.0,
                    help="N>1 parity: sharded root vs single-GPU root of a prefix of at most this size")
    ap.add_argument("--chunk", type=int, default=32 << 20, help="chunk (leaf) bytes; default 32 MiB")
    ap.add_argument("--sweep", action="store_true", help="also run the chunk-size sweep (N=1)")
    ap.add_argument("--no-sweep", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--e2e", action="store_true", help="also time the host-buffer path (N=1)")
    ap.add_argument("--no-e2e", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="N=1 object line: skip the other configs / entry points measured in the same run "
                         "(other_configs), the e2e host-buffer rates and the 64 KiB / 1 MiB sweep points")
    ap.add_argument("--no-verify", action="store_true", help="N>1: skip the single-GPU root check")
    ap.add_argument("--no-aux", action="store_true",
                    help="fullprocessing / process_upload: only the timed flow (the PMC profiling runs)")
    ap.add_argument("--workload", default="object",
                    choices=["object", "batch", "stream", "upload", "rs", "process", "proofs", "concurrent", "files", "fullprocessing", "process_upload",
                             "plumbing", "latency", "inprocess"],
                    help="object: one object per GPU (configs[1]/[3]); batch: many device-resident objects "
                         "(configs[2]); stream: many host-resident objects through the pinned ring (configs[4]); "
                         "upload: one object fed in pieces through dm_stream (hash while receiving); "
                         "files: NewHashTree(chunkPath) over --objects files of --object-mib from the page cache; "
                         "plumbing: BASELINE configs[0], one 64 MiB object at 32 MiB chunks")
    ap.add_argument("--piece-kib", type=int, default=1024, help="upload: bytes per dm_stream_write (KiB)")
    ap.add_argument("--segment-mib", type=int, default=32, help="rs: segment bytes (chain.SegmentSize)")
    ap.add_argument("--objects", type=int, default=4096, help="batch/stream: objects per GPU")
    ap.add_argument("--total-objects", type=int, default=0,
                    help="batch/stream: objects across all ranks, split evenly (100000 x 1 MiB at --gpus 8 = "
                         "BASELINE configs[4]: 12,500 per GPU); 0 = --objects per GPU")
    ap.add_argument("--object-mib", type=float, default=4.0, help="batch/stream: object size (MiB)")
    ap.add_argument("--threads", type=int, default=256, help="concurrent: caller threads")
    ap.add_argument("--mode", default="root", choices=["root", "process"], help="concurrent: request kind")
    ap.add_argument("--slots", type=int, default=0, help="concurrent: batcher worker slots (0 = library default)")
    ap.add_argument("--max-leaves", type=int, default=0, help="concurrent: leaf budget per batch (0 = default)")
    ap.add_argument("--linger-us", type=int, default=2000, help="concurrent: batcher linger after the first request")
    ap.add_argument("--no-shared", action="store_true", help="concurrent: skip the serialised shared-context timing")
    ap.add_argument("--sweep-chunks", default="4096,65536,1048576,8388608,33554432")
    ap.add_argument("--sweep-modes", action="store_true", help="sweep every leaf kernel (wide, latency, pair, quad)")
    ap.add_argument("--leaf-kernel", default="auto", choices=["auto", "wide", "latency", "pair", "quad"])
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (production); gloo = CPU exchange (rehearsal on one GPU)")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank uses cuda:0 (with --dist-backend gloo)")
    ap.add_argument("--in-process", action="store_true",
                    help="N > 1: also run the single-process multi-GPU path (one dm_ctx over every visible GPU, "
                         "ncclCommInitAll + ncclAllGather) from rank 0 after the per-rank legs; always on at N = 8. "
                         "With --same-device, virtual devices stand in for the GPUs (D2D instead of RCCL)")
    ap.add_argument("--inproc-gib", type=float, default=64.0,
                    help="in-process leg: pinned host object (GiB) hashed sharded over every GPU")
    ap.add_argument("--inproc-timeout", type=float, default=420.0,
                    help="in-process leg: seconds before the watchdog gives up on it (the line is printed anyway)")
    ap.add_argument("--inproc-devices", type=int, default=8,
                    help="--workload inprocess on one GPU: virtual devices standing in for the GPUs")
    ap.add_argument("--detail-out", default="",
                    help="where the full record goes (JSON); default gpurun_out/bench_detail_n<N>.json.  stdout's "
                         "last line is the compact headline, which names this file")
    ap.add_argument("--no-strong", action="store_true", help="N > 1: skip the strong-scaling leg")
    ap.add_argument("--deadline-s", type=float, default=DEADLINE_DEFAULT_S,
                    help="wall seconds from the job's start within which every leg after the headline must fit: a "
                         "leg whose estimate exceeds what is left is skipped (named in `problems`); the line is "
                         "printed again after every leg")
    ap.add_argument("--fake-legs", type=float, default=0.0, help=argparse.SUPPRESS)
    ap.add_argument("--fake-line", default="", help=argparse.SUPPRESS)
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--watchdog-check", type=float, default=0.0, help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.gpus > 1 and os.environ.get("WORLD_SIZE") in (None, ""):
        # no launcher: start the rank processes here, before anything touches torch or the GPU
        sys.exit(self_launch(args.gpus, sys.argv[1:]))
    if args.launch_check:
        launch_check(args)
        return
    if args.watchdog_check:
        watchdog_check(args)
        return
    if args.fake_legs:
        fake_legs(args)
        return

    start_heartbeat()
    progress(f"bench.py {' '.join(sys.argv[1:])}")
    import torch
    import torch.distributed as dist
    from deoss_amd import plan_shards

    world = env_int("WORLD_SIZE", 1)
    rank = env_int("RANK", 0)
    local_rank = env_int("LOCAL_RANK", 0)
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dev_index = 0 if args.same_device else local_rank
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    gloo = args.dist_backend == "gloo"
    wait_group = None
    if world > 1:
        if gloo:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
        # host-only group: ranks wait on it while rank 0 runs the in-process leg (no RCCL watchdog)
        import datetime
        wait_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(minutes=45))

    if args.workload == "latency":      # the N = 1 line's latency block alone
        print(json.dumps({"latency": latency_block(args, torch, dev_index)}), flush=True)
        return
    if args.workload == "inprocess":    # the N = 8 line's in-process leg alone (one process)
        ndev = torch.cuda.device_count()
        args.same_device = args.same_device or ndev < 2
        print(json.dumps({"in_process": in_process_configs(args, torch, args.inproc_devices if args.same_device
                                                           else ndev)}), flush=True)
        return
    runners = {"upload": run_upload, "files": run_files, "plumbing": run_plumbing, "rs": run_rs,
               "process": run_process, "proofs": run_proofs, "concurrent": run_concurrent,
               "batch": run_batch, "stream": run_batch, "fullprocessing": run_fullprocessing,
               "process_upload": run_process_upload}
    if args.workload in runners:
        res = runners[args.workload](args, torch, dist, world, rank, device, dev_index, gloo)
        if isinstance(res, dict) and isinstance(res.get("parity"), dict):
            res["parity"]["pinned_by"] = pinning_for(args.workload, args.mode)
        if res is not None and rank == 0:
            print(json.dumps(res), flush=True)
        if world > 1 and dist.is_initialized():
            dist.destroy_process_group()
        return

    def barrier():
        if world > 1:
            if gloo:
                torch.cuda.synchronize()
                dist.barrier()
            else:
                dist.barrier(device_ids=[dev_index])
        torch.cuda.synchronize()

    rank0 = rank == 0
    decide = (lambda mine: mine) if world == 1 else (lambda mine: _bcast_flag(torch, dist, mine, wait_group))
    detail = args.detail_out or os.path.join(ROOT, "gpurun_out", f"bench_detail_n{1 if args.same_device else world}.json")
    progress("headline: timed steps")
    out = run_object(args, torch, dist, world, rank, device, dev_index, gloo, barrier, cpu_leg=not args.no_cpu)
    if isinstance(out.get("parity"), dict):
        out["parity"]["pinned_by"] = PIN_MERKLE
    if world > 1:
        out["launch"] = launch_info(torch, dist, world, rank, local_rank, dev_index, args)
        progress("exchange: the all-gather of subtree roots alone")
        out["exchange"] = measure_exchange(plan_shards(out["config"]["object_bytes"], args.chunk, world), torch,
                                           dist, device, gloo, barrier)
    legs = Legs(out, detail if rank0 else None, args.deadline_s, job_start_time(), decide)
    full = not args.no_extras and not args.total_gib
    if world == 1:
        if rank0 and not args.no_extras:
            from bench_workloads import driver_extra_specs, run_driver_extra
            traffic, tsrc = extras_traffic()
            specs = driver_extra_specs()
            legs.plan([name for name, _, _ in specs] + ["latency"])
            legs.emit()                                       # the headline line, before any extra
            oc = out.setdefault("other_configs", {})
            for name, fn, kw in specs:
                legs.run(name, lambda name=name, fn=fn, kw=kw: oc.__setitem__(
                    name, run_driver_extra(name, fn, kw, args, torch, dist, device, dev_index, traffic, tsrc)))
            legs.run("latency", lambda: out.__setitem__("latency", latency_block(args, torch, dev_index)))
    else:
        names = []
        if not args.total_gib and not args.no_strong:
            names += ["strong_scaling", "strong_scaling_4KiB"]
        if ((world == 8 and not args.same_device) or args.multi_configs) and full:
            names += ["configs[3]", "configs[4]"]
        if (world == 8 or args.in_process) and full:
            names += ["in_process"]
        legs.plan(names)
        legs.emit()                                           # the headline line, before any leg
        weak_per_gpu = out["value"] / world

        def strong(key, chunk):
            r = strong_scaling_leg(args, torch, dist, world, rank, device, dev_index, gloo, barrier, weak_per_gpu,
                                   chunk=chunk)
            out[key] = r

        def in_process():
            inproc, hung = run_in_process_leg(args, torch, dist, world, rank, wait_group, legs)
            if rank0:
                out.setdefault("other_configs", {})["in_process"] = inproc
            if hung:   # the leg is over (killed): the line says so, then every rank leaves with status 3
                legs.pending.remove("in_process")
                out["legs"].update(pending=list(legs.pending))
                out["legs"]["done"]["in_process"] = inproc.get("watchdog_s") if rank0 else None
                exit_after_hang(out if rank0 else None, legs.detail)

        runs = {"strong_scaling": lambda: strong("strong_scaling", 32 << 20),
                "strong_scaling_4KiB": lambda: strong("strong_scaling_4KiB", 4096),
                "configs[3]": lambda: out.setdefault("other_configs", {}).__setitem__(
                    "configs[3]", config3_leg(args, torch, dist, world, rank, device, dev_index, gloo, barrier)),
                "configs[4]": lambda: out.setdefault("other_configs", {}).__setitem__(
                    "configs[4]", config4_leg(args, torch, dist, world, rank, device, dev_index, gloo, barrier)),
                "in_process": in_process}
        for name in names:
            legs.run(name, runs[name])
    if not legs.planned:
        legs.emit()
    if world > 1:
        barrier()
        dist.destroy_process_group()


# Wall seconds each leg after the headline may take at full size.  The N = 8 legs' per-rank work
# was timed on one MI355X as fresh processes (tools/n8_leg_times.sh, profiles/r06/n8_legs: the
# 64 GiB single-GPU parity root 4.2 s, configs[1] at 4 KiB 2.3 s, configs[3]'s 128 GiB share
# 4.2 s, configs[4]'s 12,500-object share 5.8 s, the in-process leg over 8 virtual devices and a
# 64 GiB pinned object 27.8 s); each estimate is ~4x that, for a first RCCL init over 8 GPUs and
# 8 ranks pinning host memory at once.  N = 1's extras were timed in the round-6
# default run (profiles/r06/r06a_bench.log: 159 s in all).  A leg starts only when its estimate
# fits in what is left of --deadline-s.
LEG_ESTIMATE_S = {
    "strong_scaling": 20.0, "strong_scaling_4KiB": 20.0, "configs[3]": 45.0, "configs[4]": 45.0,
    "in_process": 120.0, "latency": 120.0, "FullProcessing_file": 45.0, "FullProcessing_while_receiving": 60.0,
}
LEG_ESTIMATE_DEFAULT_S = 20.0
DEADLINE_DEFAULT_S = 540.0    # 90 % of the 600 s the driver gave the N = 1 bench (BENCH_r05.json)
WATCHDOG_MARGIN_S = 30.0      # what the in-process watchdog leaves before the deadline: the kill, the line


def _bcast_flag(torch, dist, mine, group):
    """Rank 0's decision, on every rank (a host-side broadcast over the gloo group)."""
    t = torch.tensor([1 if mine else 0], dtype=torch.int64)
    dist.broadcast(t, src=0, group=group)
    return bool(int(t.item()))


def _proc_start_time(pid):
    """Wall-clock start of process `pid` (Linux /proc), or None."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            st = f.read()
        ticks = int(st[st.rindex(")") + 2:].split()[19])    # field 22: starttime, clock ticks after boot
        with open("/proc/uptime") as f:
            uptime = float(f.read().split()[0])
        return time.time() - (uptime - ticks / os.sysconf("SC_CLK_TCK"))
    except (OSError, ValueError, IndexError):
        return None


def job_start_time():
    """When the driver's clock started, as near as this process can tell: DEOSS_BENCH_T0 (bench.py's
    own self-launch parent sets it), else the earliest start of this process and of the launcher
    that started it (python -m torch.distributed.run)."""
    t0 = os.environ.get("DEOSS_BENCH_T0")
    if t0:
        try:
            return float(t0)
        except ValueError:
            pass
    starts = [_proc_start_time(os.getpid()) or time.time()]
    try:
        with open(f"/proc/{os.getppid()}/cmdline", "rb") as f:
            parent = f.read().replace(b"\0", b" ").decode(errors="replace")
        if "torch.distributed.run" in parent or "torchrun" in parent:
            starts.append(_proc_start_time(os.getppid()))
    except OSError:
        pass
    return min(t for t in starts if t)


class Legs:
    """The legs after the headline, in order.  Each starts only if its estimate (LEG_ESTIMATE_S)
    fits in what is left before the deadline -- rank 0 decides, every rank follows (`decide`), so
    the collectives inside a leg stay matched -- and after the headline and after every leg rank 0
    prints the whole compact line again.  The last stdout line is therefore always complete and
    parseable and supersedes the one before: a run the driver kills at its limit still leaves the
    headline and every leg finished so far (`legs.pending` names the rest).  A skipped leg is named
    in `problems`; a leg that raised is recorded as that leg's error, never fatal to the line."""

    def __init__(self, out, detail, deadline_s, t0, decide, estimates=None):
        self.out, self.detail, self.deadline, self.t0, self.decide = out, detail, deadline_s, t0, decide
        self.estimates = estimates or LEG_ESTIMATE_S
        self.planned, self.pending = [], []
        out["legs"] = {"deadline_s": deadline_s, "done": {}, "pending": [], "skipped": {}}

    def left(self):
        return self.deadline - (time.time() - self.t0)

    def plan(self, names):
        self.planned, self.pending = list(names), list(names)
        self.out["legs"]["pending"] = list(names)

    def emit(self):
        self.out["legs"]["elapsed_s"] = round(time.time() - self.t0, 1)
        if self.detail is not None:
            emit(self.out, self.detail)

    def run(self, name, fn):
        est = self.estimates.get(name, LEG_ESTIMATE_DEFAULT_S)
        left = self.left()
        if self.decide(left >= est):
            progress(f"leg {name}: estimate {est:.1f} s, {left:.1f} s left before the {self.deadline:.1f} s deadline")
            t = time.time()
            try:
                fn()
            except Exception as e:   # recorded as the leg's error; the line and the later legs go on
                self.out.setdefault("leg_errors", {})[name] = _short(f"{type(e).__name__}: {e}", 300)
            self.out["legs"]["done"][name] = round(time.time() - t, 1)
        else:
            self.out["legs"]["skipped"][name] = (f"estimated {est:.1f} s > {max(left, 0):.1f} s left before the "
                                                 f"{self.deadline:.1f} s deadline (--deadline-s)")
            progress(f"leg {name} skipped: {self.out['legs']['skipped'][name]}")
        self.pending.remove(name)
        self.out["legs"]["pending"] = list(self.pending)
        self.emit()


def run_in_process_leg(args, torch, dist, world, rank, wait_group, legs):
    """N > 1: rank 0 runs the single-process multi-GPU leg in a child process (run_child_leg) while
    every other rank waits on the host group; its watchdog is --inproc-timeout or what is left
    before the deadline less WATCHDOG_MARGIN_S, whichever is shorter.  (result, hung) on every rank."""
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    dist.barrier(group=wait_group)
    inproc, hung = None, False
    if rank == 0:
        timeout = max(10.0, min(args.inproc_timeout, legs.left() - WATCHDOG_MARGIN_S))
        progress(f"in-process leg (rank 0 over every GPU, in a child process; watchdog {timeout:.0f} s)")
        leg = ["--workload", "inprocess", "--gpus", "1", "--inproc-gib", str(args.inproc_gib)]
        if args.same_device:
            leg += ["--same-device", "--inproc-devices", str(world)]
        inproc, hung = run_child_leg([sys.executable, os.path.abspath(__file__), *leg], "in_process", timeout)
        if isinstance(inproc, dict):
            inproc["watchdog_s"] = round(timeout, 1)
    flag = torch.tensor([1 if hung else 0], dtype=torch.int64)
    dist.all_reduce(flag, group=wait_group)           # doubles as the barrier
    return inproc, bool(int(flag.item()))


def exit_after_hang(out, detail):
    """A watchdogged leg never returned (its child was killed): rank 0 prints the line (ok false,
    the leg's error in it), then every rank leaves at once with status 3 -- never 0, so the driver
    records the hang as a failure.  No re-exec, no restart."""
    if out is not None:
        emit(out, detail)
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(3)


def watchdog_check(args) -> None:
    """Hidden --watchdog-check S (tests/test_bench_line.py): a child leg that sleeps past its
    S-second watchdog goes through the same kill and exit path as the N = 8 in-process leg -- no GPU
    touched."""
    out = {"metric": "watchdog check", "value": 0.0, "unit": "GiB/s", "n_gpus": 1, "steps": 0, "warmup": 0}
    r, hung = run_child_leg([sys.executable, "-c", "import time; time.sleep(60)"], "in_process", args.watchdog_check)
    out["other_configs"] = {"in_process": r}
    if hung:
        exit_after_hang(out, args.detail_out)
    emit(out, args.detail_out)


def fake_legs(args) -> None:
    """Hidden --fake-legs S --fake-line PATH (tests/test_bench_line.py): the N > 1 leg sequence with
    no torch and no GPU -- the headline line from PATH printed first, then five legs that each
    sleep S seconds, through the same Legs runner, deadline and per-leg line as the real run -- so a
    test can kill it mid-leg and read the last stdout line, or give it a short --deadline-s."""
    with open(args.fake_line) as f:
        out = json.load(f)
    out.pop("other_configs", None)
    names = ["strong_scaling", "strong_scaling_4KiB", "configs[3]", "configs[4]", "in_process"]
    world, rank = env_int("WORLD_SIZE", 1), env_int("RANK", 0)
    decide, deadline = (lambda mine: mine), args.deadline_s
    if world > 1:   # gloo ranks, no GPU: every rank must follow rank 0's decisions, whatever its own clock says
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        decide = lambda mine: _bcast_flag(torch, dist, mine, None)   # noqa: E731
        if rank:
            deadline = 0.0    # alone, a rank with no time left would skip every leg
    legs = Legs(out, args.detail_out if rank == 0 else None, deadline, job_start_time(), decide,
                estimates={n: args.fake_legs for n in names})
    legs.plan(names)
    legs.emit()

    def leg(name):
        time.sleep(args.fake_legs)
        r = {"value": 1.0, "unit": "GiB/s", "ms_per_step": 1.0, "bit_exact": True}
        if name.startswith("strong"):
            out[name] = r
        else:
            out.setdefault("other_configs", {})[name] = {"bit_exact": True, "devices": 8} if name == "in_process" else r
    for name in names:
        legs.run(name, lambda name=name: leg(name))
    if world > 1:
        if rank and args.detail_out:
            with open(f"{args.detail_out}.rank{rank}.json", "w") as f:
                json.dump(out["legs"], f)
        dist.barrier()
        dist.destroy_process_group()


def strong_scaling_leg(args, torch, dist, world, rank, device, dev_index, gloo, barrier, weak_per_gpu,
                       chunk=32 << 20):
    """N > 1: BASELINE configs[1]'s one 8 GiB object sharded over all N ranks (total work fixed),
    beside the weak-scaling headline; speedup_vs_one_gpu = the same object's root on rank 0's GPU
    alone (single_gpu_ms, timed in the parity leg) / the sharded step.  Checked: the sharded root
    against that single-GPU root and the CPU restatement of the same bytes.
      chunk 32 MiB (configs[1]'s): 256 leaves -- one GPU already runs all 256 serial chains at once
        (0.49 s each), so splitting them over N GPUs cannot shorten the step: ~1x by construction
        (DESIGN.md §7);
      chunk 4 KiB (the sweep's smallest): 2,097,152 leaves -- one GPU is VALU-throughput-bound (K1,
        ~1.5 TB/s), so N GPUs split the work: the regime where north_star's "6x at 8 GPUs" can hold."""
    import copy
    ns = copy.copy(args)
    ns.total_gib, ns.chunk, ns.no_extras = 8.0, chunk, True
    ns.steps, ns.warmup = (3, 1) if chunk >= (1 << 20) else (20, 3)   # 0.49 s vs ~1-6 ms steps
    t0 = time.perf_counter()
    try:
        r = run_object(ns, torch, dist, world, rank, device, dev_index, gloo, barrier)
    except Exception as e:   # reported, never fatal to the headline line
        return {"error": f"{type(e).__name__}: {e}"}
    par = r.get("parity") or {}
    n = (8 << 30) // chunk
    res = {"workload": f"configs[1] strong: one 8 GiB object ({n} leaves of {chunk} B) over {world} GPUs",
           "chunk": chunk, "value": r["value"], "unit": "GiB/s", "ms_per_step": r["ms_per_step"],
           "steps": ns.steps, "bit_exact": par.get("bit_exact"), "single_gpu_ms": par.get("single_gpu_ms"),
           "speedup_vs_one_gpu": (round(par["single_gpu_ms"] / r["ms_per_step"], 3)
                                  if par.get("single_gpu_ms") and r.get("ms_per_step") else None),
           "wall_s": round(time.perf_counter() - t0, 2)}
    if chunk >= (1 << 20):
        res["speedup_vs_one_gpu_share_of_weak"] = round(r["value"] / weak_per_gpu, 3) if weak_per_gpu else None
        res["note"] = "~1x by construction at 32 MiB chunks: 256 chains of ~0.49 s run concurrently on one GPU already"
    else:
        res["note"] = "throughput regime: 2,097,152 leaves split over the GPUs (K1 per rank)"
    return res


DIST_ENV = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK", "ROLE_WORLD_SIZE",
            "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "TORCHELASTIC_RESTART_COUNT",
            "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_USE_AGENT_STORE", "TORCHELASTIC_ERROR_FILE")


def run_child_leg(cmd, key, timeout_s):
    """Run one leg as a child process (its own session, no rank environment) and take `key` from
    the last JSON line it prints: (result, False); ({"error": ...}, False) when it crashed or printed
    no result; ({"error": ...}, True) when it outlived timeout_s, after its process group was killed.
    The N = 8 in-process leg runs this way (one dm_ctx over every GPU of the node, its own
    ncclCommInitAll): a segfault or abort inside it cannot take rank 0's line with it, and a hang is
    killed, so no thread of it is left holding GPUs when the ranks leave.  A child, not an exec: the
    ranks have initialised HIP."""
    import signal
    env = {k: v for k, v in os.environ.items() if k not in DIST_ENV}
    try:
        p = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, cwd=ROOT, text=True, start_new_session=True)
    except OSError as e:
        return {"error": f"could not start the leg: {e}"}, False
    try:
        text, _ = p.communicate(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)   # the group this call started (start_new_session), nothing else
        except OSError:
            pass
        try:   # a child stuck in an uninterruptible driver call may never exit: do not wait for it forever
            p.wait(timeout=30)
            state = "child process group killed"
        except subprocess.TimeoutExpired:
            state = f"child process group killed; pid {p.pid} had not exited 30 s later (left behind)"
        return {"error": f"did not finish within {timeout_s:.0f} s (watchdog: {state})"}, True
    for ln in reversed(text.splitlines()):
        ln = ln.strip()
        if not ln.startswith("{"):
            continue
        try:
            d = json.loads(ln)
        except ValueError:
            continue
        if isinstance(d, dict) and key in d:
            r = d[key]
            if p.returncode != 0 and isinstance(r, dict):
                r = dict(r, error=f"child exited with status {p.returncode} after printing its result")
            return r, False
    return {"error": f"child exited with status {p.returncode} without a result"}, False


def self_launch(n: int, argv) -> int:
    """`--gpus N > 1` with no launcher around it (WORLD_SIZE unset): start the N rank processes
    as a child `python -m torch.distributed.run` (one process per GPU, rendezvous on 127.0.0.1, the
    driver's own launch line) and return its exit status.  Runs before anything imports torch, so
    this parent never initialises HIP and never execs: the ranks are children.  They inherit
    stdout, so rank 0's JSON line is this command's line."""
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    env = dict(os.environ, DEOSS_BENCH_LAUNCHER="bench.py self-launch (child python -m torch.distributed.run)",
               DEOSS_BENCH_T0=os.environ.get("DEOSS_BENCH_T0") or str(job_start_time()))
    print(f"bench.py: WORLD_SIZE unset, launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def launch_check(args) -> None:
    """Hidden --launch-check (tests/test_bench_launch.py): the ranks meet over gloo and rank 0
    prints who they are; nothing touches a GPU.  Proves the self-launch without one."""
    import torch.distributed as dist
    world = env_int("WORLD_SIZE", 1)
    rank = env_int("RANK", 0)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = {"rank": rank, "local_rank": env_int("LOCAL_RANK", 0), "pid": os.getpid()}
    every = [None] * world
    if world > 1:
        dist.all_gather_object(every, mine)
    else:
        every = [mine]
    if rank == 0:
        print(json.dumps({"launch_check": True, "gpus": args.gpus, "world_size": world, "ranks": every,
                          "launcher": os.environ.get("DEOSS_BENCH_LAUNCHER", "external (WORLD_SIZE set)")}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def measure_exchange(plan, torch, dist, device, gloo, barrier, reps=100):
    """N > 1: the headline step's one collective timed alone -- all_gather_into_tensor of the
    fixed per-rank slots sharded_root sends (max nodes x 32 B per rank), `reps` back to back after
    5 warm-ups, wall clock to the device being idle, max over ranks.  This is the measured figure
    for the routing model's all-gather term (dm_plan::route, an estimate of 0.1 ms until a
    multi-GPU node runs this)."""
    slot = plan.max_nodes * 32
    comm = "cpu" if gloo else device
    send = torch.zeros(slot, dtype=torch.uint8, device=comm)
    gathered = torch.empty(plan.world * slot, dtype=torch.uint8, device=comm)
    for _ in range(5):
        dist.all_gather_into_tensor(gathered, send)
    barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_gather_into_tensor(gathered, send)
    if not gloo:
        torch.cuda.synchronize()   # RCCL runs on its own stream; gloo returns when done
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=comm)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return {"collective": "all_gather_into_tensor", "backend": "gloo" if gloo else "nccl (RCCL)",
            "bytes_per_rank": slot, "ranks": plan.world, "reps": reps,
            "avg_us": round(float(t.item()) / reps * 1e6, 2)}


def launch_info(torch, dist, world, rank, local_rank, dev_index, args):
    """What the N > 1 run actually formed: the process group's world size and backend, the GPUs
    each rank saw and used (device id, PCI bus, UUID), and the RCCL version torch runs."""
    props = torch.cuda.get_device_properties(dev_index)
    mine = {"rank": rank, "local_rank": local_rank, "device": dev_index, "pid": os.getpid(),
            "visible_devices": torch.cuda.device_count(),
            "pci_bus_id": getattr(props, "pci_bus_id", None), "uuid": str(getattr(props, "uuid", "")) or None,
            "name": props.name}
    every = [None] * world
    dist.all_gather_object(every, mine)
    try:
        rccl = ".".join(str(x) for x in torch.cuda.nccl.version())
    except Exception as e:   # reported, not fatal
        rccl = f"unavailable ({type(e).__name__})"
    distinct = len({(r["pci_bus_id"], r["uuid"], r["device"]) for r in every})
    return {"world_size": dist.get_world_size(), "backend": str(dist.get_backend()),
            "device_count": torch.cuda.device_count(), "rank_devices": every,
            "distinct_gpus": 1 if args.same_device else distinct, "rccl_version": rccl,
            "launcher": os.environ.get("DEOSS_BENCH_LAUNCHER", "external (WORLD_SIZE set by the caller's launcher)")}


def run_object(args, torch, dist, world, rank, device, dev_index, gloo, barrier, cpu_leg=False):
    """One object over all ranks (BASELINE configs[1] at N = 1, the weak-scaling curve, configs[3]
    with --total-gib 1024): timed steps, roofline, parity legs; with cpu_leg, the CPU baseline
    (N = 1: over the whole object; N > 1: over rank 0's shard).  Returns rank 0's line (other ranks
    get theirs too, unused).  Buffers are released before returning."""
    from deoss_amd import MerkleContext, plan_shards
    from deoss_amd.sharding import sharded_root
    chunk = args.chunk
    total = int(args.total_gib * (1 << 30)) if args.total_gib else int(args.object_gib * (1 << 30)) * world
    plan = plan_shards(total, chunk, world)
    b0, b1 = plan.byte_range(rank)
    local_len = b1 - b0
    ctx = MerkleContext(devices=[dev_index])
    ctx.set_leaf_kernel(args.leaf_kernel)
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream
    buf = torch.empty(local_len + 64, dtype=torch.uint8, device=device)
    ctx.fill_synthetic_async(buf.data_ptr(), b0, (local_len + 7) // 8 * 8, SEED, sptr)
    root_dev = torch.zeros(32, dtype=torch.uint8, device=device)
    nodes_dev = torch.zeros(max(plan.node_count(rank), 1) * 32, dtype=torch.uint8, device=device)

    def subtree(k):
        ctx.subtree_device_async(buf.data_ptr(), local_len, chunk, k, nodes_dev.data_ptr(), sptr)
        return nodes_dev

    def finish(nodes, n, min_one):
        ctx.finish_device_async(nodes.data_ptr(), n, min_one, root_dev.data_ptr(), sptr)
        return root_dev

    def step():
        if world == 1:
            ctx.root_device_async(buf.data_ptr(), local_len, chunk, root_dev.data_ptr(), 0, sptr)
        else:
            sharded_root(plan, rank, subtree, finish, torch, dist, device,
                         comm_device="cpu" if gloo else None)

    for _ in range(args.warmup):
        step()
    barrier()
    ctx.set_timing(True)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    t1 = time.perf_counter()
    ncalls, k1_ms_sum, call_ms_sum, k1_ms_max = ctx.timing_summary()
    ctx.set_timing(False)
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if gloo else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    root_hex = bytes(root_dev.cpu().numpy()).hex() if rank == 0 else None

    value = total * args.steps / elapsed / (1 << 30)
    read_peak_gbs, read_peak_ms = measure_read_peak(ctx, torch, buf, local_len, sptr, stream)
    cpu_out = {}
    if world > 1 and rank == 0 and cpu_leg:
        # N > 1: the CPU baseline over rank 0's shard (at most 8 GiB of whole leaves), copied back
        # from HBM before the buffer goes; when that shard is one whole block of 2^k leaves its CPU
        # root is rank 0's gathered subtree node, checked too
        sample = min(local_len, max(chunk, (8 << 30) // chunk * chunk))
        progress(f"CPU baseline over rank 0's shard ({sample} B)")
        cpu_baseline_over(torch, buf, sample, chunk, cpu_out, total,
                          f"rank 0's shard of the timed object ({sample} of its {local_len} B)")
        cpu_root = cpu_out["cpu_baseline"].pop("root")
        if plan.node_count(0) == 1 and sample == local_len and local_len // chunk == (1 << plan.k) \
                and local_len % chunk == 0:
            cpu_out["cpu_baseline"]["shard_root_bit_exact"] = bytes(nodes_dev[:32].cpu().numpy()).hex() == cpu_root
    if world > 1:   # the whole-object buffer is released before the parity legs allocate theirs
        del buf
        torch.cuda.empty_cache()
    k1_avg_ms = k1_ms_sum / max(ncalls, 1)
    k1_bytes = local_len + 32 * ((local_len + chunk - 1) // chunk)   # read N once + 32 B per leaf
    achieved_gbs = k1_bytes / (k1_avg_ms * 1e-3) / 1e9 if k1_avg_ms > 0 else 0.0
    blocks = blocks_for(local_len, chunk)
    from deoss_amd.isa import chain_instructions_per_block, kernel_counts
    n_local = (local_len + chunk - 1) // chunk
    kind = ctx.leaf_kernel_for(n_local)
    vpb, spb = kernel_counts(kind)
    traffic, traffic_src = load_traffic(kind, n_local, k1_bytes)
    kernel_name = {"wide": "leaf_kernel (K1, one lane per leaf)",
                   "latency": "leaf_kernel_lat (K1L, producer/consumer waves)",
                   "pair": "leaf_kernel_pair (K1P, producer/consumer, rounds on lane pairs)",
                   "quad": "leaf_kernel_quad (K1Q, producer/consumer, rounds spread over 8 lanes)"}[kind]

    gib = total / (1 << 30)
    if world == 1 and total == 8 << 30 and chunk == 32 << 20:
        tag = "BASELINE configs[1]"
    elif total == 1 << 40 and chunk == 32 << 20:
        tag = "BASELINE configs[3] (1 TiB object" + (", 8 GPUs)" if world == 8 else f", {world} ranks)")
    else:
        tag = "configs[1] shape per GPU, weak scaling" if not args.total_gib else "fixed total object"
    out = {
        "metric": "device-resident GiB/s hashed to Merkle root; 1/2/4/8 MI355X scaling",
        "value": round(value, 4),
        "unit": "GiB/s",
        "n_gpus": 1 if args.same_device else world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.total_gib else "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: splitmix64 bytes generated in HBM (same generator as the CPU oracle)",
        "config": {
            "workload": f"{tag}: 1 object of {gib:g} GiB ({total} B) in {world} chunk-range shard(s) of "
                        f"{local_len / (1 << 30):g} GiB, chunk {chunk} B ({plan.n_leaves} leaves)",
            "object_bytes": total, "chunk": chunk, "leaves": plan.n_leaves,
            "parallelism": f"chunk-range shards (2^{plan.k} leaves per block), 1 process per GPU, "
                           f"RCCL all-gather of subtree roots" if world > 1 else "single GPU",
        },
        "roofline": {
            "bound": "hbm", "kernel": kernel_name,
            "achieved": round(achieved_gbs, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved_gbs / HBM_PEAK_GBS, 6),
            "traffic": traffic, "traffic_source": traffic_src,
            "k1_avg_ms": round(k1_avg_ms, 4), "k1_launches": ncalls,
            "algorithmic_bytes_per_launch": k1_bytes,
            "valu": {
                "critical_wave_valu_per_block": vpb, "lane_slots_per_leaf_block": spb, "blocks_per_step": blocks,
                "achieved_slots_per_s": (blocks * spb / (k1_avg_ms * 1e-3)) if (spb and k1_avg_ms) else None,
                "peak_slots_per_s": VALU_SLOT_PEAK,
                "frac": round(blocks * spb / (k1_avg_ms * 1e-3) / VALU_SLOT_PEAK, 6) if (spb and k1_avg_ms) else None,
                "note": "SHA-256 is bound by integer VALU issue, not HBM; v_alignbit/v_add3 cost 2 slots "
                        "(measured, tools/valu_peak.hip); see DESIGN.md",
            },
            "regime": ("latency-bound: each leaf is one serial SHA-256 chain; rate = leaves x per-leaf rate"
                       if kind != "wide" else "throughput (VALU issue)"),
            "per_leaf_MBps": round(local_len / n_local / (k1_avg_ms * 1e-3) / 1e6, 3) if k1_avg_ms else None,
        },
        "root": root_hex,
    }
    if read_peak_gbs:
        out["roofline"]["measured_read_peak"] = {
            "GBps": round(read_peak_gbs, 1), "frac_of_spec": round(read_peak_gbs / HBM_PEAK_GBS, 4),
            "achieved_frac_of_measured": round(achieved_gbs / read_peak_gbs, 6), "ms": round(read_peak_ms, 4),
            "bytes": local_len // 16 * 16,
            "kernel": "read_probe_kernel (dm_read_probe_async: XOR of every word of the same object, one pass)"}
    if kind != "wide" and vpb and k1_avg_ms:
        # The bound that applies to few long leaves: one leaf's serial chain on its consumer wave,
        # which issues at most one VALU instruction every 4 cycles (MI355X_MICROARCH.md, "vector-
        # instruction ISSUE cost, one wave's stream on one SIMD") at the 2.4 GHz maximum clock.
        blocks_per_leaf = (chunk + 9 + 63) // 64
        floor_ms = blocks_per_leaf * vpb * ISSUE_CYCLES_ONE_WAVE / MAX_CLOCK_HZ * 1e3
        out["roofline"]["chain_issue_floor"] = {
            "valu_per_block_on_chain": vpb, "cycles_per_valu_one_wave": ISSUE_CYCLES_ONE_WAVE,
            "clock_ghz": MAX_CLOCK_HZ / 1e9, "blocks_per_leaf": blocks_per_leaf, "floor_ms": round(floor_ms, 3),
            "frac": round(floor_ms / k1_avg_ms, 4),
            "note": "time of one leaf chain at one issue per 4 cycles: the latency-bound kernel's roofline"}
        ipb = chain_instructions_per_block(kind)
        if ipb:
            # the same floor counting every instruction the chain's wave issues (its LDS reads of
            # -(K+W), loop SALU): one instruction per 4 cycles, whatever its type
            all_ms = blocks_per_leaf * ipb * ISSUE_CYCLES_ONE_WAVE / MAX_CLOCK_HZ * 1e3
            out["roofline"]["chain_issue_floor"].update({
                "instructions_per_block_on_chain": round(ipb, 2), "floor_all_instructions_ms": round(all_ms, 3),
                "frac_all_instructions": round(all_ms / k1_avg_ms, 4)})

    if args.same_device:
        out["ranks"] = world
        out["same_device"] = True
        out["note"] = "rehearsal: every rank on cuda:0 of one GPU; not a multi-GPU result"
    if world == 1 and rank == 0:
        extras(args, ctx, torch, buf, local_len, chunk, root_hex, out, sptr)
    out.update(cpu_out)
    cb = out.get("cpu_baseline") or {}
    par, est = cb.get("parallel") or {}, cb.get("all_physical_cores_estimate") or {}
    if rank == 0 and par.get("value") and est.get("value"):
        # BASELINE.md publishes no reference number, so vs_baseline stays null (the contract); the
        # CPU comparisons are their own fields: the job's CPU share (measured; at N > 1 the per-GPU
        # share's rate times N) and every physical core of the host (estimated from that run)
        out["vs_cpu_share"] = round(value / (par["value"] * (world if not args.same_device else 1)), 4)
        out["vs_cpu_all_cores"] = round(value / est["value"], 4)
        out["vs_cpu_basis"] = (f"GPU value / the CPU restatement on the job's {par['cores']} threads"
                               + (f" x {world} GPUs' shares" if world > 1 and not args.same_device else "")
                               + f" (vs_cpu_share) and on all {est['cores']} physical cores of this host "
                               "(vs_cpu_all_cores, estimated from that run); same bytes, same run")
    if world > 1 and not args.no_verify:
        out["parity"] = multi_rank_parity(args, torch, dist, ctx, world, rank, device, sptr, total, chunk,
                                          root_hex, barrier, gloo)
    del ctx
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def config3_leg(args, torch, dist, world, rank, device, dev_index, gloo, barrier):
    """N = 8: BASELINE configs[3], one 1 TiB object (128 GiB and 4,096 leaves per GPU): the sharded
    root timed, checked against a single-GPU root of its 64 GiB prefix and against the committed
    full-size fixture (tests/golden/config3_root.json), which replaces re-hashing 1 TiB on the host
    CPU.  Runs only if every rank has the HBM for it, agreed by one all-reduce before anything is
    allocated; an error every rank meets (DM_ERR_NOMEM, say) costs this entry, not the line."""
    import copy
    t0 = time.perf_counter()
    need = int(args.cfg3_total_gib * (1 << 30)) // world + (8 << 30)
    free, _ = torch.cuda.mem_get_info(device)
    ok = torch.tensor([1 if free >= need else 0], dtype=torch.int64, device="cpu" if gloo else device)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if not int(ok.item()):
        return {"skipped": f"a rank has less than {need} B of free HBM", "wall_s": round(time.perf_counter() - t0, 2)}
    ns = copy.copy(args)
    ns.total_gib, ns.steps, ns.warmup, ns.no_extras = args.cfg3_total_gib, 3, 1, True
    try:
        r3 = run_object(ns, torch, dist, world, rank, device, dev_index, gloo, barrier)
        res = _summary(r3)
        res["pinned_by"] = PIN_MERKLE
        fx = root_fixture(int(ns.total_gib * (1 << 30)), args.chunk, SEED)
        if fx and rank == 0:
            res["fixture_root"] = fx["root"]
            res["fixture_bit_exact"] = r3.get("root") == fx["root"]
    except Exception as e:
        res = {"error": f"{type(e).__name__}: {e}"}
        torch.cuda.empty_cache()
    res["wall_s"] = round(time.perf_counter() - t0, 2)
    barrier()
    return res


def config4_leg(args, torch, dist, world, rank, device, dev_index, gloo, barrier):
    """N = 8: BASELINE configs[4], 100,000 x 1 MiB objects from pinned host memory, 12,500 per GPU
    (replicas, no exchange); every root of every rank checked against the CPU restatement."""
    import copy
    t0 = time.perf_counter()
    ns = copy.copy(args)
    ns.workload, ns.total_objects, ns.object_mib, ns.steps, ns.warmup = "stream", args.cfg4_objects, 1.0, 2, 1
    try:
        res = _summary(run_batch(ns, torch, dist, world, rank, device, dev_index, gloo))
        res["pinned_by"] = PIN_MERKLE
    except Exception as e:
        res = {"error": f"{type(e).__name__}: {e}"}
    res["wall_s"] = round(time.perf_counter() - t0, 2)
    torch.cuda.empty_cache()
    barrier()
    return res


LINE_MAX_BYTES = 6144   # the last stdout line; the driver lost r04's 28 KB line


HEAD_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
             "vs_baseline", "dtype", "data")


def _r(x, nd=4):
    return round(x, nd) if isinstance(x, float) else x


def _short(s, n):
    return s if not isinstance(s, str) or len(s) <= n else s[:n - 3] + "..."


def _extra_line(r):
    """One extra (a BASELINE config or entry point measured beside the headline) in a few fields:
    its value, the time of one step, bit-exactness, its roofline fraction and bound, and ok."""
    if not isinstance(r, dict):
        return {"ok": False, "error": "no result"}
    if "error" in r or "skipped" in r:
        e = {"ok": "skipped" in r and "error" not in r}
        e["error" if "error" in r else "skipped"] = _short(r.get("error") or r.get("skipped"), 160)
        return e
    rf = r.get("roofline") if isinstance(r.get("roofline"), dict) else {}
    e = {"value": _r(r.get("value")), "unit": r.get("unit"), "ms": _r(r.get("ms_per_step"), 2),
         "bit_exact": r.get("bit_exact")}
    if rf:
        e.update({"bound": rf.get("bound"), "frac": _r(rf.get("frac"), 6)})
        if rf.get("traffic_over_algorithmic") is not None:
            e["traffic_x"] = rf["traffic_over_algorithmic"]
        elif rf.get("traffic") and rf.get("algorithmic_bytes_per_launch"):
            e["traffic_x"] = round(rf["traffic"] / rf["algorithmic_bytes_per_launch"], 5)
    cb = r.get("cpu_baseline")
    if isinstance(cb, dict) and cb.get("value") is not None:
        e["cpu"] = {"value": _r(cb["value"]), "cores": cb.get("cores")}
    if r.get("fixture_bit_exact") is not None:
        e["fixture_bit_exact"] = r["fixture_bit_exact"]
    e["ok"] = e["bit_exact"] is True and r.get("fixture_bit_exact") is not False
    return e


def _in_process_line(r):
    if not isinstance(r, dict):
        return {"ok": False, "error": "no result"}
    if "error" in r or "skipped" in r:
        return {"ok": "error" not in r, **{k: _short(r[k], 160) for k in ("error", "skipped") if k in r}}
    e = {"devices": r.get("devices"), "virtual": r.get("virtual_devices"), "bit_exact": r.get("bit_exact")}
    for leg in ("sharded_object", "batch_by_objects", "concurrent_calls"):
        v = r.get(leg) or {}
        e[leg] = ({"GiBps": v.get("GiBps"), "bit_exact": (v.get("parity") or {}).get("bit_exact")}
                  if "error" not in v else {"error": _short(v["error"], 120)})
    x = (r.get("sharded_object") or {}).get("exchange") or {}
    if x:
        e["exchange_avg_us"] = x.get("avg_us")
    hf = r.get("host_feed")
    if isinstance(hf, dict):
        e["host_feed"] = ({k: hf.get(k) for k in ("alone_GBps", "all_GBps", "consistent")} if "error" not in hf
                          else {"error": _short(hf["error"], 120)})
    e["ok"] = r.get("bit_exact") is True
    return e


def route_constants(out):
    """What this N > 1 line measured for the routing model's two estimated constants (dm_plan::route,
    DESIGN.md §7), as the environment variables dm_create reads in their place: DEOSS_ALLGATHER_US
    (the all-gather timed alone, `exchange.avg_us`) and DEOSS_HOST_BYTES_PER_S (the node's aggregate
    zero-copy host read rate, `in_process.host_feed.all_GBps`).  Only from real GPUs over RCCL: a
    one-GPU rehearsal's numbers are not a node's."""
    ex = out.get("exchange") or {}
    if out.get("same_device") or "nccl" not in str(ex.get("backend", "")):
        return None
    rc = {}
    if ex.get("avg_us"):
        rc["DEOSS_ALLGATHER_US"] = round(float(ex["avg_us"]), 1)
    hf = ((out.get("other_configs") or {}).get("in_process") or {}).get("host_feed") or {}
    if isinstance(hf, dict) and hf.get("all_GBps") and hf.get("consistent"):
        rc["DEOSS_HOST_BYTES_PER_S"] = int(float(hf["all_GBps"]) * 1e9)
    return rc or None


def compact_line(out, detail_path=None):
    """Rank 0's last stdout line, at most LINE_MAX_BYTES: the headline and its evidence (roofline,
    CPU baseline, parity, host-buffer rate, launch at N > 1) plus one short entry per extra.  The
    full record (every extra's nested roofline, traffic and CPU legs, the latency tables, the
    in-process leg) goes to the detail file this line names.  `ok` is false when any parity check
    failed or any extra / leg errored; `problems` says which."""
    line = {k: _r(out[k]) for k in HEAD_KEYS if k in out}
    cfg = out.get("config") or {}
    line["config"] = {k: cfg[k] for k in ("workload", "object_bytes", "chunk", "leaves", "parallelism") if k in cfg}
    line["config"]["workload"] = _short(cfg.get("workload"), 240)
    problems = []
    rf = out.get("roofline") or {}
    if rf:
        roof = {k: _r(rf.get(k), 6) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic") if k in rf}
        kn = rf.get("kernel") or ""     # "leaf_kernel_quad (K1Q, producer/...)" -> "leaf_kernel_quad (K1Q)"
        roof["kernel"] = kn.split(" (")[0] + (f" ({kn.split(' (')[1].split(',')[0].rstrip(')')})" if " (" in kn else "")
        alg = rf.get("algorithmic_bytes_per_launch")
        roof.update({"algorithmic_bytes_per_launch": alg, "k1_avg_ms": rf.get("k1_avg_ms"),
                     "k1_launches": rf.get("k1_launches")})
        if rf.get("traffic") and alg:
            roof["traffic_over_algorithmic"] = round(rf["traffic"] / alg, 5)
        cf = rf.get("chain_issue_floor") or {}
        if cf:
            roof["chain_issue_floor"] = {"floor_ms": cf.get("floor_ms"), "frac": cf.get("frac"),
                                         "valu_per_block": cf.get("valu_per_block_on_chain")}
        mp = rf.get("measured_read_peak") or {}
        if mp:
            roof["measured_read_peak_GBps"] = mp.get("GBps")
        line["roofline"] = roof
    cb = out.get("cpu_baseline")
    if isinstance(cb, dict):
        c = {k: _r(cb.get(k)) for k in ("value", "unit", "cores", "kind") if k in cb}
        c["sample"] = _short(cb.get("sample"), 200)
        par = cb.get("parallel") or {}
        if par:
            c["parallel"] = {"value": par.get("value"), "cores": par.get("cores")}
        est = cb.get("all_physical_cores_estimate") or {}
        if est.get("value"):
            c["all_cores_estimate"] = {"value": est.get("value"), "cores": est.get("cores")}
        host = cb.get("host") or {}
        if host.get("model"):
            c["host"] = _short(host["model"], 60)
        line["cpu_baseline"] = c
        for k in ("parallel_roots_agree", "shard_root_bit_exact"):
            if k in cb:
                c[k] = cb[k]
                if cb[k] is False:
                    problems.append(f"cpu_baseline.{k}")
    for k in ("vs_cpu_share", "vs_cpu_all_cores", "vs_cpu_threads"):
        if k in out:
            line[k] = out[k]
    if out.get("vs_cpu_basis"):
        line["vs_cpu_basis"] = _short(out["vs_cpu_basis"], 220)
    par = out.get("parity")
    if isinstance(par, dict):
        p = {k: par[k] for k in ("bit_exact", "prefix_bit_exact", "prefix_fixture_bit_exact", "cpu_bit_exact",
                                 "gpu_root", "cpu_root", "sharded_root", "prefix_bytes", "cpu_threads",
                                 "cpu_root_gibs", "single_gpu_ms") if k in par}
        if par.get("cpu_root_source"):
            p["cpu_root_source"] = _short(par["cpu_root_source"], 90)
        line["parity"] = p
        if par.get("bit_exact") is not True:
            problems.append("parity")
    elif out.get("root"):
        line["root"] = out["root"]
    e2e = out.get("e2e")
    if isinstance(e2e, dict):
        line["e2e"] = {k: e2e[k] for k in ("pinned_host_gibs", "pageable_host_gibs", "root_matches") if k in e2e}
        if e2e.get("root_matches") is False:
            problems.append("e2e")
    sw = out.get("sweep")
    if isinstance(sw, list) and sw:
        line["sweep_gibs"] = {str(s.get("chunk")): s.get("gibs") for s in sw}
        if any(s.get("bit_exact") is False for s in sw):
            problems.append("sweep")
    la = out.get("launch")
    if isinstance(la, dict):
        line["launch"] = {k: la.get(k) for k in ("world_size", "backend", "device_count", "distinct_gpus",
                                                 "rccl_version", "launcher")}
        line["launch"]["launcher"] = _short(la.get("launcher"), 60)
    ex = out.get("exchange")
    if isinstance(ex, dict):
        line["exchange"] = {k: ex.get(k) for k in ("backend", "bytes_per_rank", "ranks", "avg_us")}
        rc = route_constants(out)
        if rc:
            line["route_constants"] = rc
    for k in ("same_device", "note", "ranks"):
        if k in out:
            line[k] = out[k]
    for key in ("strong_scaling", "strong_scaling_4KiB"):
        st = out.get(key)
        if isinstance(st, dict):
            line[key] = {k: _short(v, 160) for k, v in st.items() if k != "note"}
            if st.get("bit_exact") is False or "error" in st:
                problems.append(key)
    extras = {}
    for name, r in (out.get("other_configs") or {}).items():
        extras[name] = _in_process_line(r) if name == "in_process" else _extra_line(r)
        if not extras[name].get("ok"):
            problems.append(name)
    if extras:
        line["extras"] = extras
    lat = out.get("latency")
    if isinstance(lat, dict):
        lt = {}
        for k, v in lat.items():
            if not isinstance(v, dict) or k == "pinned_by":
                continue
            if "error" in v:
                lt[k] = {"error": _short(v["error"], 100)}
            elif k.startswith("crossover"):
                lt[k] = {"gpu_faster_from": v.get("gpu_faster_from"), "bit_exact": v.get("bit_exact")}
            elif "gpu" in v:
                lt[k] = {"gpu_p50_ms": v["gpu"].get("p50_ms"), "cpu_p50_ms": v.get("cpu_1core", {}).get("p50_ms"),
                         "bit_exact": v.get("bit_exact")}
        lt["bit_exact"] = lat.get("bit_exact")
        line["latency"] = lt
        if lat.get("bit_exact") is not True:
            problems.append("latency")
    lg = out.get("legs")
    if isinstance(lg, dict):
        line["legs"] = {k: lg[k] for k in ("deadline_s", "elapsed_s", "done", "pending") if k in lg}
        if lg.get("skipped"):
            line["legs"]["skipped"] = {k: _short(v, 120) for k, v in lg["skipped"].items()}
            problems += [f"skipped:{k}" for k in lg["skipped"]]
        line["complete"] = not lg.get("pending")
    for k, v in (out.get("leg_errors") or {}).items():
        line.setdefault("leg_errors", {})[k] = _short(v, 160)
        problems.append(f"error:{k}")
    line["ok"] = not problems
    if problems:
        line["problems"] = problems
    line["detail"] = detail_path
    # last resort: never let the line outgrow the bound (drop the least important blocks first)
    for k in ("sweep_gibs", "latency", "vs_cpu_basis"):
        if len(json.dumps(line, separators=(",", ":"))) <= LINE_MAX_BYTES:
            break
        line.pop(k, None)
    if len(json.dumps(line, separators=(",", ":"))) > LINE_MAX_BYTES and "extras" in line:
        line["extras"] = {k: {"ok": v.get("ok"), "value": v.get("value")} for k, v in line["extras"].items()}
    return line


def write_detail(out, path):
    """The full record of the run (everything compact_line leaves out) as JSON at `path`; the path
    written, or None when it could not be written (the line says so, the run goes on)."""
    if not path:
        return None
    try:
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        return os.path.relpath(os.path.abspath(path), ROOT) if os.path.abspath(path).startswith(ROOT) else path
    except OSError as e:
        print(f"[bench] detail file {path}: {e}", file=sys.stderr, flush=True)
        return None


def emit(out, detail_path):
    """Rank 0: write the detail file, then print the compact line as stdout's last line."""
    where = write_detail(out, detail_path)
    line = compact_line(out, where)
    print(json.dumps(line, separators=(",", ":")), flush=True)
    return line


def measure_read_peak(ctx, torch, buf, nbytes, sptr, stream, reps=5):
    """Measured HBM read peak (SURVEY.md 8d asks for it next to the spec): the library's streaming
    read probe over the timed object itself, HIP events on the launch stream."""
    n = nbytes // 16 * 16
    if n < (64 << 20):
        return None, None
    x = torch.zeros(1, dtype=torch.int64, device=buf.device)
    ctx.read_probe_async(buf.data_ptr(), n, x.data_ptr(), sptr)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        ctx.read_probe_async(buf.data_ptr(), n, x.data_ptr(), sptr)
    e1.record(stream)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return n / (ms * 1e-3) / 1e9, ms


def multi_rank_parity(args, torch, dist, ctx, world, rank, device, sptr, total, chunk, root_hex, barrier, gloo):
    """Untimed N>1 checks that fit any object size:
    1. prefix: the sharded path over a prefix of <= --prefix-gib (the whole object when it fits)
       vs a single-GPU root of the same prefix on rank 0;
    2. the whole object's root vs its committed full-size fixture (root_fixture: made leaf by leaf
       by the C oracle; the prefix too when one is committed) -- no host re-hash of up to 1 TiB
       inside the driver's time limit.  Without a fixture (reduced rehearsal sizes): the oracle's
       N-thread root of the WHOLE object, its bytes regenerated leaf by leaf on the host."""
    from deoss_amd import plan_shards
    from deoss_amd.sharding import parity_prefix, sharded_root
    res = {"sharded_root": root_hex}
    prefix = parity_prefix(total, chunk, int(args.prefix_gib * (1 << 30)))
    if prefix == total:
        sharded_prefix = root_hex      # the timed result itself
    else:
        pplan = plan_shards(prefix, chunk, world)
        p0, p1 = pplan.byte_range(rank)
        pbuf = torch.empty(max(p1 - p0, 8) + 64, dtype=torch.uint8, device=device)
        if p1 > p0:
            ctx.fill_synthetic_async(pbuf.data_ptr(), p0, (p1 - p0 + 7) // 8 * 8, SEED, sptr)
        pnodes = torch.zeros(max(pplan.node_count(rank), 1) * 32, dtype=torch.uint8, device=device)
        proot = torch.zeros(32, dtype=torch.uint8, device=device)

        def sub(k):
            if p1 > p0:
                ctx.subtree_device_async(pbuf.data_ptr(), p1 - p0, chunk, k, pnodes.data_ptr(), sptr)
            return pnodes

        def fin(nodes, n, min_one):
            ctx.finish_device_async(nodes.data_ptr(), n, min_one, proot.data_ptr(), sptr)
            return proot
        sharded_root(pplan, rank, sub, fin, torch, dist, device, comm_device="cpu" if gloo else None)
        torch.cuda.synchronize()
        sharded_prefix = bytes(proot.cpu().numpy()).hex() if rank == 0 else None
        del pbuf
        torch.cuda.empty_cache()
    barrier()
    if rank == 0:
        full = torch.empty(prefix + 64, dtype=torch.uint8, device=device)
        ctx.fill_synthetic_async(full.data_ptr(), 0, (prefix + 7) // 8 * 8, SEED, sptr)
        one = torch.zeros(32, dtype=torch.uint8, device=device)
        ctx.root_device_async(full.data_ptr(), prefix, chunk, one.data_ptr(), 0, sptr)
        torch.cuda.synchronize()
        single = bytes(one.cpu().numpy()).hex()
        if prefix == total:   # the whole object on this one GPU, timed warm: the strong leg's 1-GPU time
            reps = 3 if chunk >= (1 << 20) else 10
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.root_device_async(full.data_ptr(), prefix, chunk, one.data_ptr(), 0, sptr)
            torch.cuda.synchronize()
            res["single_gpu_ms"] = round((time.perf_counter() - t0) * 1e3 / reps, 3)
        del full
        torch.cuda.empty_cache()
        res.update({"prefix_bytes": prefix, "prefix_sharded_root": sharded_prefix, "prefix_single_gpu_root": single,
                    "prefix_bit_exact": single == sharded_prefix})
        ok = single == sharded_prefix
        pfx = root_fixture(prefix, chunk, SEED) if prefix != total else None
        if pfx:
            res.update({"prefix_fixture_root": pfx["root"], "prefix_fixture_bit_exact": single == pfx["root"]})
            ok = ok and single == pfx["root"]
        fx = root_fixture(total, chunk, SEED)
        if fx:
            res.update({"cpu_root": fx["root"], "cpu_root_source": f"{fx['file']} [{fx['name']}] (oracle, leaf by leaf)",
                        "cpu_bit_exact": fx["root"] == root_hex})
            ok = ok and fx["root"] == root_hex
        elif not args.no_cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            from oracle import Oracle
            threads = max(1, min(os.cpu_count() or 1, cpu_share() * (1 if args.same_device else world)))   # job CPU share
            t0 = time.perf_counter()
            _, cr = Oracle().root_synthetic(total, chunk, SEED, nthreads=threads)
            dt = time.perf_counter() - t0
            res.update({"cpu_root": cr.hex(), "cpu_threads": threads, "cpu_seconds": round(dt, 3),
                        "cpu_root_gibs": round(total / dt / (1 << 30), 4),
                        "cpu_bit_exact": cr.hex() == root_hex})
            ok = ok and cr.hex() == root_hex
        res["bit_exact"] = ok
    barrier()
    return res


def concurrent_callers(ctx, host, length, chunk, root_hex, one_s, dev_index):
    """T threads each hash the same pinned object through dm_root_buffer at once (T concurrent
    uploads on one GPU): on the bench's context (DEOSS_LANES call lanes per GPU, default 2) and on a
    one-lane context (every call serialised on the GPU's one lane)."""
    import threading
    from deoss_amd import MerkleContext

    def run(c, T):
        roots = [None] * T
        go = threading.Barrier(T + 1)

        def work(i):
            go.wait()
            roots[i] = c.root_buffer_ptr(host.data_ptr(), length, chunk)[1].hex()

        th = [threading.Thread(target=work, args=(i,)) for i in range(T)]
        for t in th:
            t.start()
        go.wait()
        t0 = time.perf_counter()
        for t in th:
            t.join()
        return time.perf_counter() - t0, all(r == root_hex for r in roots)

    res, ok = {"lanes": ctx.lane_count, "one_call_s": round(one_s, 4)}, True
    for T in (2, 4):
        s, good = run(ctx, T)
        ok &= good
        res[f"threads_{T}"] = {"wall_s": round(s, 4), "GiBps": round(T * length / s / (1 << 30), 4)}
    with MerkleContext(devices=[dev_index], lanes=1) as one:
        one.root_buffer_ptr(host.data_ptr(), min(length, 64 << 20), chunk)
        s, good = run(one, 2)
        ok &= good
        res["one_lane_threads_2"] = {"wall_s": round(s, 4), "GiBps": round(2 * length / s / (1 << 30), 4)}
    res["roots_match"] = ok
    return res


def cpu_baseline_block(orc, host_ptr, length, chunk, total, out, what):
    """out["cpu_baseline"]: the faithful serial restatement of common/hashtree (1 core, SHA-NI when
    present: stands in for Go crypto/sha256) over `length` bytes of pinned host memory, the same
    bytes on the job's CPU share and on half of it, and the rate every physical core of this host
    would reach on the whole `total`-byte object.  Returns (serial root, the parallel roots agree)."""
    facts = host_cpu_facts()
    t0 = time.perf_counter()
    _, cpu_root = orc.root_buffer_ptr(host_ptr, length, chunk, nthreads=1)
    t1 = time.perf_counter()
    nthr = facts["share"]
    _, cpu_root_p = orc.root_buffer_ptr(host_ptr, length, chunk, nthreads=nthr)
    t2 = time.perf_counter()
    half = max(1, nthr // 2)
    _, cpu_root_h = orc.root_buffer_ptr(host_ptr, length, chunk, nthreads=half)
    t3 = time.perf_counter()
    serial = length / (t1 - t0) / (1 << 30)
    par = length / (t2 - t1) / (1 << 30)
    # Every leaf is one serial chain on one core, so P physical cores hash the object's n leaves in
    # ceil(n / P) rounds of one chain, each as long as one round measured at the share.
    n_sample = (length + chunk - 1) // chunk
    n_total = (total + chunk - 1) // chunk
    P = facts["physical_cores"] or facts["logical_cpus"]
    chain_s = (t2 - t1) / -(-n_sample // nthr)
    rounds_all = -(-n_total // P)
    est_all = total / (rounds_all * chain_s) / (1 << 30) if chain_s > 0 else None
    out["cpu_baseline"] = {
        "value": round(serial, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
        "sample": f"{what}, chunk {chunk}, serial leaves then tree (oracle/merkle_oracle.c, SHA-256 backend "
                  f"{orc.backend()}; stands in for Go crypto/sha256)",
        "host": facts, "root": cpu_root.hex(),
        "parallel": {"value": round(par, 4), "cores": nthr,
                     "scaling": {"1": round(serial, 4), str(half): round(length / (t3 - t2) / (1 << 30), 4),
                                 str(nthr): round(par, 4)},
                     "note": "leaves across the job's CPU share (the GPU box allots 16 CPUs per GPU; "
                             "os.cpu_count() there is the whole machine)"},
        "all_physical_cores_estimate": {
            "value": round(est_all, 4) if est_all else None, "cores": P,
            "method": f"the whole {total} B object's {n_total} leaves in ceil({n_total}/{P}) = {rounds_all} rounds "
                      f"of one chain, a chain as long as one round measured at the share ({chain_s:.3f} s); "
                      "estimated, not run: the box's job limits forbid using every core"},
    }
    return cpu_root, cpu_root_h == cpu_root_p == cpu_root


def cpu_baseline_over(torch, buf, length, chunk, out, total, what):
    """cpu_baseline_block over the first `length` bytes of device buffer `buf`, copied to pinned
    host memory first (N > 1: rank 0's shard)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle   # CPU baseline / checker only
    host = torch.empty(length, dtype=torch.uint8, pin_memory=True)
    host.copy_(buf[:length])
    torch.cuda.synchronize()
    root, ok = cpu_baseline_block(Oracle(), host.data_ptr(), length, chunk, total, out, what)
    out["cpu_baseline"]["parallel_roots_agree"] = ok
    del host
    return root


def extras(args, ctx, torch, buf, length, chunk, root_hex, out, sptr):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    from oracle import Oracle   # CPU baseline / checker only
    orc = Oracle()
    host = None
    do_e2e = (args.e2e or not args.no_extras) and not args.no_e2e
    if not args.no_cpu or do_e2e:
        host = torch.empty(length, dtype=torch.uint8, pin_memory=True)
        host.copy_(buf[:length])
        torch.cuda.synchronize()
    if not args.no_cpu:
        progress("CPU baseline over the headline object")
        cpu_root, cpu_ok = cpu_baseline_block(orc, host.data_ptr(), length, chunk, length, out,
                                              f"the full {length} B object of the timed workload")
        out["cpu_baseline"].pop("root")
        out["parity"] = {"gpu_root": root_hex, "cpu_root": cpu_root.hex(),
                         "bit_exact": cpu_root.hex() == root_hex and cpu_ok}
    if do_e2e and host is not None:
        progress("host-buffer end to end")
        # host pinned buffer -> H2D (overlapped) -> root -> 32 B back (the upload-handler path)
        ctx.root_buffer_ptr(host.data_ptr(), min(length, 64 << 20), chunk)   # warm staging
        t0 = time.perf_counter()
        _, r = ctx.root_buffer_ptr(host.data_ptr(), length, chunk)
        t1 = time.perf_counter()
        pageable = torch.empty(length, dtype=torch.uint8)          # ordinary (pageable) host memory
        pageable.copy_(host)
        ctx.root_buffer_ptr(pageable.data_ptr(), length, chunk)   # warm: the copy path's HBM buffer
        t2 = time.perf_counter()
        _, r2 = ctx.root_buffer_ptr(pageable.data_ptr(), length, chunk)
        t3 = time.perf_counter()
        del pageable
        conc = concurrent_callers(ctx, host, length, chunk, root_hex, t1 - t0, buf.device.index or 0)
        out["e2e"] = {"pinned_host_gibs": round(length / (t1 - t0) / (1 << 30), 4),
                      "pageable_host_gibs": round(length / (t3 - t2) / (1 << 30), 4),
                      "concurrent_callers": conc,
                      "root_matches": r.hex() == root_hex and r2.hex() == root_hex and conc["roots_match"],
                      "path": "dm_root_buffer: pinned host memory hashed in place by K1Q over PCIe (zero-copy); "
                              "pageable memory through the pinned ring, H2D striped and overlapped with the leaf "
                              "kernel; tree; 32 B root back"}
    if not args.sweep and not args.no_extras and not args.no_sweep:
        # the GPU / host crossover: 1 MiB and 64 KiB chunks of the same object
        args.sweep, args.sweep_chunks = True, "65536,1048576"
    if args.sweep and not args.no_sweep:
        progress("chunk-size sweep")
        sweep = []
        root = torch.zeros(32, dtype=torch.uint8, device=buf.device)
        modes = ["wide", "latency", "pair", "quad"] if args.sweep_modes else ["auto"]
        for c, mode in [(int(x), m) for x in args.sweep_chunks.split(",") for m in modes]:
            ctx.set_leaf_kernel(mode)
            reps = 3 if c < (8 << 20) else 2
            ctx.root_device_async(buf.data_ptr(), length, c, root.data_ptr(), 0, sptr)
            torch.cuda.synchronize()
            ctx.set_timing(True)
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.root_device_async(buf.data_ptr(), length, c, root.data_ptr(), 0, sptr)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            n, k1, tot, _ = ctx.timing_summary()
            ctx.set_timing(False)
            gpu_root = bytes(root.cpu().numpy())
            entry = {"chunk": c, "leaves": (length + c - 1) // c, "leaf_kernel": mode,
                     "gibs": round(length * reps / (t1 - t0) / (1 << 30), 3),
                     "k1_gbs": round(length / (k1 / n * 1e-3) / 1e9, 2),
                     "k1_hbm_frac": round(length / (k1 / n * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}
            if host is not None and not args.no_cpu:
                _, cr = orc.root_buffer_ptr(host.data_ptr(), length, c, nthreads=cpu_share())
                entry["bit_exact"] = cr == gpu_root
            sweep.append(entry)
        ctx.set_leaf_kernel("auto")
        out["sweep"] = sweep


if __name__ == "__main__":
    main()
