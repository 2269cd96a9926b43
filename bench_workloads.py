"""The workloads bench.py measures beside its headline (each is also `bench.py --workload ...`):
BASELINE configs[0], [2] and [4] as batches, files through NewHashTree, the streamed upload,
Reed-Solomon, FullProcessing (in HBM, from a file, while receiving), proofs, concurrent callers,
the per-request latency block and the single-process multi-GPU leg; plus the N = 1 line's
`driver_extra_specs` / `run_driver_extra` and the step-level roofline each extra carries.  Every result is
checked against the CPU oracle (test infrastructure, outside the timed regions)."""
from __future__ import annotations

import gc
import hashlib
import json
import os
import subprocess
import sys
import time

from bench_common import (
    ROOT, HBM_PEAK_GBS, SEED, progress, cpu_share, PIN_MERKLE, PIN_PROCESS, pinning_for,
    _host_mem_available, _fill_host, _pcts, PCIE_PEAK_GBS, golden_case)


def latency_block(args, torch, dev_index):
    """Per-request latency of the calls an upload handler makes, GPU vs the serial CPU restatement
    on the same bytes, every result checked bit-exact (N = 1 line, "latency"):
      FullProcessing of a 1 MiB and of a 64 MiB upload -- one call per upload
        (/root/reference/node/objectHandler.go:168, node/fileHandler.go:771): GPU dm_process_buffer
        with every fragment back in host memory, CPU oracle/process_oracle.c, both from a pageable
        host buffer, no files;
      NewHashTreeFromBuffer of 1 MiB at 32 MiB chunks (one leaf);
      NewHashTree(chunkPath) over 256 x 32 MiB files in the page cache (GPU dm_new_hash_tree; CPU
        reads each file whole, then hashes: common/hashtree/types.go:24-38).
    p50 / p99 over repeated single calls on an otherwise idle GPU.  Then "crossover": c requests
    arriving at once, the GPU through the coalescing batcher (dm_batcher) vs the CPU restatement
    on the job's CPU share (one request per core at a time, as gin runs one goroutine per upload),
    wall time for all c: the smallest c at which the GPU finishes first."""
    import ctypes
    import shutil
    import tempfile
    import threading
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    from deoss_amd import MerkleContext
    from deoss_amd.batcher import PROCESS as B_PROCESS, ROOT as B_ROOT, Batcher
    from deoss_amd.process import Processor
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    orc = Oracle()
    share = cpu_share()
    seg, chunk = 32 << 20, 32 << 20
    out = {"gpu": "one MI355X, idle, device " + str(dev_index),
           "cpu": f"serial restatement on 1 core ({orc.backend()} SHA-256, table GF(2^8)); crossover: {share} threads",
           "pinned_by": {"FullProcessing": PIN_PROCESS, "hashtree": PIN_MERKLE}}

    def host(nbytes, seed):
        a = np.empty((nbytes + 7) // 8 * 8, dtype=np.uint8)
        orc.fill_splitmix_ptr(a.ctypes.data, 0, a.size, seed)
        return a

    def timed(fn, reps):
        fn()   # warm
        xs, r = [], None
        for _ in range(reps):
            t = time.perf_counter()
            r = fn()
            xs.append(time.perf_counter() - t)
        return xs, r

    def entry(gx, cx, ok, **kw):
        g, c = _pcts(gx), _pcts(cx)
        e = {"gpu": g, "cpu_1core": c, "gpu_over_cpu_p50": round(g["p50_ms"] / c["p50_ms"], 2), "bit_exact": ok}
        e.update(kw)
        return e

    with MerkleContext(devices=[dev_index]) as ctx:
        proc = Processor(ctx, 4, 8, seg)
        for name, nbytes, reps in (("FullProcessing_1MiB", 1 << 20, 12), ("FullProcessing_64MiB", 64 << 20, 6)):
            try:
                a = host(nbytes, SEED + 0x600 + nbytes)
                nseg = -(-nbytes // seg)
                # the C calls alone, into output buffers allocated and touched once (as a handler that
                # reuses its buffers): Python's allocation and bytes copies stay out of both legs
                bufs = {side: [np.ones(x, dtype=np.uint8) for x in (32 * nseg, 32 * nseg * 12, 32,
                                                                    nseg * 12 * (seg // 4))]
                        for side in ("gpu", "cpu")}

                def gpu_call(b=bufs["gpu"]):
                    proc._check(proc.ctx._L.dm_process_buffer(
                        proc.enc._h, ctypes.c_void_p(a.ctypes.data), nbytes, seg, ctypes.c_void_p(b[3].ctypes.data),
                        ctypes.c_void_p(b[0].ctypes.data), ctypes.c_void_p(b[1].ctypes.data),
                        ctypes.c_void_p(b[2].ctypes.data)), "dm_process_buffer")

                def cpu_call(b=bufs["cpu"]):
                    rc = orc.L.or_full_processing(ctypes.c_void_p(a.ctypes.data), nbytes, seg, 4, 8,
                                                  ctypes.c_void_p(b[0].ctypes.data), ctypes.c_void_p(b[1].ctypes.data),
                                                  ctypes.c_void_p(b[2].ctypes.data), ctypes.c_void_p(b[3].ctypes.data), 1)
                    if rc < 0:
                        raise ValueError(f"or_full_processing rc={rc}")

                gx, _ = timed(gpu_call, reps)
                cx, _ = timed(cpu_call, reps)
                ok = all(np.array_equal(x, y) for x, y in zip(bufs["gpu"], bufs["cpu"]))
                out[name] = entry(gx, cx, ok,
                                  what=f"{nbytes} B upload -> {nseg} zero-padded 32 MiB segment(s), RS 4+8, every "
                                       "segment / fragment digest, fid, fragments back in host memory "
                                       "(dm_process_buffer vs or_full_processing: the C calls, outputs preallocated)")
            except Exception as e:
                out[name] = {"error": f"{type(e).__name__}: {e}"}
        try:
            a = host(1 << 20, SEED + 0x700)
            gx, g = timed(lambda: ctx.root_buffer_ptr(a.ctypes.data, 1 << 20, chunk)[1], 30)
            cx, c = timed(lambda: orc.root_buffer_ptr(a.ctypes.data, 1 << 20, chunk, nthreads=1)[1], 30)
            out["NewHashTreeFromBuffer_1MiB"] = entry(gx, cx, g == c, what="1 MiB pageable buffer, chunk 32 MiB "
                                                      "(one leaf): H2D, one SHA-256 chain, root back")
        except Exception as e:
            out["NewHashTreeFromBuffer_1MiB"] = {"error": f"{type(e).__name__}: {e}"}
        base = "/dev/shm" if os.path.isdir("/dev/shm") and shutil.disk_usage("/dev/shm").free > (12 << 30) else None
        d = tempfile.mkdtemp(prefix="deoss_lat_", dir=base)
        try:
            size, nfiles = 32 << 20, 256
            buf = np.empty(size, dtype=np.uint8)
            paths = []
            for i in range(nfiles):
                orc.fill_splitmix_ptr(buf.ctypes.data, i * size, size, SEED)
                pth = os.path.join(d, f"seg{i:05d}")
                buf.tofile(pth)
                paths.append(pth)

            whole = np.empty(size * nfiles, dtype=np.uint8)

            def cpu_files(threads):
                # read every file whole (io.ReadAll, types.go:25-29) into one buffer, then hash the
                # leaves (one leaf per file; equal sizes, so the buffer split at `size`); reads on
                # `threads` threads too, so the share leg is not bound by one reader
                def rd(i):
                    with open(paths[i], "rb") as f:
                        f.readinto(memoryview(whole)[i * size:(i + 1) * size])
                if threads == 1:
                    for i in range(nfiles):
                        rd(i)
                else:
                    with ThreadPoolExecutor(threads) as ex:
                        list(ex.map(rd, range(nfiles)))
                return orc.root_buffer_ptr(whole.ctypes.data, size * nfiles, size, nthreads=threads)[1]

            gx, g = timed(lambda: ctx.new_hash_tree(paths)[1], 5)
            cx, c = timed(lambda: cpu_files(1), 3)
            px, pc = timed(lambda: cpu_files(share), 3)
            out["NewHashTree_256x32MiB_files"] = entry(
                gx, cx, g == c == pc, cpu_share=dict(_pcts(px), threads=share),
                what="256 files of 32 MiB in the page cache (= BASELINE configs[1] bytes): GPU dm_new_hash_tree; "
                     "CPU reads each file whole into one buffer, then hashes the leaves (types.go:24-38, "
                     "without Go's extra string copy)")
            del whole
        except Exception as e:
            out["NewHashTree_256x32MiB_files"] = {"error": f"{type(e).__name__}: {e}"}
        finally:
            shutil.rmtree(d, ignore_errors=True)

    # crossover: c simultaneous requests, GPU batcher vs the CPU share
    def crossover(mode, nbytes, cs, unit, pinned=False):
        pool_n = 64
        a = host(pool_n * nbytes, SEED + 0x800 + mode)
        pin = None
        if pinned:   # request bodies in page-locked memory (Go: hashtree.NewPinnedBuffer)
            from deoss_amd import PinnedBuffer
            pin = PinnedBuffer(a.size)
            pin.array()[:] = a
            a = pin.array()
        addr = a.ctypes.data

        def want(j):
            p = addr + (j % pool_n) * nbytes
            if mode == B_ROOT:
                return orc.root_buffer_ptr(p, nbytes, unit, nthreads=1)[1]
            return orc.full_processing_ptr(p, nbytes, unit, 4, 8, nthreads=1)[2]

        wants = [want(j) for j in range(pool_n)]
        b = (Batcher(B_ROOT, unit, device=dev_index, linger_us=2000) if mode == B_ROOT
             else Batcher(B_PROCESS, unit, 4, 8, device=dev_index, linger_us=2000))

        def gpu_one(j):
            p = (addr + (j % pool_n) * nbytes, nbytes)
            return b.root(p)[1] if mode == B_ROOT else b.process(p)[2]

        def gpu_wave(c):
            got = [None] * c
            go = threading.Barrier(c + 1)

            def th(j):
                go.wait()
                got[j] = gpu_one(j)

            ts = [threading.Thread(target=th, args=(j,)) for j in range(c)]
            for x in ts:
                x.start()
            go.wait()
            t = time.perf_counter()
            for x in ts:
                x.join()
            return time.perf_counter() - t, all(got[j] == wants[j % pool_n] for j in range(c))

        rows, ok, first = [], True, None
        try:
            gpu_wave(max(cs))   # warm every slot's buffers at the largest wave
            with ThreadPoolExecutor(share) as ex:
                for c in cs:   # each side: the better of 2 waves (Python thread start-up is noisy)
                    w1, w2 = gpu_wave(c), gpu_wave(c)
                    tg, good = min(w1[0], w2[0]), w1[1] and w2[1]
                    tcs = []
                    for _ in range(2):
                        t = time.perf_counter()
                        got = list(ex.map(want, range(c)))
                        tcs.append(time.perf_counter() - t)
                        good = good and all(got[j] == wants[j % pool_n] for j in range(c))
                    tc = min(tcs)
                    ok = ok and good
                    rows.append({"concurrent": c, "gpu_ms": round(tg * 1e3, 2), "cpu_ms": round(tc * 1e3, 2),
                                 "gpu_faster": tg < tc})
            # the smallest c from which the GPU finishes first at every larger c measured too
            for r in reversed(rows):
                if not r["gpu_faster"]:
                    break
                first = r["concurrent"]
        finally:
            b.close()
            if pin is not None:
                del a
                pin.free()
        return {"rows": rows, "gpu_faster_from": first, "bit_exact": ok, "cpu_threads": share,
                "request_bytes": nbytes, "bodies": "pinned host memory" if pinned else "pageable host memory"}

    try:
        out["crossover_FullProcessing_1MiB"] = crossover(B_PROCESS, 1 << 20, (1, 16, 64, 256), seg)
    except Exception as e:
        out["crossover_FullProcessing_1MiB"] = {"error": f"{type(e).__name__}: {e}"}
    for pinned in (False, True):
        name = "crossover_NewHashTreeFromBuffer_1MiB" + ("_pinned" if pinned else "")
        try:
            # at most 512 caller threads: a GPU box caps the processes / threads a job may run
            out[name] = crossover(B_ROOT, 1 << 20, (1, 64, 256, 512), chunk, pinned)
        except Exception as e:
            out[name] = {"error": f"{type(e).__name__}: {e}"}
    out["bit_exact"] = all(v.get("bit_exact") is True for k, v in out.items() if isinstance(v, dict) and
                           k not in ("pinned_by",))
    return out


def in_process_configs(args, torch, world):
    """The single-process multi-GPU path -- what go/hashtree gets from one dm_ctx over every GPU of
    the node (ncclCommInitAll at dm_create, one ncclAllGather per sharded call) -- run
    by rank 0 over every visible GPU after the per-rank legs, while the other ranks wait on a host
    barrier.  Three legs, each checked against the CPU oracle on the same bytes:
      sharded_object: one pinned host object (--inproc-gib, 32 MiB chunks, /root/reference
        common/hashtree/types.go:38's tree) forced through multi_root: aligned block partition
        (dm_plan::plan_shards), every GPU hashing its chunk range in place over PCIe, the RCCL
        all-gather of subtree roots, final levels on device 0; exchange time measured
        (dm_exchange_timing), leaf digests and root checked;
      batch_by_objects: a host batch of 4,096 x 4 MiB objects split by objects over the GPUs;
      concurrent_calls: 8 threads each making one NewHashTree-shaped call (dm_root_chunks over 64 x
        32 MiB) on an unforced context: the GPU each landed on (dm_last_call_devices) and its wall.
    With --same-device (one GPU) the GPUs are DEOSS_VIRTUAL_DEVICES = N stand-ins on cuda:0: the
    same code with a D2D copy in place of RCCL (a rehearsal, not a multi-GPU result)."""
    import ctypes
    import threading
    from concurrent.futures import ThreadPoolExecutor
    from deoss_amd import MerkleContext, PinnedBuffer
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    orc = Oracle()
    virtual = bool(args.same_device)
    visible = torch.cuda.device_count()
    ndev = world if virtual else visible
    res = {"virtual_devices": virtual, "visible_devices": visible, "devices": ndev}
    if ndev < 2:
        res["skipped"] = f"{visible} visible GPU(s): nothing to shard over"
        return res
    chunk = 32 << 20
    size = int(args.inproc_gib * (1 << 30)) // chunk * chunk
    avail = _host_mem_available()
    while size > (4 << 30) and avail and 2 * size + (16 << 30) > avail:   # leave the host room
        size //= 2
    size = max(chunk * 2 * ndev, size // chunk * chunk)
    threads = max(1, min(os.cpu_count() or 1, cpu_share() * (1 if virtual else world)))
    res.update({"object_bytes": size, "chunk": chunk, "host_mem_available": avail, "cpu_threads": threads})
    seed = SEED + 0x500
    t0 = time.perf_counter()
    pin = PinnedBuffer(size)
    _fill_host(orc, pin.ptr, size, seed, threads)
    res["setup_s"] = round(time.perf_counter() - t0, 2)
    L = None

    def make_ctx(forced):
        env = {"DEOSS_FORCE_SHARDED": "1"} if forced else {}
        if virtual:
            env["DEOSS_VIRTUAL_DEVICES"] = str(ndev)
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            t = time.perf_counter()
            c = MerkleContext(devices=None if virtual else list(range(ndev)))
            return c, time.perf_counter() - t
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    try:
        # a. one object sharded over every GPU: multi_root + the RCCL all-gather
        ctx, t_create = make_ctx(True)
        L = ctx._L
        leg = {"dm_create_s": round(t_create, 3), "context_devices": ctx.device_count, "lanes": ctx.lane_count,
               "what": "dm_root_buffer of a pinned host object, DEOSS_FORCE_SHARDED: chunk ranges over every GPU, "
                       "ncclAllGather of the 32-byte subtree roots, final levels on device 0"}
        try:
            ctx.root_buffer_ptr(pin.ptr, size, chunk)            # warm: staging, communicators
            ctx.set_timing(True)
            walls = []
            for _ in range(3):
                t = time.perf_counter()
                leaves, root = ctx.root_buffer_ptr(pin.ptr, size, chunk, want_leaves=True)
                walls.append(time.perf_counter() - t)
            xn, xsum, xmax, xg = ctx.exchange_timing()
            devs, ids, lane = ctx.last_call_devices()
            ctx.set_timing(False)
            t = time.perf_counter()
            want_leaves, want = orc.root_buffer_ptr(pin.ptr, size, chunk, nthreads=threads, want_leaves=True)
            cpu_s = time.perf_counter() - t
            from deoss_amd import plan_shards
            plan = plan_shards(size, chunk, ctx.device_count)
            leg.update({
                "GiBps": round(size / (sum(walls) / len(walls)) / (1 << 30), 4),
                "wall_ms": [round(w * 1e3, 2) for w in walls],
                "ran_on": {"context_devices": devs, "hip_devices": ids, "lane": lane},
                "partition": {"k": plan.k, "blocks": plan.n_blocks, "leaves": plan.n_leaves},
                "exchange": {"calls": xn, "avg_us": round(xsum / xn, 1) if xn else None,
                             "max_us": round(xmax, 1) if xn else None, "devices": xg,
                             "kind": "D2D copies (virtual devices)" if virtual else "ncclAllGather (RCCL)"},
                "cpu": {"seconds": round(cpu_s, 3), "threads": threads,
                        "GiBps": round(size / cpu_s / (1 << 30), 4)},
                "parity": {"root": root.hex(), "cpu_root": want.hex(), "leaves": len(leaves) // 32,
                           "bit_exact": root == want and leaves == want_leaves, "pinned_by": PIN_MERKLE}})
        except Exception as e:
            leg["error"] = f"{type(e).__name__}: {e}"
        res["sharded_object"] = leg

        # b. host batch split by objects (no exchange)
        leg = {"what": "dm_root_batch of 4 MiB objects in pinned host memory, split by objects over the GPUs"}
        try:
            osz = 4 << 20
            nobj = min(4096, size // osz)
            P = (ctypes.c_void_p * nobj)(*[pin.ptr + j * osz for j in range(nobj)])
            Ls = (ctypes.c_uint64 * nobj)(*([osz] * nobj))
            out = ctypes.create_string_buffer(32 * nobj)
            ctx._check(L.dm_root_batch(ctx._h, P, Ls, nobj, chunk, out), "dm_root_batch")   # warm
            walls = []
            for _ in range(2):
                t = time.perf_counter()
                ctx._check(L.dm_root_batch(ctx._h, P, Ls, nobj, chunk, out), "dm_root_batch")
                walls.append(time.perf_counter() - t)
            devs, ids, lane = ctx.last_call_devices()
            with ThreadPoolExecutor(threads) as ex:
                wants = list(ex.map(lambda j: orc.root_buffer_ptr(pin.ptr + j * osz, osz, chunk)[1], range(nobj)))
            got = out.raw
            mism = sum(wants[j] != got[32 * j:32 * j + 32] for j in range(nobj))
            leg.update({"objects": nobj, "object_bytes": osz,
                        "GiBps": round(nobj * osz / (sum(walls) / len(walls)) / (1 << 30), 4),
                        "wall_ms": [round(w * 1e3, 2) for w in walls],
                        "ran_on": {"context_devices": devs, "hip_devices": ids},
                        "parity": {"checked_objects": nobj, "mismatches": int(mism), "bit_exact": mism == 0}})
        except Exception as e:
            leg["error"] = f"{type(e).__name__}: {e}"
        res["batch_by_objects"] = leg
        ctx.close()

        # c. 8 concurrent NewHashTree-shaped calls, routed by the library (unforced context)
        ctx, t_create = make_ctx(False)
        leg = {"dm_create_s": round(t_create, 3), "lanes": ctx.lane_count,
               "what": "8 threads, each one dm_root_chunks over 64 x 32 MiB chunks of pinned host memory at once "
                       "(NewHashTree's in-memory form), routed by the library"}
        try:
            ncall = 8
            per = max(1, min(64, size // chunk // ncall))
            span = per * chunk

            def call(i, rec):
                P = (ctypes.c_void_p * per)(*[pin.ptr + i * span + j * chunk for j in range(per)])
                Ls = (ctypes.c_uint64 * per)(*([chunk] * per))
                root = ctypes.create_string_buffer(32)
                t = time.perf_counter()
                ctx._check(L.dm_root_chunks(ctx._h, P, Ls, per, None, root), "dm_root_chunks")
                w = time.perf_counter() - t
                if rec is not None:
                    devs, ids, lane = ctx.last_call_devices()
                    rec[i] = {"call": i, "wall_ms": round(w * 1e3, 2), "context_devices": devs, "hip_devices": ids,
                              "lane": lane, "root": root.raw}

            for i in range(ncall):            # warm every lane's staging
                call(i, None)
            rec = [None] * ncall
            go = threading.Barrier(ncall + 1)

            def th_main(i):
                go.wait()
                call(i, rec)

            ths = [threading.Thread(target=th_main, args=(i,)) for i in range(ncall)]
            for x in ths:
                x.start()
            go.wait()
            t = time.perf_counter()
            for x in ths:
                x.join()
            wall = time.perf_counter() - t
            with ThreadPoolExecutor(min(threads, ncall)) as ex:
                wants = list(ex.map(lambda i: orc.root_buffer_ptr(pin.ptr + i * span, span, chunk)[1], range(ncall)))
            ok = all(r is not None and r["root"] == wants[i] for i, r in enumerate(rec))
            for r in rec:
                if r is not None:
                    r.pop("root")
            leg.update({"calls": rec, "wall_ms": round(wall * 1e3, 2), "chunks_per_call": per,
                        "GiBps": round(ncall * span / wall / (1 << 30), 4),
                        "gpus_used": sorted({d for r in rec if r for d in r["hip_devices"]}) if not virtual
                        else sorted({d for r in rec if r for d in r["context_devices"]}),
                        "parity": {"checked_calls": ncall, "bit_exact": ok}})
        except Exception as e:
            leg["error"] = f"{type(e).__name__}: {e}"
        res["concurrent_calls"] = leg

        # d. the host feed: PCIe reads of pinned host memory, one GPU alone, then every GPU at once
        leg = {"what": "dm_read_probe_async over the pinned object (zero-copy reads over PCIe): GPU 0 reads its "
                       "slice alone, then every GPU its own slice at once -- the routing model's host-memory "
                       "bandwidth term (dm_plan::route, an estimate of 500 GB/s until measured; DESIGN.md §7)"}
        try:
            leg.update(_host_feed(ctx, torch, pin.ptr, size, ndev, virtual))
        except Exception as e:
            leg["error"] = f"{type(e).__name__}: {e}"
        res["host_feed"] = leg
        ctx.close()
    finally:
        pin.free()
    res["bit_exact"] = all(res.get(k, {}).get("parity", {}).get("bit_exact") is True
                           for k in ("sharded_object", "batch_by_objects", "concurrent_calls"))
    if virtual:
        res["note"] = "rehearsal: virtual devices on one GPU (D2D gather); not a multi-GPU result"
    return res


def _host_feed(ctx, torch, host_ptr, size, ndev, virtual, reps=3):
    """Zero-copy PCIe read rate of pinned host memory (in_process_configs leg d): each device reads
    an equal slice of the object with the library's read probe (XOR of every 16-byte word, one
    pass), on a stream of its own; GPU 0 alone, then every device at once.  Best of `reps`, wall
    clock from the first launch to the last stream idle.  The all-device XOR of slice 0 must equal
    the alone one (the same bytes read twice)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    dp = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(dp), ctypes.c_void_p(host_ptr), 0)
    if rc != 0 or not dp.value:
        raise RuntimeError(f"hipHostGetDevicePointer returned {rc}")
    sl = size // ndev // 16 * 16
    gpu = [0] * ndev if virtual else list(range(ndev))
    xs = [torch.zeros(1, dtype=torch.int64, device=f"cuda:{g}") for g in gpu]
    streams = [torch.cuda.Stream(device=f"cuda:{g}") for g in gpu]

    def run(idx):
        for g in sorted(set(gpu)):
            torch.cuda.synchronize(g)
        t = time.perf_counter()
        for i in idx:
            ctx.read_probe_async(dp.value + i * sl, sl, xs[i].data_ptr(), streams[i].cuda_stream)
        for i in idx:
            streams[i].synchronize()
        return time.perf_counter() - t

    run([0])                                         # warm: the probe's first launch on each device
    alone = min(run([0]) for _ in range(reps))
    x_alone = int(xs[0].item())
    every = min(run(list(range(ndev))) for _ in range(reps))
    return {"slice_bytes": sl, "devices": ndev, "alone_GBps": round(sl / alone / 1e9, 2),
            "all_GBps": round(ndev * sl / every / 1e9, 2), "all_ms": round(every * 1e3, 2),
            "consistent": int(xs[0].item()) == x_alone,
            "note": "virtual devices share one GPU's link: not a multi-GPU figure" if virtual else
                    "aggregate host-to-GPU zero-copy read rate of this node"}


def _summary(r):
    """The fields of a workload's result line worth keeping inside the headline line."""
    if not isinstance(r, dict):
        return {"error": "no result"}
    keep = {k: r[k] for k in ("metric", "value", "unit", "ms_per_step", "steps") if k in r}
    keep["workload"] = r.get("config", {}).get("workload")
    par = r.get("parity", {})
    keep["bit_exact"] = par.get("bit_exact")
    if "prefix_bit_exact" in par or "ranks" in par or "checked_objects" in par:
        keep["parity"] = par
    for k in ("n_gpus", "scaling"):
        if k in r:
            keep[k] = r[k]
    for k in ("k1_avg_ms", "tail_ms_after_last_write", "leaf_kernel", "cpu", "gpu", "streamed", "after_file_saved",
              "at_10GbE", "fragment_lookup"):
        if k in r:
            keep[k] = r[k]
    if "leaf_kernel" in r.get("config", {}):
        keep["leaf_kernel"] = r["config"]["leaf_kernel"]
    rf = r.get("roofline")
    if rf:
        keep["roofline"] = {k: rf.get(k) for k in ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic",
                                                   "traffic_source", "algorithmic_bytes_per_launch") if k in rf}
    if "cpu_baseline" in r:
        keep["cpu_baseline"] = r["cpu_baseline"]
    return keep


# Step-level roofline of each N = 1 extra: (profiles/extras_traffic.json key, bound, algorithmic
# bytes one step must move on the bound's link, what they are, the bytes this design's own kernels
# must move on the memory side per step, what those are).  Sizes are driver_extra_specs()'s.  The PMC
# traffic of the kernels is compared with the design bytes; the blit copies (__amd_rocclr_*) are
# reported apart, since their counter widths across PCIe are uncalibrated.
EXTRA_ROOF = {
    "configs[0]": ("configs0", "hbm", (64 << 20) + 2 * 32, "read the 64 MiB object once + 2 leaf digests",
                   64 << 20, "the leaf kernel reads the object once"),
    "configs[2]": ("configs2", "hbm", 4096 * (4 << 20) + 4096 * 32, "read 4,096 x 4 MiB once + one digest each",
                   4096 * (4 << 20), "the leaf kernel reads every object once"),
    "configs[4]_per_gpu_share": ("configs4", "pcie", 12500 * (1 << 20) + 12500 * 32,
                                 "12,500 x 1 MiB read once from pinned host memory (zero-copy K1Q over PCIe)",
                                 12500 * (1 << 20), "the leaf kernel reads every object once from pinned memory"),
    "files_NewHashTree": ("files", "pcie", 256 * (32 << 20), "256 x 32 MiB files: every byte H2D once",
                          256 * (32 << 20), "the leaf kernel reads the pinned staging once (zero-copy)"),
    "upload_stream_1MiB_chunks": ("upload", "pcie", 8 << 30, "8 GiB pageable body: every byte H2D once",
                                  8 << 30, "the leaf kernel reads the pinned staging once (zero-copy)"),
    "FullProcessing": ("process", "hbm", (8 << 30) * 7,
                       "RS reads 8 GiB and writes 16 GiB of parity; the leaf kernel reads the 8 GiB of segments "
                       "and all 24 GiB of fragments (the data fragments are the segments' bytes again: unfused; "
                       "a single-read fused pipeline would move 24 GiB)",
                       (8 << 30) * 7, "RS 8 GiB read + 16 GiB written, leaf 32 GiB read"),
    "reed_solomon_4+8": ("rs", "hbm", (8 << 30) * 3, "read 8 GiB of segments, write 16 GiB of parity",
                         (8 << 30) * 3, "RS 8 GiB read + 16 GiB written"),
    "FullProcessing_file": ("fullprocessing", "pcie", (2 << 30) * 3, "2 GiB file H2D + 4 GiB parity D2H",
                            (2 << 30) * 7, "RS 2 GiB read + 4 GiB written, leaf 8 GiB read (segments + fragments)"),
    "FullProcessing_while_receiving": ("process_upload", "pcie", (2 << 30) * 3, "2 GiB body H2D + 4 GiB parity D2H",
                                       (2 << 30) * 7,
                                       "RS 2 GiB read + 4 GiB written, leaf 8 GiB read (segments + fragments)"),
}


def extras_traffic():
    """profiles/extras_traffic.json (tools/profile_extras.sh: PMC passes over one step of each
    extra, this round's code), or {}."""
    path = os.path.join(ROOT, "profiles", "extras_traffic.json")
    if not os.path.exists(path):
        return {}, None
    with open(path) as f:
        return json.load(f).get("workloads", {}), "profiles/extras_traffic.json"


def extra_roofline(name, r, traffic, src):
    """Attach the step-level roofline (and the PMC traffic of one step) to extra `name`'s summary.
    A kernel-level roofline the workload reports itself is kept under "kernel_level"."""
    if name not in EXTRA_ROOF or not isinstance(r, dict) or not r.get("ms_per_step"):
        return
    key, bound, alg, what, design, design_what = EXTRA_ROOF[name]
    e = traffic.get(key) or {}
    peak = HBM_PEAK_GBS if bound == "hbm" else PCIE_PEAK_GBS
    ach = alg / (r["ms_per_step"] * 1e-3) / 1e9
    roof = {"bound": bound, "achieved": round(ach, 3), "peak": peak, "unit": "GB/s", "frac": round(ach / peak, 6),
            "traffic": e.get("traffic_bytes_per_step"), "algorithmic_bytes_per_step": alg, "what": what,
            "time_basis": "ms_per_step (the whole step, wall clock)",
            "traffic_scope": (f"{src}[{key}]: memory-side bytes (PMC FETCH_SIZE x 2 + WRITE_SIZE) of every kernel "
                              "and blit copy of one warm step (PMC of 2 steps - PMC of 1 step); host-memory "
                              "reads by the zero-copy kernels count too") if e else
                             "not profiled"}
    if e:
        roof["traffic_over_algorithmic"] = round(e["traffic_bytes_per_step"] / alg, 4)
        roof["traffic_kernels"] = {k: round(v["read_bytes"] + v["write_bytes"]) for k, v in e["kernels"].items()}
        kern = sum(v["read_bytes"] + v["write_bytes"] for k, v in e["kernels"].items() if not k.startswith("__amd_"))
        roof.update({"design_kernel_bytes_per_step": design, "design_what": design_what,
                     "kernel_traffic": round(kern), "kernel_traffic_over_design": round(kern / design, 4),
                     "copy_traffic": round(e["traffic_bytes_per_step"] - kern)})
        if e.get("method"):
            roof["traffic_method"] = e["method"]
    if isinstance(r.get("roofline"), dict):
        kl = dict(r["roofline"])
        if kl.get("traffic") is None and e:   # the kernel-level line's own kernel, from the same passes
            leaf = [k for k in e["kernels"] if k.startswith("leaf_kernel")]
            if len(leaf) == 1:
                kv = e["kernels"][leaf[0]]
                kl["traffic"] = (kv["read_bytes"] + kv["write_bytes"]) / max(kv["launches"], 1)
                kl["traffic_source"] = f"{src}[{key}].kernels.{leaf[0]} (per launch)"
        roof["kernel_level"] = kl
    r["roofline"] = roof


def driver_extra_specs():
    """N = 1 only: the other BASELINE configs and entry points measured in the same run as the
    headline so the round's driver records them (each is also its own --workload), as
    (name, runner, argument overrides), in the order bench.py runs them (one leg each)."""
    return [
        ("configs[0]", run_plumbing, dict(workload="plumbing", steps=2, warmup=1)),
        ("configs[2]", run_batch, dict(workload="batch", objects=4096, object_mib=4.0, steps=3, warmup=1)),
        ("configs[4]_per_gpu_share", run_batch, dict(workload="stream", objects=12500, object_mib=1.0, steps=2,
                                                     warmup=1)),
        ("files_NewHashTree", run_files, dict(workload="files", objects=256, object_mib=32.0, steps=2, warmup=1)),
        ("upload_stream_1MiB_chunks", run_upload, dict(workload="upload", chunk=1 << 20, object_gib=8.0, steps=2,
                                                       warmup=1)),
        ("FullProcessing", run_process, dict(workload="process", object_gib=8.0, steps=2, warmup=1)),
        ("reed_solomon_4+8", run_rs, dict(workload="rs", object_gib=8.0, steps=3, warmup=1)),
        ("FullProcessing_file", run_fullprocessing, dict(workload="fullprocessing", object_gib=2.0, steps=2,
                                                         warmup=1)),
        ("FullProcessing_while_receiving", run_process_upload, dict(workload="process_upload", object_gib=2.0,
                                                                    piece_kib=1024, steps=2, warmup=1)),
    ]


def run_driver_extra(name, fn, kw, args, torch, dist, device, dev_index, traffic, tsrc):
    """One extra of driver_extra_specs() on this GPU: its summary with the step-level roofline
    (extra_roofline) and its wall time.  A failing extra is reported as an error field; it never
    fails the headline."""
    import copy
    progress(f"extra {name}")
    ns = copy.copy(args)
    ns.__dict__.update(kw)
    t0 = time.perf_counter()
    try:
        r = _summary(fn(ns, torch, dist, 1, 0, device, dev_index, False))
        r["pinned_by"] = pinning_for(ns.workload, getattr(ns, "mode", "root"))
        extra_roofline(name, r, traffic, tsrc)
    except Exception as e:   # reported, never fatal to the headline line
        r = {"error": f"{type(e).__name__}: {e}"}
    r["wall_s"] = round(time.perf_counter() - t0, 2)
    gc.collect()   # the workload's contexts and buffers go now, not during the next one's timing
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return r


def cpu_fp_baseline(orc, addr, length, seg, what, serial_segs=2, par_segs=64):
    """cpu_baseline of the FullProcessing restatement (oracle/process_oracle.c: SHA-NI SHA-256 +
    table GF(2^8) RS, segment after segment like the SDK) over the first segments of the same
    bytes: 1 thread on `serial_segs`, and the job's CPU share on `par_segs` (one segment per thread
    at a time: how a host with more cores runs concurrent uploads)."""
    from concurrent.futures import ThreadPoolExecutor
    nseg = max(1, -(-length // seg))
    n1, np_ = min(nseg, serial_segs), min(nseg, par_segs)
    b1 = min(length, n1 * seg)
    t = time.perf_counter()
    orc.full_processing_ptr(addr, b1, seg, 4, 8, nthreads=1)
    serial = b1 / (time.perf_counter() - t) / (1 << 30)
    share = cpu_share()
    bp = min(length, np_ * seg)

    def one(s_i):
        return orc.full_processing_ptr(addr + s_i * seg, min(seg, length - s_i * seg), seg, 4, 8, nthreads=1)[2]

    t = time.perf_counter()
    with ThreadPoolExecutor(share) as ex:
        list(ex.map(one, range(np_)))
    par = bp / (time.perf_counter() - t) / (1 << 30)
    return {"value": round(serial, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{n1} segment(s) ({b1} B) of {what} through oracle/process_oracle.c (SHA-256 + RS 4+8 "
                      "+ fid, serial like the SDK; in memory, no file writes)",
            "parallel": {"value": round(par, 4), "cores": share,
                         "sample": f"{np_} segments ({bp} B), one per thread at a time"}}


def cpu_root_baseline(orc, addr, length, chunk, what, serial_bytes, par_s=None, par_bytes=None):
    """cpu_baseline of the hashtree restatement (oracle/merkle_oracle.c, SHA-NI): 1 thread over the
    first serial_bytes (whole chunks) of the same bytes, and the job's CPU share over all of them
    (par_s: the seconds a parity check already spent doing exactly that, else timed here)."""
    share = cpu_share()
    b1 = max(chunk, min(length, serial_bytes) // chunk * chunk) if length > chunk else length
    t = time.perf_counter()
    orc.root_buffer_ptr(addr, b1, chunk, nthreads=1)
    serial = b1 / (time.perf_counter() - t) / (1 << 30)
    if par_s is None:
        t = time.perf_counter()
        orc.root_buffer_ptr(addr, length, chunk, nthreads=share)
        par_s, par_bytes = time.perf_counter() - t, length
    return {"value": round(serial, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{b1} B of {what}, chunk {chunk}: serial leaves then tree (oracle/merkle_oracle.c, SHA-NI; "
                      "stands in for Go common/hashtree)",
            "parallel": {"value": round(par_bytes / par_s / (1 << 30), 4), "cores": share,
                         "sample": f"{par_bytes} B, leaves across threads"}}


def run_files(args, torch, dist, world, rank, device, dev_index, gloo):
    """The reference's own entry point, NewHashTree(chunkPath) (common/hashtree/types.go:19-39):
    --objects files of --object-mib each, already in the page cache (DeOSS writes segment files
    and hashes them right after).  File i holds bytes [i*S, (i+1)*S) of the configs[1] synthetic
    object, so 256 x 32 MiB files give the configs[1] root (tests/golden fixture).  One step =
    dm_new_hash_tree (open + fstat, parallel pread into pinned staging, H2D overlapped with the
    reads and the leaf kernel, tree, root and leaf digests back)."""
    import shutil
    import tempfile
    from deoss_amd import MerkleContext
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    nfiles = args.objects if args.objects != 4096 else 256     # bench default: 256 x 32 MiB = 8 GiB
    size = int(args.object_mib * (1 << 20)) if args.object_mib != 4.0 else 32 << 20
    total = nfiles * size
    orc = Oracle()
    base = "/dev/shm" if os.path.isdir("/dev/shm") and shutil.disk_usage("/dev/shm").free > 2 * total else None
    d = tempfile.mkdtemp(prefix="deoss_files_", dir=base)
    try:
        buf = torch.empty(size, dtype=torch.uint8)
        paths = []
        for i in range(nfiles):
            orc.fill_splitmix_ptr(buf.data_ptr(), i * size, size // 8 * 8, SEED)
            p = os.path.join(d, f"seg{i:05d}")
            buf.numpy().tofile(p)
            paths.append(p)
        del buf
        ctx = MerkleContext(devices=[dev_index])
        ctx.set_leaf_kernel(args.leaf_kernel)
        for _ in range(args.warmup):
            ctx.new_hash_tree(paths)
        times = []
        for _ in range(args.steps):
            t0 = time.perf_counter()
            leaves, root = ctx.new_hash_tree(paths)
            times.append(time.perf_counter() - t0)
        tavg = sum(times) / len(times)
        threads = cpu_share()
        want_leaves, want = orc.root_synthetic(total, size, SEED, nthreads=threads, want_leaves=True)
        parity = {"root": root.hex(), "cpu_root": want.hex(),
                  "bit_exact": root == want and b"".join(leaves) == want_leaves}
        if nfiles == 256 and size == 32 << 20:
            parity["fixture_root"] = golden_case("config1_8192MiB_chunk32MiB")["root"]
            parity["bit_exact"] = parity["bit_exact"] and root.hex() == parity["fixture_root"]
        out = {
            "metric": "GiB/s of files hashed to a Merkle root through NewHashTree(chunkPath) (page cache -> root)",
            "value": round(total / tavg / (1 << 30), 4), "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(tavg * 1e3, 3), "higher_is_better": True,
            "scaling": "none", "vs_baseline": None, "dtype": "u32",
            "data": f"synthetic: {nfiles} files in {'/dev/shm' if base else 'the temp dir'} (page cache)",
            "config": {"workload": f"{nfiles} files x {size} B ({total} B), one leaf per file",
                       "files": nfiles, "file_bytes": size, "leaf_kernel": ctx.leaf_kernel_for(nfiles)},
            "step_ms": [round(t * 1e3, 2) for t in times],
            "parity": parity,
        }
        if not args.no_cpu:
            # faithful serial restatement of types.go:24-38 on a sample: read each file whole, then hash
            sample = paths[:min(nfiles, 16)]
            t0 = time.perf_counter()
            chunks = []
            for p in sample:
                with open(p, "rb") as f:
                    chunks.append(f.read())
            orc.root_chunks(chunks, nthreads=1)
            dt = time.perf_counter() - t0
            del chunks
            # every file on the job's CPU share: threads read the files into one buffer, then hash
            import numpy as np
            from concurrent.futures import ThreadPoolExecutor
            share = cpu_share()
            big = np.empty(total, dtype=np.uint8)

            def rd(i):
                with open(paths[i], "rb") as f:
                    f.readinto(memoryview(big)[i * size:(i + 1) * size])

            t0 = time.perf_counter()
            with ThreadPoolExecutor(share) as ex:
                list(ex.map(rd, range(nfiles)))
            _, proot = orc.root_buffer_ptr(big.ctypes.data, total, size, nthreads=share)
            dtp = time.perf_counter() - t0
            del big
            out["cpu_baseline"] = {"value": round(len(sample) * size / dt / (1 << 30), 4), "unit": "GiB/s", "cores": 1,
                                   "kind": "port", "sample": f"{len(sample)} of the same files: read whole (io.ReadAll), "
                                   "then serial SHA-256 leaves + tree (oracle/merkle_oracle.c, SHA-NI)",
                                   "parallel": {"value": round(total / dtp / (1 << 30), 4), "cores": share,
                                                "sample": f"all {nfiles} files read by {share} threads, leaves across "
                                                          "them", "bit_exact": proot == root}}
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


def run_plumbing(args, torch, dist, world, rank, device, dev_index, gloo):
    """BASELINE configs[0]: one 64 MiB synthetic object at 32 MiB chunks (2 leaves) -- the
    reference's CPU plumbing config.  Times the faithful serial CPU restatement (the stand-in for
    the Go path) and the GPU path on the same bytes; both roots against the committed fixture."""
    from deoss_amd import MerkleContext
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    case = golden_case("config0_64MiB_chunk32MiB")
    length, chunk, seed = case["len"], case["chunk"], case["seed"]
    orc = Oracle()
    host = torch.empty(length, dtype=torch.uint8)
    orc.fill_splitmix_ptr(host.data_ptr(), 0, length, seed)
    reps = max(args.steps, 3)
    t0 = time.perf_counter()
    for _ in range(reps):
        _, cpu_root = orc.root_buffer_ptr(host.data_ptr(), length, chunk, nthreads=1)
    cpu_s = (time.perf_counter() - t0) / reps
    ctx = MerkleContext(devices=[dev_index])
    buf = torch.empty(length + 64, dtype=torch.uint8, device=device)
    sptr = torch.cuda.current_stream().cuda_stream
    ctx.fill_synthetic_async(buf.data_ptr(), 0, length, seed, sptr)
    root_dev = torch.zeros(32, dtype=torch.uint8, device=device)
    elapsed, n, k_sum, _ = timed_steps(args, torch, dist, world, device, gloo, ctx,
                                       lambda: ctx.root_device_async(buf.data_ptr(), length, chunk,
                                                                     root_dev.data_ptr(), 0, sptr))
    gpu_root = bytes(root_dev.cpu().numpy()).hex()
    out = {
        "metric": "BASELINE configs[0]: 64 MiB object through common/hashtree (CPU plumbing config)",
        "value": round(length / cpu_s / (1 << 30), 4), "unit": "GiB/s", "n_gpus": 0, "steps": reps,
        "warmup": 0, "ms_per_step": round(cpu_s * 1e3, 3), "higher_is_better": True, "scaling": "none",
        "vs_baseline": None, "dtype": "u32", "data": "synthetic splitmix64 object (seed 0xDE0550000)",
        "config": {"workload": f"configs[0]: 1 object of {length} B, chunk {chunk} B (2 leaves)", "object_bytes": length,
                   "chunk": chunk},
        "cpu": {"kind": "port", "cores": 1, "seconds": round(cpu_s, 4),
                "what": "oracle/merkle_oracle.c faithful serial restatement (SHA-NI), stands in for Go common/hashtree"},
        "cpu_baseline": cpu_root_baseline(orc, host.data_ptr(), length, chunk, "the configs[0] object", length),
        "gpu": {"device_resident_GiBps": round(length * args.steps / elapsed / (1 << 30), 4),
                "ms_per_root": round(elapsed / args.steps * 1e3, 3), "leaf_kernel": ctx.leaf_kernel_for(2)},
        "parity": {"fixture_root": case["root"], "cpu_root": cpu_root.hex(), "gpu_root": gpu_root,
                   "bit_exact": cpu_root.hex() == case["root"] == gpu_root},
    }
    return out


def run_upload(args, torch, dist, world, rank, device, dev_index, gloo):
    """§8f #1: the upload body arrives in pieces; dm_stream hashes whole leaves while later pieces
    are still being written.  Timed from open to the root; the tail (last write -> root) is the
    latency a handler sees after the body ends."""
    from deoss_amd import MerkleContext
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    length = int(args.object_gib * (1 << 30))
    chunk = args.chunk
    piece = args.piece_kib << 10
    ctx = MerkleContext(devices=[dev_index])
    ctx.set_leaf_kernel(args.leaf_kernel)
    orc = Oracle()
    host = torch.empty(length, dtype=torch.uint8)            # pageable, like a Go []byte body
    orc.fill_splitmix_ptr(host.data_ptr(), 0, length // 8 * 8, SEED)
    base = host.data_ptr()

    def one():
        st = ctx.open_stream(chunk)
        t0 = time.perf_counter()
        for off in range(0, length, piece):
            st.write((base + off, min(piece, length - off)))
        t1 = time.perf_counter()
        _, r = st.close()
        t2 = time.perf_counter()
        return r, t2 - t0, t2 - t1

    for _ in range(args.warmup):
        one()
    times, tails, root = [], [], None
    for _ in range(args.steps):
        root, t, tail = one()
        times.append(t)
        tails.append(tail)
    t0 = time.perf_counter()
    _, want = orc.root_buffer_ptr(base, length, chunk, nthreads=cpu_share())
    par_s = time.perf_counter() - t0
    tavg = sum(times) / len(times)
    out = {
        "metric": "host-buffer upload GiB/s hashed to Merkle root while receiving (dm_stream, pageable pieces)",
        "value": round(length / tavg / (1 << 30), 4), "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(tavg * 1e3, 3), "higher_is_better": True,
        "scaling": "none", "vs_baseline": None, "dtype": "u32", "data": "synthetic splitmix64 object",
        "config": {"workload": f"{length} B object written in {piece} B pieces, chunk {chunk}",
                   "leaf_kernel": ctx.leaf_kernel_for(min(64, (length + chunk - 1) // chunk))},
        "tail_ms_after_last_write": round(sum(tails) / len(tails) * 1e3, 3),
        "write_ms": round((tavg - sum(tails) / len(tails)) * 1e3, 3),
        "parity": {"root": root.hex(), "cpu_root": want.hex(), "bit_exact": root == want},
    }
    if not args.no_cpu:
        out["cpu_baseline"] = cpu_root_baseline(orc, base, length, chunk, "the same upload body", 1 << 30,
                                                par_s, length)
    return out


def load_rs_traffic(key: str):
    """PMC HBM bytes per rs_code_kernel launch (profiles/rs_traffic.json, tools/pmc_traffic.py)."""
    path = os.path.join(ROOT, "profiles", "rs_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    e = d.get("by_kernel_grid", {}).get(key)
    if not e:
        return None, None
    return e["hbm_bytes_per_launch"], f"profiles/rs_traffic.json[{key}] <- " + d.get("source", "")


def run_rs(args, torch, dist, world, rank, device, dev_index, gloo):
    """§8f #3: Reed-Solomon 4 + 8 fragment coding (cess-go-sdk via klauspost/reedsolomon, go.mod:65)
    of device-resident segments.  One step = every segment of this rank coded into 8 parity
    fragments by one rs_code_kernel launch.  Weak scaling, no exchange (segments are independent)."""
    from deoss_amd import MerkleContext
    from deoss_amd.reedsolomon import New
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    seg = args.segment_mib << 20
    shard = seg // 4
    nseg = max(1, int(args.object_gib * (1 << 30)) // seg)
    ctx = MerkleContext(devices=[dev_index])
    enc = New(ctx, 4, 8)
    data = torch.empty(nseg * seg, dtype=torch.uint8, device=device)
    parity = torch.empty(nseg * 2 * seg, dtype=torch.uint8, device=device)
    sptr = torch.cuda.current_stream().cuda_stream
    ctx.fill_synthetic_async(data.data_ptr(), 0, nseg * seg, SEED + 0x100 * (rank + 1), sptr)

    def step():
        enc.encode_device_async(data.data_ptr(), seg, parity.data_ptr(), 2 * seg, shard, nseg, sptr)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    n, k_sum, _, _ = ctx.timing_summary()
    ctx.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if gloo else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # parity: first and last segment vs the CPU restatement
    orc = Oracle()
    checked, ok = [], True
    for s_i in sorted({0, nseg - 1}):
        d = data[s_i * seg:(s_i + 1) * seg].cpu().numpy()
        want = orc.rs_encode([d[j * shard:(j + 1) * shard].tobytes() for j in range(4)], 8,
                             nthreads=cpu_share())
        got = parity[s_i * 2 * seg:(s_i + 1) * 2 * seg].cpu().numpy()
        same = all(got[i * shard:(i + 1) * shard].tobytes() == want[i] for i in range(8))
        checked.append(s_i)
        ok = ok and same
    if rank != 0:
        return
    total = nseg * seg * world
    k_avg_ms = k_sum / max(n, 1)
    alg = 3 * nseg * seg                 # read 4 data shards + write 8 parity shards, per launch
    achieved = alg / (k_avg_ms * 1e-3) / 1e9 if k_avg_ms > 0 else 0.0
    grid_key = f"rs:{nseg}x{seg}"
    traffic, traffic_src = load_rs_traffic(grid_key)
    out = {
        "metric": "device-resident GiB/s of segment data Reed-Solomon coded (4 data + 8 parity fragments)",
        "value": round(total * args.steps / elapsed / (1 << 30), 4), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8 (GF(2^8))",
        "data": "synthetic splitmix64 segments generated in HBM",
        "config": {"workload": f"{nseg} segments x {seg} B per GPU -> 4 + 8 fragments of {shard} B "
                               "(klauspost/reedsolomon New(4, 8) as cess-go-sdk uses it)",
                   "segments_per_gpu": nseg, "segment_bytes": seg, "parallelism": f"{world} x independent"},
        "roofline": {"bound": "hbm", "kernel": "rs_code_kernel<4> (LDS table lookup per input byte)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                     "kernel_avg_ms": round(k_avg_ms, 4), "launches": n, "algorithmic_bytes_per_launch": alg},
        "parity": {"segments_checked": checked, "bit_exact": ok},
    }
    if world == 1 and not args.no_cpu:
        sample = min(nseg, 8)
        d = data[:sample * seg].cpu().numpy()
        import ctypes
        buf = d.ctypes.data
        outs = [ctypes.create_string_buffer(shard) for _ in range(8)]
        pp = [ctypes.addressof(b) for b in outs]
        res = {}
        for threads in (1, cpu_share()):
            t0 = time.perf_counter()
            for s_i in range(sample):
                orc.rs_encode_ptrs(4, 8, [buf + s_i * seg + j * shard for j in range(4)], pp, shard, threads)
            res[threads] = sample * seg / (time.perf_counter() - t0) / (1 << 30)
        out["cpu_baseline"] = {"value": round(res[1], 4), "unit": "GiB/s", "cores": 1, "kind": "port",
                               "sample": f"{sample} segments x {seg} B of the same data, scalar table-driven "
                                         "GF(2^8) encode (oracle/rs_oracle.c, stands in for klauspost's Go path)",
                               "parallel": {"value": round(res[max(res)], 4), "cores": max(res)}}
    return out


def timed_steps(args, torch, dist, world, device, gloo, ctx, step):
    """Warmup, then exactly args.steps steps between barrier + synchronize; max over ranks.
    Returns (elapsed s, timed calls, sum of leaf-kernel ms, sum of whole-call ms)."""
    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed = time.perf_counter() - t0
    n, k_sum, call_sum, _ = ctx.timing_summary()
    ctx.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if gloo else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, n, k_sum, call_sum


def run_process(args, torch, dist, world, rank, device, dev_index, gloo):
    """§8f #2: cess-go-sdk FullProcessing (cipher "") of a device-resident object: zero-padded
    32 MiB segments -> RS 4 + 8 fragments -> SHA-256 of every segment and fragment -> fid.  One
    step = one dm_process_device_async call (RS launch + one leaf-kernel launch over 13 leaves per
    segment + the fid tree).  Weak scaling: objects are independent, no exchange."""
    from deoss_amd import MerkleContext
    from deoss_amd.process import Processor
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    seg = args.segment_mib << 20
    k, m = 4, 8
    frag = seg // k
    length = int(args.object_gib * (1 << 30))
    nseg = -(-length // seg)
    ctx = MerkleContext(devices=[dev_index])
    ctx.set_leaf_kernel(args.leaf_kernel)
    proc = Processor(ctx, k, m, seg)
    sptr = torch.cuda.current_stream().cuda_stream
    obj = torch.empty(nseg * seg, dtype=torch.uint8, device=device)
    ctx.fill_synthetic_async(obj.data_ptr(), 0, (length + 7) // 8 * 8, SEED + 0x200 * (rank + 1), sptr)
    parity = torch.empty(nseg * m * frag, dtype=torch.uint8, device=device)
    segh = torch.empty(nseg * 32, dtype=torch.uint8, device=device)
    fragh = torch.empty(nseg * (k + m) * 32, dtype=torch.uint8, device=device)
    fid = torch.empty(32, dtype=torch.uint8, device=device)

    def step():
        proc.process_device_async(obj.data_ptr(), length, parity.data_ptr(), segh.data_ptr(), fragh.data_ptr(),
                                  fid.data_ptr(), sptr)

    elapsed, n, k_sum, call_sum = timed_steps(args, torch, dist, world, device, gloo, ctx, step)
    # parity: every segment digest and the fid (CPU, 16 threads over the same bytes), all 12
    # fragment digests of the first and last segment (CPU restatement of Split + Encode + SHA-256)
    orc = Oracle()
    host = obj[:length].cpu().numpy()
    threads = cpu_share()
    padded = host[(nseg - 1) * seg:].tobytes() + bytes(nseg * seg - length)
    want_seg, _ = orc.root_buffer_ptr(host.ctypes.data, (nseg - 1) * seg, seg, threads, True) if nseg > 1 \
        else (b"", None)
    want_seg = (want_seg or b"") + orc.sha256(padded)
    want_fid = orc.reduce(want_seg)[:32]
    got_seg = bytes(segh.cpu().numpy())
    got_frag = bytes(fragh.cpu().numpy())
    frag_ok = True
    for s_i in sorted({0, nseg - 1}):
        sbytes = padded if s_i == nseg - 1 else host[s_i * seg:(s_i + 1) * seg].tobytes()
        wseg, wfrag, _, _ = orc.full_processing(sbytes, seg, k, m, nthreads=threads)
        frag_ok &= wfrag == got_frag[s_i * (k + m) * 32:(s_i + 1) * (k + m) * 32]
    parity_ok = got_seg == want_seg and bytes(fid.cpu().numpy()) == want_fid and frag_ok
    if rank != 0:
        return
    k_avg_ms = k_sum / max(n, 1)
    hashed = nseg * seg + nseg * (k + m) * frag        # leaf-kernel bytes per launch
    achieved = hashed / (k_avg_ms * 1e-3) / 1e9 if k_avg_ms > 0 else 0.0
    kind = ctx.leaf_kernel_for(nseg * (1 + k + m))
    out = {
        "metric": "device-resident GiB/s of object bytes through FullProcessing (RS 4+8, SHA-256 names, fid)",
        "value": round(length * world * args.steps / elapsed / (1 << 30), 4), "unit": "GiB/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32 (SHA-256), u8 (GF(2^8))",
        "data": "synthetic splitmix64 object generated in HBM",
        "config": {"workload": f"{length} B object per GPU -> {nseg} segments of {seg} B -> {k}+{m} fragments "
                               f"of {frag} B, {nseg * (1 + k + m)} SHA-256 leaves in one launch",
                   "object_bytes": length, "segment_bytes": seg, "leaf_kernel": kind,
                   "parallelism": f"{world} x independent"},
        "roofline": {"bound": "hbm", "kernel": f"leaf kernel ({kind}) over segments + fragments",
                     "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                     "leaf_kernel_avg_ms": round(k_avg_ms, 3), "call_avg_ms": round(call_sum / max(n, 1), 3),
                     "algorithmic_bytes_per_launch": hashed,
                     "regime": "latency-bound: one serial SHA-256 chain per 32 MiB segment sets the time"},
        "parity": {"segment_digests": nseg, "fid": bytes(fid.cpu().numpy()).hex(),
                   "fragment_digests_checked_segments": sorted({0, nseg - 1}), "bit_exact": bool(parity_ok)},
    }
    if world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_fp_baseline(orc, host.ctypes.data, length, seg, "the same object")
    return out


def run_fullprocessing(args, torch, dist, world, rank, device, dev_index, gloo):
    """§8f #2 end to end, as every upload handler calls it: FullProcessing(file, "", savedir) on a
    --object-gib file in /dev/shm (page cache) -> fragment and segment files in savedir, fid.  One
    step = one dm_full_processing call (pread into pinned slots, H2D, data-fragment writes while
    reading, one RS + one leaf launch, parity back and written while the leaf chains run, renames).
    Beside it, untimed for the value: the window path (read 8 segments, one dm_process_buffer
    call, write their fragments from Python, repeat: serial, the Python mirror's earlier shape) and
    the same file I/O done from Python alone (read the file, write the same bytes as 8 MiB / 32 MiB
    files, 16 threads, no hashing or coding).
    savedir is emptied (untimed) before every run, so every run writes every file."""
    import shutil
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    from deoss_amd import MerkleContext
    from deoss_amd.process import Processor
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    seg, k, m = 32 << 20, 4, 8
    frag, total = seg // k, k + m
    length = int(args.object_gib * (1 << 30))
    nseg = -(-length // seg)
    out_bytes = nseg * (total * frag + seg)               # fragments + segment files
    orc = Oracle()
    need = length + out_bytes + (1 << 30)
    base = "/dev/shm" if os.path.isdir("/dev/shm") and shutil.disk_usage("/dev/shm").free > need else None
    d = tempfile.mkdtemp(prefix="deoss_fp_", dir=base)
    try:
        path = os.path.join(d, "object.bin")
        piece = torch.empty(64 << 20, dtype=torch.uint8)
        with open(path, "wb") as f:
            for off in range(0, length, 64 << 20):
                n = min(64 << 20, length - off)
                orc.fill_splitmix_ptr(piece.data_ptr(), off, (n + 7) // 8 * 8, SEED + 0x300)
                f.write(piece.numpy()[:n].tobytes())
        del piece
        ctx = MerkleContext(devices=[dev_index])
        proc = Processor(ctx, k, m, seg)
        savedir = os.path.join(d, "cache")

        def fresh():
            shutil.rmtree(savedir, ignore_errors=True)

        for _ in range(args.warmup):
            fresh()
            proc.full_processing_file(path, savedir)
        times = []
        ctx.set_timing(True)
        for _ in range(args.steps):
            fresh()
            t0 = time.perf_counter()
            segd, fragd, fid = proc.full_processing_file(path, savedir)
            times.append(time.perf_counter() - t0)
        n_t, k_sum, _, _ = ctx.timing_summary()
        ctx.set_timing(False)
        tavg = sum(times) / len(times)
        # parity: every segment digest + fid against the CPU restatement over the same bytes, all
        # fragment digests of the first and last segment, the files on disk (names = SHA-256 of
        # their bytes for a sample, exactly the expected set, no temporary left)
        import numpy as np
        host = np.fromfile(path, dtype=np.uint8)
        threads = cpu_share()
        padded = host[(nseg - 1) * seg:].tobytes() + bytes(nseg * seg - length)
        want_seg = orc.root_buffer_ptr(host.ctypes.data, (nseg - 1) * seg, seg, threads, True)[0] if nseg > 1 else b""
        want_seg = (want_seg or b"") + orc.sha256(padded)
        frag_ok = True
        for s_i in sorted({0, nseg - 1}):
            sbytes = padded if s_i == nseg - 1 else host[s_i * seg:(s_i + 1) * seg].tobytes()
            frag_ok &= orc.full_processing(sbytes, seg, k, m, nthreads=threads)[1] == \
                fragd[s_i * total * 32:(s_i + 1) * total * 32]
        del host
        names = set(os.listdir(savedir))
        expect = {fragd[32 * t:32 * t + 32].hex() for t in range(nseg * total)} | \
                 {segd[32 * t:32 * t + 32].hex() for t in range(nseg)}
        sample = sorted(expect)[:8]
        files_ok = names == expect and all(
            hashlib.sha256(open(os.path.join(savedir, n), "rb").read()).hexdigest() == n for n in sample)
        parity = {"fid": fid.hex(), "segment_digests": nseg, "fragment_digests_checked_segments": sorted({0, nseg - 1}),
                  "files_on_disk": len(names), "files_expected": len(expect), "files_hash_checked": len(sample),
                  "bit_exact": bool(segd == want_seg and fid == orc.reduce(want_seg)[:32] and frag_ok and files_ok)}
        # the download handler's question (node/fileHandler.go:962-979): one fragment by its name.
        # dm_fragment_lookup vs the FullProcessing call the handler makes for it; bytes checked
        # against the fragment file FullProcessing just wrote
        if args.no_aux:   # profiling run (tools/profile_extras.sh): the timed calls' kernels only
            return {"metric": "FullProcessing(file) (profiling run, --no-aux)",
                    "value": round(length / tavg / (1 << 30), 4), "unit": "GiB/s", "ms_per_step": round(tavg * 1e3, 3),
                    "parity": parity}
        lookup = {}
        for tag, t_idx in [("last_fragment", nseg * total - 1), ("first_segment_parity", k)]:
            name = fragd[32 * t_idx:32 * t_idx + 32].hex()
            best, got = None, None
            for _ in range(2):
                t0 = time.perf_counter()
                got = proc.fragment_lookup(path, name)
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            with open(os.path.join(savedir, name), "rb") as fh:
                ok = got is not None and got[:2] == (t_idx // total, t_idx % total) and got[2] == fh.read()
            lookup[tag] = {"ms": round(best * 1e3, 1), "speedup_vs_full_processing": round(tavg / best, 2),
                           "bit_exact": bool(ok)}
        parity["fragment_lookup_bit_exact"] = all(v["bit_exact"] for v in lookup.values())
        # the window path, same file, same savedir state
        fresh()
        t0 = time.perf_counter()
        info, wfid, err = proc.FullProcessingWindows(path, "", savedir)
        t_win = time.perf_counter() - t0
        parity["window_path_fid_equal"] = err is None and wfid == fid.hex()
        # the same file I/O from Python alone: read the file, write the same output bytes as files
        fresh()
        os.makedirs(savedir)
        t0 = time.perf_counter()

        def rd(off):
            with open(path, "rb") as f:
                f.seek(off)
                return f.read(min(64 << 20, length - off))

        def wr(i):
            src = blob[(i % (len(blob) // frag)) * frag:][:frag] if i < nseg * total else blob[:seg]   # views
            with open(os.path.join(savedir, f"io{i}"), "wb") as f:
                f.write(src)

        with ThreadPoolExecutor(16) as ex:
            blob = memoryview(b"".join(ex.map(rd, range(0, min(length, 256 << 20), 64 << 20))))
            list(ex.map(rd, range(256 << 20, length, 64 << 20)))
            list(ex.map(wr, range(nseg * total + nseg)))
        t_io = time.perf_counter() - t0
        fresh()
        # the host file-I/O floor in C (tools/io_floor.c): read the file with 4 threads and write
        # the same files with 16 (dm_full_processing's reader / writer counts), nothing else
        floor = None
        exe = os.path.join(ROOT, "tools", "io_floor")
        if not os.path.exists(exe):
            subprocess.run(["gcc", "-O2", "-pthread", "-o", exe, exe + ".c"], check=False)
        if os.path.exists(exe):
            os.makedirs(savedir)
            r = subprocess.run([exe, path, savedir, str(frag), str(nseg * total), str(seg), str(nseg), "4", "16"],
                               capture_output=True, text=True)
            if r.returncode == 0:
                floor = float(r.stdout.strip())
            fresh()
        k_avg = k_sum / max(n_t, 1)
        out = {
            "metric": "GiB/s of a file through FullProcessing(file, \"\", savedir): file -> fragment + segment files, fid",
            "value": round(length / tavg / (1 << 30), 4), "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(tavg * 1e3, 3), "higher_is_better": True,
            "scaling": "none", "vs_baseline": None, "dtype": "u32 (SHA-256), u8 (GF(2^8))",
            "data": f"synthetic splitmix64 file in {'/dev/shm' if base else 'the temp dir'}",
            "config": {"workload": f"1 file of {length} B -> {nseg} segments of {seg} B -> {k}+{m} fragments of "
                                   f"{frag} B; writes {out_bytes} B ({nseg * total} fragment + {nseg} segment files)",
                       "object_bytes": length, "output_bytes": out_bytes},
            "step_ms": [round(t * 1e3, 1) for t in times],
            "leaf_kernel_avg_ms": round(k_avg, 3),
            "fragment_lookup": dict(lookup, what="dm_fragment_lookup: the one fragment the download handler serves, "
                                    "found by name (file read through 64 MiB pinned slots into windows of a quarter file, RS + "
                                    "fragment hashes on the GPU, no files written) instead of FullProcessing + scan"),
            "window_path": {"GiBps": round(length / t_win / (1 << 30), 4), "ms": round(t_win * 1e3, 1),
                            "what": "read 8 segments, dm_process_buffer, write their files from Python, repeat"},
            "host_io_floor": None if floor is None else {
                "GiBps": round(length / floor / (1 << 30), 4), "ms": round(floor * 1e3, 1),
                "frac_of_floor": round(floor / tavg, 4),
                "what": f"tools/io_floor.c: read {length} B (4 threads) + write {out_bytes} B as the same files "
                        "(16 threads); no hashing, coding or GPU"},
            "python_io_only": {"GiBps": round(length / t_io / (1 << 30), 4), "ms": round(t_io * 1e3, 1),
                               "what": f"read {length} B + write {out_bytes} B as the same number of files from "
                                       "Python, 16 threads, no hashing or coding (a host-side reference point)"},
            "parity": parity,
        }
        if not args.no_cpu:
            host = np.fromfile(path, dtype=np.uint8, count=min(length, 64 * seg))
            out["cpu_baseline"] = cpu_fp_baseline(orc, host.ctypes.data, host.size, seg, "the same file")
            del host
        return out
    finally:
        shutil.rmtree(d, ignore_errors=True)


def run_process_upload(args, torch, dist, world, rank, device, dev_index, gloo):
    """§8f #1 + #2: the upload handler's whole flow, body -> file + FullProcessing.  The body
    (--object-gib, synthetic, in host memory) arrives in --piece-kib pieces; the handler writes each
    piece to its file (saveObjectToFile, node/objectHandler.go:248-266) and:
      streamed: hands the same piece to a dm_pstream, and closes it after the last piece (coding,
        hashing and fragment writes happen while the body arrives);
      after:    runs dm_full_processing over the saved file (node/objectHandler.go:168 order).
    One step = the whole flow for one body, files in /dev/shm, savedir emptied (untimed) before
    each run.  Reported: body GiB/s from the first piece to the fid, and the tail after the last
    piece."""
    import shutil
    import tempfile
    from deoss_amd import MerkleContext
    from deoss_amd.process import Processor
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    seg, k, m = 32 << 20, 4, 8
    length = int(args.object_gib * (1 << 30))
    piece = args.piece_kib << 10
    nseg = -(-length // seg)
    orc = Oracle()
    need = 2 * length + nseg * (k + m + 4) * (seg // k) + (1 << 30)
    base = "/dev/shm" if os.path.isdir("/dev/shm") and shutil.disk_usage("/dev/shm").free > need else None
    d = tempfile.mkdtemp(prefix="deoss_pu_", dir=base)
    try:
        body = torch.empty(length, dtype=torch.uint8)
        orc.fill_splitmix_ptr(body.data_ptr(), 0, length // 8 * 8, SEED + 0x400)
        mv = memoryview(body.numpy())
        addr = body.data_ptr()
        ctx = MerkleContext(devices=[dev_index])
        proc = Processor(ctx, k, m, seg)
        fpath, savedir = os.path.join(d, "upload.bin"), os.path.join(d, "cache")

        def fresh():
            shutil.rmtree(savedir, ignore_errors=True)
            if os.path.exists(fpath):
                os.unlink(fpath)

        def pace(t0, off, rate):   # the body arrives at `rate` B/s (None: as fast as the host goes)
            if rate:
                dt = t0 + off / rate - time.perf_counter()
                if dt > 0:
                    time.sleep(dt)

        def streamed(nbytes=length, rate=None):
            t0 = time.perf_counter()
            st = proc.NewProcessingStream(savedir)
            with open(fpath, "wb") as f:
                for off in range(0, nbytes, piece):
                    pace(t0, off, rate)
                    n = min(piece, nbytes - off)
                    f.write(mv[off:off + n])
                    st.write((addr + off, n))
            t_last = time.perf_counter()
            info, fid = st.close()
            t1 = time.perf_counter()
            return t1 - t0, t1 - t_last, fid, st

        def after(nbytes=length, rate=None):
            t0 = time.perf_counter()
            with open(fpath, "wb") as f:
                for off in range(0, nbytes, piece):
                    pace(t0, off, rate)
                    f.write(mv[off:off + min(piece, nbytes - off)])
            t_last = time.perf_counter()
            segd, fragd, fid = proc.full_processing_file(fpath, savedir)
            t1 = time.perf_counter()
            return t1 - t0, t1 - t_last, fid.hex(), (segd, fragd)

        res = {}
        for name, fn in (("streamed", streamed),) + ((("after", after),) if not args.no_aux else ()):
            for _ in range(args.warmup):
                fresh()
                fn()
            runs = []
            for _ in range(args.steps):
                fresh()
                runs.append(fn())
            res[name] = runs
        if args.no_aux:   # profiling run (tools/profile_extras.sh): the streamed flow's kernels only
            tot = sum(r[0] for r in res["streamed"]) / len(res["streamed"])
            return {"metric": "upload body through the streamed handler flow (profiling run, --no-aux)",
                    "value": round(length / tot / (1 << 30), 4), "unit": "GiB/s", "ms_per_step": round(tot * 1e3, 1),
                    "fid": res["streamed"][-1][2]}
        # the same flows with the body arriving at a network link's rate (2 GiB at 1.25 GB/s = 10 GbE)
        link, link_bytes = 1.25e9, min(length, 2 << 30)
        for name, fn in (("streamed_10GbE", streamed), ("after_10GbE", after)):
            runs = []
            for _ in range(max(1, args.steps)):
                fresh()
                runs.append(fn(link_bytes, link))
            res[name] = runs
        s_fid, a_fid = res["streamed"][-1][2], res["after"][-1][2]
        st = res["streamed"][-1][3]
        segd, fragd = res["after"][-1][3]
        # parity: streamed = file form (every digest, the fid); segment digests + fid vs the CPU
        threads = cpu_share()
        host = body.numpy()
        padded = host[(nseg - 1) * seg:].tobytes() + bytes(nseg * seg - length)
        want_seg = orc.root_buffer_ptr(addr, (nseg - 1) * seg, seg, threads, True)[0] if nseg > 1 else b""
        want_seg = (want_seg or b"") + orc.sha256(padded)
        want_fid = orc.reduce(want_seg)[:32].hex()
        parity = {"fid": s_fid, "cpu_fid": want_fid, "segment_digests": nseg,
                  "bit_exact": bool(s_fid == a_fid == want_fid and st.segment_digests == segd == want_seg
                                    and st.fragment_digests == fragd)}
        fresh()

        def summ(runs):
            tot = sum(r[0] for r in runs) / len(runs)
            return {"GiBps": round(length / tot / (1 << 30), 4), "ms": round(tot * 1e3, 1),
                    "tail_ms_after_last_piece": round(sum(r[1] for r in runs) / len(runs) * 1e3, 1),
                    "step_ms": [round(r[0] * 1e3, 1) for r in runs]}

        sv, av = summ(res["streamed"]), summ(res["after"])

        def summ_link(runs):
            tot = sum(r[0] for r in runs) / len(runs)
            return {"GiBps": round(link_bytes / tot / (1 << 30), 4), "ms": round(tot * 1e3, 1),
                    "tail_ms_after_last_piece": round(sum(r[1] for r in runs) / len(runs) * 1e3, 1)}
        cpu = cpu_fp_baseline(orc, addr, length, seg, "the same upload body") if not args.no_cpu else None
        res_line = {
            "metric": "GiB/s of upload body through the handler flow: body -> file + FullProcessing (fid, fragment files)",
            "value": sv["GiBps"], "unit": "GiB/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": sv["ms"], "higher_is_better": True, "scaling": "none", "vs_baseline": None,
            "dtype": "u32 (SHA-256), u8 (GF(2^8))",
            "data": f"synthetic splitmix64 body in host memory, {piece} B pieces, files in "
                    f"{'/dev/shm' if base else 'the temp dir'}",
            "config": {"workload": f"1 body of {length} B -> {nseg} segments; the file is written as the pieces arrive",
                       "object_bytes": length, "piece_bytes": piece},
            "streamed": sv, "after_file_saved": av,
            "at_10GbE": {"body_bytes": link_bytes, "link_GBps": link / 1e9,
                         "streamed": summ_link(res["streamed_10GbE"]), "after_file_saved": summ_link(res["after_10GbE"])},
            "parity": parity,
        }
        if cpu:
            res_line["cpu_baseline"] = cpu
        return res_line
    finally:
        shutil.rmtree(d, ignore_errors=True)


def run_proofs(args, torch, dist, world, rank, device, dev_index, gloo):
    """§8f #4: merkletree proofs on the GPU.  A tree of --objects leaves of --object-mib each
    (default 2^20 x 4 KiB) is built in HBM; one step = verify every leaf's GetMerklePath proof
    (re-hash the leaf content, fold depth node hashes, compare with the root) in one call.
    Also reports the level build and path gather times."""
    from deoss_amd import MerkleContext
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    n = args.objects
    leaf = int(args.object_mib * (1 << 20))
    ctx = MerkleContext(devices=[dev_index])
    sptr = torch.cuda.current_stream().cuda_stream
    obj = torch.empty(n * leaf, dtype=torch.uint8, device=device)
    ctx.fill_synthetic_async(obj.data_ptr(), 0, n * leaf, SEED + 0x300 * (rank + 1), sptr)
    leaves = torch.empty(n * 32, dtype=torch.uint8, device=device)
    root = torch.empty(32, dtype=torch.uint8, device=device)
    ctx.root_device_async(obj.data_ptr(), n * leaf, leaf, root.data_ptr(), leaves.data_ptr(), sptr)
    nodes = torch.empty(ctx.tree_node_count(n) * 32, dtype=torch.uint8, device=device)
    depth = ctx.tree_depth(n)
    idx = torch.arange(n, dtype=torch.int64, device=device)
    paths = torch.empty(n * depth * 32, dtype=torch.uint8, device=device)
    bits = torch.empty(n * depth, dtype=torch.uint8, device=device)
    ok = torch.zeros(n, dtype=torch.uint8, device=device)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.tree_levels_device_async(leaves.data_ptr(), n, nodes.data_ptr(), sptr)
    torch.cuda.synchronize()
    t_levels = time.perf_counter() - t0
    t0 = time.perf_counter()
    ctx.merkle_paths_device_async(leaves.data_ptr(), nodes.data_ptr(), n, idx.data_ptr(), n, paths.data_ptr(),
                                  bits.data_ptr(), sptr)
    torch.cuda.synchronize()
    t_paths = time.perf_counter() - t0
    def step():
        ctx.verify_object_device_async(obj.data_ptr(), n * leaf, leaf, paths.data_ptr(), bits.data_ptr(), depth,
                                       root.data_ptr(), 0, ok.data_ptr(), sptr)

    elapsed, calls, k_sum, call_sum = timed_steps(args, torch, dist, world, device, gloo, ctx, step)
    all_ok = int(ok.sum().item()) == n
    orc = Oracle()
    host = obj.cpu().numpy()
    _, want_root = orc.root_buffer_ptr(host.ctypes.data, n * leaf, leaf, cpu_share())
    root_ok = bytes(root.cpu().numpy()) == want_root and bytes(nodes[-32:].cpu().numpy()) == want_root
    if rank != 0:
        return
    out = {
        "metric": "GetMerklePath proofs verified per second (leaf re-hash + path fold on the GPU)",
        "value": round(n * world * args.steps / elapsed, 1), "unit": "proofs/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic splitmix64 leaves generated in HBM",
        "config": {"workload": f"{n} leaves x {leaf} B, depth {depth}, every leaf's proof per step",
                   "leaves": n, "leaf_bytes": leaf, "depth": depth},
        "levels_ms": round(t_levels * 1e3, 3), "paths_ms": round(t_paths * 1e3, 3),
        "leaf_kernel_avg_ms": round(k_sum / max(calls, 1), 3), "call_avg_ms": round(call_sum / max(calls, 1), 3),
        "leaf_kernel": ctx.leaf_kernel_for(n),
        "content_GiBps": round(n * leaf * world * args.steps / elapsed / (1 << 30), 3),
        "parity": {"all_proofs_verify": all_ok, "root_matches_cpu": root_ok, "bit_exact": all_ok and root_ok},
    }
    return out


def run_concurrent(args, torch, dist, world, rank, device, dev_index, gloo):
    """Upload-gateway regime: --threads caller threads, each blocking on one request at a time
    (NewHashTreeFromBuffer at --chunk, or FullProcessing at 32 MiB segments), --objects requests of
    --object-mib each from host memory.  Timed twice: through the coalescing dm_batcher, and
    through one shared context (what one call per request gives: calls serialise).  Host
    residency and H2D are inside the timed region."""
    import threading
    from deoss_amd import MerkleContext
    from deoss_amd.batcher import PROCESS as B_PROCESS, ROOT as B_ROOT, Batcher
    from deoss_amd.process import Processor
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    obj = int(args.object_mib * (1 << 20))
    nreq = args.objects
    seg = args.segment_mib << 20
    unit = args.chunk if args.mode == "root" else seg
    ctx = MerkleContext(devices=[dev_index])
    pitch = (obj + 4095) // 4096 * 4096
    dev = torch.empty(pitch * nreq, dtype=torch.uint8, device=device)
    for j in range(nreq):
        ctx.fill_synthetic_async(dev.data_ptr() + j * pitch, 0, (obj + 7) // 8 * 8, SEED + 0x400 + j)
    host = dev.cpu().numpy()
    del dev
    base = host.ctypes.data
    outs = [None] * nreq

    def drive(call, n=nreq):
        nxt = [0]
        lock = threading.Lock()

        def worker():
            while True:
                with lock:
                    j = nxt[0]
                    nxt[0] += 1
                if j >= n:
                    return
                outs[j] = call(j)

        th = [threading.Thread(target=worker) for _ in range(args.threads)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        return time.perf_counter() - t0

    res = {}
    if args.mode == "root":
        b = Batcher(B_ROOT, unit, device=dev_index, slots=args.slots, max_leaves=args.max_leaves,
                    linger_us=args.linger_us)
        for _ in range(args.warmup):   # untimed passes: every slot grows its buffers once
            drive(lambda j: b.root((base + j * pitch, obj))[1])
        s0 = b.stats()
        res["batcher"] = drive(lambda j: b.root((base + j * pitch, obj))[1])
        stats = [x - y for x, y in zip(b.stats(), s0)]
        stats[2] = b.stats()[2]
        b.close()
        got = list(outs)
        if not args.no_shared:   # serialised: time a sample of requests and scale
            sample = max(1, min(nreq, 256))
            res["shared_context"] = drive(lambda j: ctx.root_buffer_ptr(base + j * pitch, obj, unit)[1],
                                          sample) * nreq / sample
    else:
        b = Batcher(B_PROCESS, unit, 4, 8, device=dev_index, slots=args.slots, max_leaves=args.max_leaves,
                    linger_us=args.linger_us)
        for _ in range(args.warmup):
            drive(lambda j: b.process((base + j * pitch, obj))[2])
        s0 = b.stats()
        res["batcher"] = drive(lambda j: b.process((base + j * pitch, obj))[2])
        stats = [x - y for x, y in zip(b.stats(), s0)]
        stats[2] = b.stats()[2]
        b.close()
        got = list(outs)
        proc = Processor(ctx, 4, 8, unit)
        import ctypes as _ct
        sample = max(1, min(nreq, 8))

        def one(j):
            src = (_ct.c_char * obj).from_address(base + j * pitch)
            return proc.process_buffer(src, want_frags=False)[2]
        # the serialised path is slow: time a sample of requests and scale
        if not args.no_shared:
            res["shared_context"] = drive(one, sample) * nreq / sample
    # every request's result against the CPU oracle (the job's CPU share, untimed)
    from concurrent.futures import ThreadPoolExecutor
    orc = Oracle()

    def want_of(j):
        addr = base + j * pitch
        if args.mode == "root":
            return orc.root_buffer_ptr(addr, obj, unit, nthreads=1)[1]
        return orc.full_processing_ptr(addr, obj, unit, 4, 8, nthreads=1)[2]

    with ThreadPoolExecutor(cpu_share()) as pool:
        wants = list(pool.map(want_of, range(nreq)))
    check = nreq
    mism = sum(wants[j] != got[j] for j in range(nreq))
    total = obj * nreq
    out = {
        "metric": ("host-resident GiB/s of uploads hashed to Merkle roots by concurrent callers" if args.mode == "root"
                   else "host-resident GiB/s of uploads through FullProcessing by concurrent callers"),
        "value": round(total / res["batcher"] / (1 << 30), 4), "unit": "GiB/s", "n_gpus": 1,
        "steps": 1, "warmup": args.warmup, "ms_per_step": round(res["batcher"] * 1e3, 3), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic splitmix64 objects in host memory",
        "config": {"workload": f"{nreq} requests x {obj} B from {args.threads} threads, "
                               f"{'chunk' if args.mode == 'root' else 'segment'} {unit} B ({args.mode})",
                   "threads": args.threads, "requests": nreq, "object_bytes": obj, "unit": unit},
        "batcher": {"seconds": round(res["batcher"], 4), "requests": stats[0], "batches": stats[1],
                    "largest_batch": stats[2], "slots": args.slots or 2, "max_leaves": args.max_leaves or 4096,
                    "linger_us": args.linger_us},
        "parity": {"checked": check, "mismatches": int(mism), "bit_exact": mism == 0},
    }
    if "shared_context" in res:
        out["shared_context"] = {"seconds": round(res["shared_context"], 4),
                                 "GiBps": round(total / res["shared_context"] / (1 << 30), 4),
                                 "note": "one dm_ctx for all threads: calls serialise (timed on a sample of "
                                         "256 (root) / 8 (process) requests, scaled)"}
        out["speedup_vs_shared_context"] = round(res["shared_context"] / res["batcher"], 2)
    return out


def run_batch(args, torch, dist, world, rank, device, dev_index, gloo):
    """configs[2] (batch: objects already in HBM) and configs[4] (stream: objects in host memory,
    pinned staging + H2D inside the timed region).  Objects are split across ranks with no
    exchange (each object's tree is independent)."""
    from deoss_amd import MerkleContext
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    obj = int(args.object_mib * (1 << 20))
    if args.total_objects:   # replicas: rank r takes objects [T*r/N, T*(r+1)/N), no exchange
        nobj = args.total_objects * (rank + 1) // world - args.total_objects * rank // world
    else:
        nobj = args.objects
    chunk = args.chunk
    ctx = MerkleContext(devices=[dev_index])
    ctx.set_leaf_kernel(args.leaf_kernel)
    sptr = torch.cuda.current_stream().cuda_stream
    first = args.total_objects * rank // world if args.total_objects else rank * nobj
    seed0 = SEED + 1000 + first     # object g of the whole job: its own splitmix64 stream
    total_local = obj * nobj
    pitch = (obj + 255) // 256 * 256
    buf = torch.empty(pitch * nobj + 64, dtype=torch.uint8, device=device)
    for j in range(nobj):   # object j of this rank: splitmix64 stream with its own seed
        ctx.fill_synthetic_async(buf.data_ptr() + j * pitch, 0, (obj + 7) // 8 * 8, seed0 + j, sptr)
    ptrs = [buf.data_ptr() + j * pitch for j in range(nobj)]
    lens = [obj] * nobj
    roots = torch.zeros(32 * nobj, dtype=torch.uint8, device=device)
    host = None
    if args.workload == "stream":
        host = torch.empty(pitch * nobj, dtype=torch.uint8, pin_memory=True)
        host.copy_(buf[:pitch * nobj])
        torch.cuda.synchronize()
        del buf
        import ctypes
        hptrs = [host.data_ptr() + j * pitch for j in range(nobj)]

        def step():
            n = len(hptrs)
            P = (ctypes.c_void_p * n)(*hptrs)
            L = (ctypes.c_uint64 * n)(*lens)
            out = ctypes.create_string_buffer(32 * n)
            ctx._check(ctx._L.dm_root_batch(ctx._h, P, L, n, chunk, out), "dm_root_batch")
            return out.raw
    else:
        def step():
            ctx.root_batch_device_async(ptrs, lens, chunk, roots.data_ptr(), sptr)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier() if gloo else dist.barrier(device_ids=[dev_index])
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    last = None
    for _ in range(args.steps):
        last = step()
    barrier()
    t1 = time.perf_counter()
    ncalls, k1_ms_sum, call_ms_sum, _ = ctx.timing_summary()
    ctx.set_timing(False)
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if gloo else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    got = last if args.workload == "stream" else bytes(roots.cpu().numpy())
    # parity: EVERY root of this rank against the CPU oracle (the job's CPU share, untimed).  The
    # device-resident objects are copied back once and hashed from host memory; the generator
    # itself is checked on a sample of objects against the oracle's independent splitmix64.
    from concurrent.futures import ThreadPoolExecutor
    from oracle import Oracle
    orc = Oracle()
    gen_checked = gen_bad = 0
    if host is None:
        host = torch.empty(pitch * nobj, dtype=torch.uint8, pin_memory=True)
        host.copy_(buf[:pitch * nobj])
        torch.cuda.synchronize()
        del buf
        hv = host.numpy()
        for j in sorted({0, nobj // 3, nobj // 2, nobj - 1}):
            gen_checked += 1
            gen_bad += bytes(hv[j * pitch:j * pitch + obj]) != orc.splitmix_bytes(obj, seed0 + j)
    base = host.data_ptr()

    def want_root(j):
        return orc.root_buffer_ptr(base + j * pitch, obj, chunk, nthreads=1)[1]

    t0 = time.perf_counter()
    with ThreadPoolExecutor(cpu_share()) as pool:
        wants = list(pool.map(want_root, range(nobj)))
    par_s = time.perf_counter() - t0
    ns = min(nobj, 64)
    t0 = time.perf_counter()
    for j in range(ns):
        want_root(j)
    ser_s = time.perf_counter() - t0
    check = nobj
    mism = sum(wants[j] != got[32 * j:32 * j + 32] for j in range(nobj)) + gen_bad
    leaves = (obj + chunk - 1) // chunk * nobj
    kind = ctx.leaf_kernel_for(leaves)
    out = {
        "metric": "device-resident GiB/s hashed to Merkle root; 1/2/4/8 MI355X scaling" if args.workload == "batch"
        else "host-resident GiB/s hashed to Merkle roots (pinned H2D inside the timed region)",
        "value": round((obj * args.total_objects if args.total_objects else total_local * world) * args.steps
                       / elapsed / (1 << 30), 4), "unit": "GiB/s",
        "n_gpus": 1 if args.same_device else world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong" if args.total_objects else "weak",
        "vs_baseline": None, "dtype": "u32", "data": "synthetic splitmix64 objects",
        "config": {"workload": (f"{args.total_objects} objects x {obj} B over {world} rank(s) ({args.workload}), "
                                f"chunk {chunk}" if args.total_objects else
                                f"{nobj} objects x {obj} B per GPU ({args.workload}), chunk {chunk}"),
                   "objects_per_gpu": nobj, "object_bytes": obj, "chunk": chunk, "leaf_kernel": kind,
                   "parallelism": f"{world} replica(s), objects split across ranks, no exchange"},
        "k1_avg_ms": round(k1_ms_sum / max(ncalls, 1), 4), "call_avg_ms": round(call_ms_sum / max(ncalls, 1), 4),
        "parity": {"checked_objects": check, "objects": nobj, "mismatches": int(mism), "bit_exact": mism == 0,
                   "generator_sample_checked": gen_checked},
        "cpu_baseline": {"value": round(ns * obj / ser_s / (1 << 30), 4), "unit": "GiB/s", "cores": 1, "kind": "port",
                         "sample": f"{ns} of the same objects, one after another (oracle/merkle_oracle.c, SHA-NI)",
                         "parallel": {"value": round(total_local / par_s / (1 << 30), 4), "cores": cpu_share(),
                                      "sample": f"all {nobj} objects of this rank, one per thread at a time"}},
    }
    if args.same_device:
        out.update({"ranks": world, "same_device": True,
                    "note": "rehearsal: every rank on cuda:0 of one GPU; not a multi-GPU result"})
    if world > 1:   # every rank's roots were checked against the CPU: report all ranks' mismatches
        t = torch.tensor([mism, check], dtype=torch.int64, device="cpu" if gloo else device)
        dist.all_reduce(t)
        out["parity"] = {"checked_objects": int(t[1]), "mismatches": int(t[0]), "bit_exact": int(t[0]) == 0,
                         "ranks": world}
    if world > 1:
        barrier()
    return out if rank == 0 else None
