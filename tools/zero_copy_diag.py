"""Diagnose the zero-copy host paths on the GPU box: pointer queries on a torch pinned buffer,
then dm_root_buffer (8 GiB @ 32 MiB, 8 GiB @ 1 MiB) and dm_root_batch (12,500 x 1 MiB) from
pinned memory, timed.  Run once with DEOSS_ZERO_COPY=0 and once without to compare."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from deoss_amd import MerkleContext
    zc = os.environ.get("DEOSS_ZERO_COPY", "1")
    ctx = MerkleContext(devices=[0])
    hip = ctypes.CDLL("libamdhip64.so")
    total = 8 << 30
    alloc = 12500 << 20    # the batch below reads 12,500 x 1 MiB
    host = torch.empty(alloc + 64, dtype=torch.uint8, pin_memory=True)
    dev = torch.empty(alloc + 64, dtype=torch.uint8, device="cuda")
    ctx.fill_synthetic_async(dev.data_ptr(), 0, alloc, 3, 0)
    host.copy_(dev)
    torch.cuda.synchronize()
    del dev
    dp = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(dp), ctypes.c_void_p(host.data_ptr()), ctypes.c_uint(0))
    print(f"[zc={zc}] host {host.data_ptr():#x} hipHostGetDevicePointer rc={rc} dev={dp.value or 0:#x}", flush=True)
    for chunk in (32 << 20, 1 << 20):
        ctx.root_buffer_ptr(host.data_ptr(), total, chunk)
        t0 = time.perf_counter()
        for _ in range(2):
            _, r = ctx.root_buffer_ptr(host.data_ptr(), total, chunk)
        dt = (time.perf_counter() - t0) / 2
        print(f"[zc={zc}] root_buffer pinned 8 GiB chunk {chunk >> 20} MiB: {dt * 1e3:.1f} ms "
              f"{total / dt / (1 << 30):.2f} GiB/s root {r.hex()[:16]}", flush=True)
    nobj, size = 12500, 1 << 20
    P = (ctypes.c_void_p * nobj)(*[host.data_ptr() + i * size for i in range(nobj)])
    L = (ctypes.c_uint64 * nobj)(*([size] * nobj))
    out = ctypes.create_string_buffer(32 * nobj)
    ctx._check(ctx._L.dm_root_batch(ctx._h, P, L, nobj, 32 << 20, out), "dm_root_batch")
    t0 = time.perf_counter()
    for _ in range(2):
        ctx._check(ctx._L.dm_root_batch(ctx._h, P, L, nobj, 32 << 20, out), "dm_root_batch")
    dt = (time.perf_counter() - t0) / 2
    import hashlib
    print(f"[zc={zc}] root_batch pinned {nobj} x 1 MiB: {dt * 1e3:.1f} ms {nobj * size / dt / (1 << 30):.2f} GiB/s "
          f"roots sha {hashlib.sha256(out.raw).hexdigest()[:16]}", flush=True)
    for nobj in (4096, 8192, 10000):
        t0 = time.perf_counter()
        ctx._check(ctx._L.dm_root_batch(ctx._h, P, L, nobj, 32 << 20, out), "dm_root_batch")
        dt = time.perf_counter() - t0
        print(f"[zc={zc}] root_batch pinned {nobj} x 1 MiB: {dt * 1e3:.1f} ms {nobj * size / dt / (1 << 30):.2f} GiB/s",
              flush=True)


if __name__ == "__main__":
    main()
