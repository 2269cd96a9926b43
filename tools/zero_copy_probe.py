"""Experiment: can the latency-bound leaf kernels read the object straight from pinned host
memory (zero-copy over PCIe) at the chain rate?  256 chains need ~17 GB/s of reads, a third of
PCIe.  Times dm_root_device_async on a pinned host pointer against the same bytes in HBM, and
checks the roots agree.  Run on the GPU box: python tools/zero_copy_probe.py"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    import torch
    from deoss_amd import MerkleContext
    ctx = MerkleContext(devices=[0])
    s = torch.cuda.current_stream()
    sp = s.cuda_stream
    for total, chunk, reps, mode in ((8 << 30, 32 << 20, 3, "auto"), (8 << 30, 1 << 20, 3, "auto"),
                                     (8 << 30, 512 << 10, 3, "auto"), (8 << 30, 512 << 10, 3, "latency"),
                                     (8 << 30, 512 << 10, 3, "pair"), (2 << 30, 64 << 10, 2, "wide")):
        ctx.set_leaf_kernel(mode)
        dev = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        ctx.fill_synthetic_async(dev.data_ptr(), 0, total, 0xDE0550002, sp)
        host = torch.empty(total + 64, dtype=torch.uint8, pin_memory=True)
        host.copy_(dev)
        torch.cuda.synchronize()
        res = {}
        for name, ptr in (("hbm", dev.data_ptr()), ("pinned_host", host.data_ptr())):
            r = torch.zeros(32, dtype=torch.uint8, device="cuda")
            ctx.root_device_async(ptr, total, chunk, r.data_ptr(), 0, sp)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.root_device_async(ptr, total, chunk, r.data_ptr(), 0, sp)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / reps
            res[name] = (bytes(r.cpu().numpy()).hex(), dt)
            print(f"{total >> 20} MiB chunk {chunk >> 10} KiB {ctx.leaf_kernel_for(total // chunk):7s} {name:12s} {dt * 1e3:9.2f} ms  "
                  f"{total / dt / (1 << 30):8.2f} GiB/s  root {res[name][0][:16]}", flush=True)
        print("roots equal:", res["hbm"][0] == res["pinned_host"][0], flush=True)
        del dev, host
        torch.cuda.empty_cache()
    ctx.set_leaf_kernel("auto")
    # table mode: configs[4]'s per-GPU share, 12,500 one-leaf objects of 1 MiB
    nobj, size = 12500, 1 << 20
    dev = torch.empty(nobj * size + 64, dtype=torch.uint8, device="cuda")
    ctx.fill_synthetic_async(dev.data_ptr(), 0, nobj * size, 7, sp)
    host = torch.empty(nobj * size + 64, dtype=torch.uint8, pin_memory=True)
    host.copy_(dev)
    torch.cuda.synchronize()
    roots = {}
    for name, base in (("hbm", dev.data_ptr()), ("pinned_host", host.data_ptr())):
        r = torch.zeros(nobj * 32, dtype=torch.uint8, device="cuda")
        ptrs = [base + i * size for i in range(nobj)]
        ctx.root_batch_device_async(ptrs, [size] * nobj, 32 << 20, r.data_ptr(), sp)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            ctx.root_batch_device_async(ptrs, [size] * nobj, 32 << 20, r.data_ptr(), sp)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 3
        roots[name] = bytes(r.cpu().numpy())
        print(f"batch {nobj} x 1 MiB ({ctx.leaf_kernel_for(nobj)}) {name:12s} {dt * 1e3:9.2f} ms  "
              f"{nobj * size / dt / (1 << 30):8.2f} GiB/s", flush=True)
    print("batch roots equal:", roots["hbm"] == roots["pinned_host"], flush=True)


if __name__ == "__main__":
    main()
