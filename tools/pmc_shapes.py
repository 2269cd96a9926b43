"""The leaf-kernel launch shapes of every N > 1 bench leg's per-rank work, run in ONE process so
one rocprofv3 --pmc pass per counter covers them all (tools/pmc_traffic.py then gives per-launch
HBM bytes by kernel and grid, merged into profiles/k1_traffic.json, which bench.py's
roofline.traffic reads): configs[3]'s 128 GiB share (4,096 leaves of 32 MiB), the strong legs'
per-rank shares at N = 2 / 4 / 8 (configs[1]'s 8 GiB split: 4 / 2 / 1 GiB at 32 MiB and at 4 KiB
chunks).  The weak headline's 8 GiB share is the N = 1 headline's launch (profiled by
tools/profile_bench.sh).  Every shape: two device-resident roots over a prefix of one synthetic
object (the bench's generator and seed).
usage (GPU box): rocprofv3 --pmc FETCH_SIZE -d <dir> -o fetch --output-format csv -- python3 tools/pmc_shapes.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = [(128 << 30, 32 << 20), (4 << 30, 32 << 20), (2 << 30, 32 << 20), (1 << 30, 32 << 20),
          (4 << 30, 4096), (2 << 30, 4096), (1 << 30, 4096)]


def main():
    import torch
    from bench_common import SEED
    from deoss_amd import MerkleContext
    biggest = max(n for n, _ in SHAPES)
    buf = torch.empty(biggest + 64, dtype=torch.uint8, device="cuda:0")
    root = torch.zeros(32, dtype=torch.uint8, device="cuda:0")
    with MerkleContext(devices=[0]) as ctx:
        s = torch.cuda.current_stream().cuda_stream
        ctx.fill_synthetic_async(buf.data_ptr(), 0, biggest, SEED, s)
        for n, chunk in SHAPES:
            for _ in range(2):
                ctx.root_device_async(buf.data_ptr(), n, chunk, root.data_ptr(), 0, s)
            torch.cuda.synchronize()
            print(f"{n} B at chunk {chunk}: {(n + chunk - 1) // chunk} leaves, kernel "
                  f"{ctx.leaf_kernel_for((n + chunk - 1) // chunk)}, root {bytes(root.cpu().numpy()).hex()}",
                  flush=True)


if __name__ == "__main__":
    main()
