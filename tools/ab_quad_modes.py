"""A/B helper: K1Q leaf-kernel time for one 4096-leaf object in uniform mode with fused levels,
uniform mode without fusion (subtree, 0 levels) and table mode (batch of 4096 objects)."""
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from deoss_amd import MerkleContext

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 2 << 20
ctx = MerkleContext()
buf = torch.empty(n * chunk + 64, dtype=torch.uint8, device="cuda")
ctx.fill_synthetic_async(buf.data_ptr(), 0, n * chunk, 7)
root = torch.empty(32, dtype=torch.uint8, device="cuda")
nodes = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
roots = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
ptrs = [buf.data_ptr() + i * chunk for i in range(n)]


def timed(f, reps=3):
    f()
    torch.cuda.synchronize()
    ctx.set_timing(True)
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    c, k, _, _ = ctx.timing_summary()
    ctx.set_timing(False)
    return k / c


print("uniform+fuse", timed(lambda: ctx.root_device_async(buf.data_ptr(), n * chunk, chunk, root.data_ptr())))
print("uniform k=0 ", timed(lambda: ctx.subtree_device_async(buf.data_ptr(), n * chunk, chunk, 0, nodes.data_ptr())))
print("table       ", timed(lambda: ctx.root_batch_device_async(ptrs, [chunk] * n, chunk, roots.data_ptr())))
# order check: does a uniform launch right after a batch (K3) run slow too?
ctx.set_timing(True)
ctx.root_batch_device_async(ptrs, [chunk] * n, chunk, roots.data_ptr())
ctx.subtree_device_async(buf.data_ptr(), n * chunk, chunk, 0, nodes.data_ptr())
torch.cuda.synchronize()
print("note: per-call leaf ms after a batch:", ctx.timing_summary())
ctx.set_timing(False)
