"""Diagnose subtree/finish on one device against the oracle (GPU box debugging aid)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402
import numpy as np  # noqa: E402
from deoss_amd import MerkleContext  # noqa: E402
from oracle import Oracle, split_chunks  # noqa: E402

orc = Oracle()
ctx = MerkleContext()
s = torch.cuda.current_stream().cuda_stream


def dev(b):
    t = torch.zeros(len(b) + 64, dtype=torch.uint8, device="cuda")
    t[:len(b)] = torch.from_numpy(np.frombuffer(b, dtype=np.uint8).copy()).cuda()
    return t


for (length, chunk, levels) in [(65536, 1024, 5), (32768, 1024, 5), (32 * 64, 64, 5), (64 * 64, 64, 5),
                                 (65536, 1024, 6), (65536, 1024, 4), (65536, 1024, 1)]:
    host = orc.splitmix_bytes(length, 7)
    leaves = orc.root_buffer(host, chunk)[0]
    want_nodes = orc.reduce(leaves, levels)
    t = dev(host)
    n_nodes = len(want_nodes) // 32
    out = torch.zeros(max(n_nodes, 1) * 32, dtype=torch.uint8, device="cuda")
    cnt = ctx.subtree_device_async(t.data_ptr(), length, chunk, levels, out.data_ptr(), s)
    torch.cuda.synchronize()
    got = bytes(out.cpu().numpy())
    print(f"subtree len={length} chunk={chunk} levels={levels}: cnt={cnt} want={n_nodes} ok={got == want_nodes}")
    # finish over the oracle's nodes
    nodes_dev = dev(want_nodes)
    root = torch.zeros(32, dtype=torch.uint8, device="cuda")
    ctx.finish_device_async(nodes_dev.data_ptr(), n_nodes, False, root.data_ptr(), s)
    torch.cuda.synchronize()
    want_root = orc.reduce(want_nodes, -1) if n_nodes > 1 else want_nodes
    print(f"   finish n={n_nodes}: ok={bytes(root.cpu().numpy()) == want_root[:32]}")
