"""CPU tests of the multi-rank path (deoss_amd.sharding) with torch.distributed gloo.

The per-rank compute is a CPU test double built on the oracle (this container has no GPU); what
is under test is the product's partition plan, the fixed-slot all-gather exchange and the
rank-0 finish ordering.  The same sharded_root() drives RCCL on the GPU box (bench.py).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deoss_amd.sharding import plan_shards, sharded_root
from oracle import py_reduce, py_root_chunks, split_chunks, splitmix64_bytes


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cases, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for (length, chunk, seed) in cases:
            buf = splitmix64_bytes(length, seed)
            plan = plan_shards(length, chunk, world)
            b0, b1 = plan.byte_range(rank)
            local = buf[b0:b1]

            def subtree(k, local=local, chunk=chunk):
                if not local:
                    return torch.zeros(0, dtype=torch.uint8)
                import hashlib
                leaves = [hashlib.sha256(c).digest() for c in split_chunks(local, chunk)]
                nodes = py_reduce(leaves, k)
                return torch.frombuffer(bytearray(b"".join(nodes)), dtype=torch.uint8)

            def finish(nodes, n, min_one):
                raw = bytes(nodes.numpy())
                lst = [raw[32 * i:32 * i + 32] for i in range(n)]
                out = py_reduce(lst) if (min_one or n > 1) else lst
                return torch.frombuffer(bytearray(out[0]), dtype=torch.uint8)

            root = sharded_root(plan, rank, subtree, finish, torch, dist, "cpu")
            if rank == 0:
                results.append((length, chunk, seed, bytes(root.numpy())))
    finally:
        dist.destroy_process_group()


CASES = [(1000 * 64 + 5, 64, 1), (64 * 1024, 1024, 2), (3000, 1000, 3), (5 * 64, 64, 4), (100, 64, 5),
         (256 * 4096, 4096, 6), (33 * 128, 128, 7)]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_root_gloo(world):
    mgr = mp.Manager()
    results = mgr.list()
    port = _free_port()
    mp.spawn(_worker, args=(world, port, CASES, results), nprocs=world, join=True)
    assert len(results) == len(CASES)
    for length, chunk, seed, got in results:
        _, want = py_root_chunks(split_chunks(splitmix64_bytes(length, seed), chunk))
        assert got == want, (world, length, chunk)


def test_plan_properties():
    for world in (1, 2, 3, 4, 8):
        for n in (1, 2, 3, 7, 8, 255, 256, 257, 1000, 4096, 32768):
            plan = plan_shards(n * 4096 - 1, 4096, world)
            assert plan.n_leaves == n
            covered = []
            for r in range(world):
                l0, l1 = plan.leaf_range(r)
                assert l0 % (1 << plan.k) == 0           # aligned block start
                covered.extend(range(l0, l1))
            assert covered == list(range(n))
            assert sum(plan.node_count(r) for r in range(world)) == plan.n_blocks
    # the bench's weak-scaling layout: 256 leaves per rank -> one block of 2^8 per rank
    plan = plan_shards(8 * (8 << 30), 32 << 20, 8)
    assert plan.k == 8 and plan.n_blocks == 8 and all(plan.node_count(r) == 1 for r in range(8))
