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

from deoss_amd.sharding import parity_prefix, plan_shards, sharded_root
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


def _prefix_worker(rank, world, port, cases, results):
    """bench.py's N>1 parity plan on gloo: every rank regenerates ONLY its slice of the object (at
    its byte offset) for the timed root, then its slice of the parity prefix; rank 0 checks the
    sharded roots against a one-rank root of the prefix and the leaf-by-leaf CPU root."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import Oracle
    orc = Oracle()
    try:
        for (total, chunk, seed, cap) in cases:
            def run(length):
                plan = plan_shards(length, chunk, world)
                b0, b1 = plan.byte_range(rank)
                local = orc.splitmix_bytes(b1 - b0, seed, off=b0) if b1 > b0 else b""

                def subtree(k):
                    if not local:
                        return torch.zeros(0, dtype=torch.uint8)
                    lv, _ = orc.root_buffer(local, chunk)
                    nodes = orc.reduce(lv, k) if k else lv
                    return torch.frombuffer(bytearray(nodes), dtype=torch.uint8)

                def finish(nodes, n, min_one):
                    raw = bytes(nodes.numpy())[:32 * n]
                    out = orc.reduce(raw)[:32] if (min_one or n > 1) else raw
                    return torch.frombuffer(bytearray(out), dtype=torch.uint8)
                r = sharded_root(plan, rank, subtree, finish, torch, dist, "cpu")
                return bytes(r.numpy()) if rank == 0 else None
            timed = run(total)
            prefix = parity_prefix(total, chunk, cap)
            sharded_prefix = timed if prefix == total else run(prefix)
            if rank == 0:
                single = orc.root_buffer(orc.splitmix_bytes(prefix, seed), chunk)[1]
                cpu = orc.root_synthetic(total, chunk, seed, nthreads=2)[1]
                results.append((total, chunk, prefix, timed == cpu, sharded_prefix == single))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_multi_rank_parity_plan_gloo(world):
    cases = [(1 << 20, 4096, 11, 1 << 20),          # prefix = whole object
             (1 << 20, 4096, 12, 300 * 1024),       # prefix shorter than the object (the 1 TiB case)
             ((777 << 10) + 64, 1 << 14, 13, 100 << 10),
             (64 * 1000 + 8, 64, 14, 4096)]
    mgr = mp.Manager()
    results = mgr.list()
    mp.spawn(_prefix_worker, args=(world, _free_port(), cases, results), nprocs=world, join=True)
    assert len(results) == len(cases)
    for total, chunk, prefix, cpu_ok, prefix_ok in results:
        assert cpu_ok and prefix_ok, (world, total, chunk, prefix)
    assert parity_prefix(1 << 40, 32 << 20, 64 << 30) == 64 << 30
    assert parity_prefix(64 << 30, 32 << 20, 64 << 30) == 64 << 30
    assert parity_prefix((64 << 30) + 5, 3 << 20, 64 << 30) == (64 << 30) // (3 << 20) * (3 << 20)


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
    # BASELINE configs[3]: 1 TiB over 8 ranks -> 4,096 leaves (128 GiB) per rank, one 2^12 block each
    plan = plan_shards(1 << 40, 32 << 20, 8)
    assert plan.k == 12 and plan.n_blocks == 8
    assert all(plan.byte_range(r) == (r << 37, (r + 1) << 37) for r in range(8))


def _exchange_worker(rank, world, port, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        import bench
        plan = plan_shards(world * (8 << 30), 32 << 20, world)      # the weak-scaling headline's layout
        r = bench.measure_exchange(plan, torch, dist, "cpu", True, dist.barrier, reps=20)
        if rank == 0:
            results.append(r)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_exchange_timing_gloo(world):
    """bench.measure_exchange (the N > 1 line's `exchange`): the headline's all-gather alone, on
    every rank, max over ranks -- one 32-byte subtree root per rank at the weak-scaling layout."""
    mgr = mp.Manager()
    results = mgr.list()
    mp.spawn(_exchange_worker, args=(world, _free_port(), results), nprocs=world, join=True)
    (r,) = list(results)
    assert r["bytes_per_rank"] == 32 and r["ranks"] == world and r["reps"] == 20
    assert r["backend"] == "gloo" and 0 < r["avg_us"] < 1e6
