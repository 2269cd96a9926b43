"""Multi-GPU sharding of one object by aligned chunk ranges (DESIGN.md "C1").

One process per GPU.  The object's n leaves are cut into blocks of S = 2^k leaves; each rank
owns a contiguous range of blocks, hashes its leaves and reduces them for exactly k levels with
the merkletree v0.2.0 rule.  Because every block starts at a multiple of 2^k, the parity of the
last block's level size equals the parity of the global level size at every level below k, so
the per-rank nodes are exactly the global tree's level-k nodes (the odd-node duplication only
ever touches the global last node, which lives in the last block).  One all-gather of the
32-byte level-k nodes (RCCL over xGMI on the GPU, gloo in the CPU tests) then lets rank 0 run
the final levels.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple


def _ceil_shift(n: int, k: int) -> int:
    return (n + (1 << k) - 1) >> k


@dataclass(frozen=True)
class ShardPlan:
    length: int          # object bytes
    chunk: int           # chunk (leaf) size
    world: int           # ranks
    k: int               # levels each rank reduces (block = 2^k leaves)
    n_leaves: int
    n_blocks: int

    def blocks(self, r: int) -> Tuple[int, int]:
        return self.n_blocks * r // self.world, self.n_blocks * (r + 1) // self.world

    def leaf_range(self, r: int) -> Tuple[int, int]:
        b0, b1 = self.blocks(r)
        return min(self.n_leaves, b0 << self.k), min(self.n_leaves, b1 << self.k)

    def byte_range(self, r: int) -> Tuple[int, int]:
        l0, l1 = self.leaf_range(r)
        return min(self.length, l0 * self.chunk), min(self.length, l1 * self.chunk)

    def node_count(self, r: int) -> int:
        l0, l1 = self.leaf_range(r)
        return _ceil_shift(l1 - l0, self.k) if l1 > l0 else 0

    @property
    def max_nodes(self) -> int:
        return max(self.node_count(r) for r in range(self.world))


def plan_shards(length: int, chunk: int, world: int) -> ShardPlan:
    """The library's partition rule (deoss_amd/csrc/shard_plan.hpp dm_plan::plan_shards, exported as
    dm_plan_shards; tests/test_dispatch_plan.py checks both agree): k = the largest block size that
    keeps every rank within 1/8 of an even split of the leaves and gives every rank at least one
    block (k = 0 when n < world), never more than ceil(log2 n) levels."""
    if length <= 0 or chunk <= 0 or world <= 0:
        raise ValueError("length, chunk and world must be positive")
    n = (length + chunk - 1) // chunk
    even = (n + world - 1) // world
    best = 0
    k = 0
    while k < 63 and (k == 0 or (1 << (k - 1)) < n):
        nb = _ceil_shift(n, k)
        if nb < world:
            break
        plan = ShardPlan(length=length, chunk=chunk, world=world, k=k, n_leaves=n, n_blocks=nb)
        if 8 * max(l1 - l0 for l0, l1 in (plan.leaf_range(r) for r in range(world))) <= 9 * even:
            best = k
        k += 1
    return ShardPlan(length=length, chunk=chunk, world=world, k=best, n_leaves=n, n_blocks=_ceil_shift(n, best))


def parity_prefix(length: int, chunk: int, cap_bytes: int) -> int:
    """Bytes of the prefix the multi-GPU parity leg re-roots on one GPU: the whole object when it
    fits in cap_bytes, else the largest whole-chunk prefix that does (bench.py multi_rank_parity;
    SURVEY.md 8d config 4: "vs the single-GPU root on a <= 64 GiB prefix")."""
    if length <= cap_bytes:
        return length
    p = cap_bytes // chunk * chunk
    if p <= 0:
        raise ValueError("prefix cap smaller than one chunk")
    return p


def sharded_root(plan: ShardPlan, rank: int, local_subtree: Callable[[int], "object"],
                 finish: Callable[["object", int, bool], "object"], torch_mod, dist_mod,
                 device, group=None, comm_device=None):
    """Run one sharded root computation.

    local_subtree(k) -> uint8 tensor of this rank's level-k nodes (node_count(rank) * 32 bytes)
    finish(nodes, n, min_one_level) -> 32-byte root tensor (rank 0 only)
    Returns the root tensor on rank 0 and None elsewhere.  The only data exchange is one
    all_gather_into_tensor of fixed-size slots (max_nodes * 32 bytes per rank).
    comm_device: where the exchange buffers live (default: device; "cpu" for a gloo group).
    """
    comm = device if comm_device is None else comm_device
    slot = plan.max_nodes * 32
    mine = local_subtree(plan.k)
    cnt = plan.node_count(rank)
    if cnt * 32 == slot and str(comm) == str(device):
        send = mine[:slot]
    else:
        send = torch_mod.zeros(slot, dtype=torch_mod.uint8, device=comm)
        if cnt:
            send[:cnt * 32] = mine[:cnt * 32].to(comm)
    gathered = torch_mod.empty(plan.world * slot, dtype=torch_mod.uint8, device=comm)
    dist_mod.all_gather_into_tensor(gathered, send, group=group)
    if rank != 0:
        return None
    counts = [plan.node_count(r) for r in range(plan.world)]
    if all(c * 32 == slot for c in counts):
        nodes = gathered             # every slot full (one block per rank, the bench layouts): no copy
    else:
        parts: List = [gathered[r * slot:r * slot + c * 32] for r, c in enumerate(counts) if c]
        nodes = parts[0] if len(parts) == 1 else torch_mod.cat(parts)
    if str(comm) != str(device):
        nodes = nodes.to(device)
    return finish(nodes, plan.n_blocks, plan.k == 0)
