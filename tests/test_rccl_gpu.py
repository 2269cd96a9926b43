"""The N > 1 bench path's RCCL calls, executed on this box's one GPU.

The 8-GPU node is the driver's, never ours, and RCCL refuses two ranks on one GPU, so the
multi-rank exchange itself only runs there.  What one GPU can run is the same code over a real
RCCL communicator of world size 1: bench.py's `nccl` process group (init with device_id, the
all_gather_into_tensor of sharded_root, the barrier with device_ids, all_gather_object of the
launch record, the exchange timing), so the first 8-GPU line does not also carry the first
execution of that code.  (The library's own ncclCommInitAll / ncclAllGather run on one GPU in
tests/test_gpu_parity.py::test_single_process_sharded_path through DEOSS_FORCE_SHARDED.)
Contract anchor: /root/reference/common/hashtree/types.go:38 (the root this exchange finishes).
"""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_nccl_process_group_world1_bench_exchange(oracle_lib):
    import torch
    import torch.distributed as dist
    import bench
    from deoss_amd import MerkleContext, plan_shards
    from deoss_amd.sharding import sharded_root
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=device)
    try:
        assert "nccl" in str(dist.get_backend())
        length, chunk, seed = (96 << 20) + 12345, 1 << 20, 0xDE0550003
        want = oracle_lib.root_buffer(oracle_lib.splitmix_bytes(length, seed), chunk, nthreads=8)[1]
        plan = plan_shards(length, chunk, 1)
        buf = torch.empty(length + 64, dtype=torch.uint8, device=device)
        nodes = torch.zeros(max(plan.node_count(0), 1) * 32, dtype=torch.uint8, device=device)
        root = torch.zeros(32, dtype=torch.uint8, device=device)
        with MerkleContext(devices=[0]) as ctx:
            s = torch.cuda.current_stream().cuda_stream
            ctx.fill_synthetic_async(buf.data_ptr(), 0, (length + 7) // 8 * 8, seed, s)

            def subtree(k):
                ctx.subtree_device_async(buf.data_ptr(), length, chunk, k, nodes.data_ptr(), s)
                return nodes

            def finish(n_, n, min_one):
                ctx.finish_device_async(n_.data_ptr(), n, min_one, root.data_ptr(), s)
                return root

            for _ in range(3):         # the bench's step, over RCCL (device buffers, the default comm)
                got = sharded_root(plan, 0, subtree, finish, torch, dist, device)
                torch.cuda.synchronize()
                assert bytes(got.cpu().numpy()) == want

        def barrier():
            dist.barrier(device_ids=[0])
            torch.cuda.synchronize()
        ex = bench.measure_exchange(plan, torch, dist, device, False, barrier, reps=20)
        assert ex["backend"] == "nccl (RCCL)" and ex["ranks"] == 1 and ex["avg_us"] > 0
        rc = bench.route_constants({"exchange": ex})
        assert rc == {"DEOSS_ALLGATHER_US": round(float(ex["avg_us"]), 1)}

        class A:
            same_device = False
        info = bench.launch_info(torch, dist, 1, 0, 0, 0, A())
        assert info["world_size"] == 1 and info["rank_devices"][0]["device"] == 0 and info["distinct_gpus"] == 1
        assert info["rccl_version"] and "unavailable" not in info["rccl_version"]
    finally:
        dist.destroy_process_group()
