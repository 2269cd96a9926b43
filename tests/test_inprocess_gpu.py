"""The N = 8 bench line's in-process leg (bench.in_process_configs), rehearsed small on one GPU.

At N = 8 rank 0 opens one dm_ctx over every GPU -- what go/hashtree gets -- and runs a forced-
sharded pinned object (multi_root + the all-gather), a host batch split by objects, and 8
concurrent NewHashTree-shaped calls, each against the CPU oracle.  Here the GPUs are 4
DEOSS_VIRTUAL_DEVICES on cuda:0 (the gather becomes D2D copies), so the leg's own code runs on
every GPU round, not only on the driver's 8-GPU node."""
import os
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.gpu
def test_in_process_leg_virtual_devices():
    import torch
    import bench
    args = types.SimpleNamespace(inproc_gib=0.5, same_device=True)
    res = bench.in_process_configs(args, torch, 4)
    assert res["virtual_devices"] and res["devices"] == 4, res
    assert res["bit_exact"], res
    sh = res["sharded_object"]
    assert sh["context_devices"] == 4 and sh["parity"]["leaves"] == res["object_bytes"] // res["chunk"]
    assert sh["exchange"]["calls"] == 3 and sh["exchange"]["devices"] == 4 and sh["exchange"]["avg_us"] > 0
    assert sorted(sh["ran_on"]["context_devices"]) == [0, 1, 2, 3]      # the call spanned every device
    b = res["batch_by_objects"]
    assert b["parity"]["checked_objects"] == b["objects"] > 0 and b["parity"]["mismatches"] == 0
    c = res["concurrent_calls"]
    assert c["parity"]["checked_calls"] == 8 and len(c["gpus_used"]) >= 2   # routed over the devices
    h = res["host_feed"]
    assert "error" not in h, h
    assert h["devices"] == 4 and h["consistent"] and h["alone_GBps"] > 1 and h["all_GBps"] > 1
