"""GPU tests of the host runtime (merkle_capi.hip): scratch growth near full HBM, where a call
ran, the exchange timing of sharded calls, the lane default.  Results are checked bit-exact
against the CPU oracle.  Run on the MI355X box: pytest -m gpu."""
import os

import pytest

pytestmark = pytest.mark.gpu

CHUNK = 32 << 20


def _torch():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _context(**env):
    """A context created with the given DEOSS_* environment (read at dm_create), restored after."""
    from deoss_amd import MerkleContext
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return MerkleContext()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_lane_growth_near_full_hbm_waits_for_deferred_frees(oracle_lib):
    """A lane's object buffer grows while another context's 0.5 s chain runs and the free HBM is
    below the new size: the old block sits in the reaper (its hipFree waits for that chain), so
    DevBuf::ensure sees too little free memory, drains the reaper and only then allocates, instead
    of failing with DM_ERR_NOMEM -- or, as a hipMalloc racing the pending hipFree once did inside
    the HSA runtime in the full suite, crashing."""
    import numpy as np
    torch = _torch()
    from deoss_amd import MerkleContext
    small, big = 4 << 30, 6 << 30
    host = np.empty(big, dtype=np.uint8)                 # pageable: the copy path grows d.data
    oracle_lib.fill_splitmix_ptr(host.ctypes.data, 0, big, 0xDE0554400)
    _, want_small = oracle_lib.root_buffer_ptr(host.ctypes.data, small, CHUNK, nthreads=16)
    _, want_big = oracle_lib.root_buffer_ptr(host.ctypes.data, big, CHUNK, nthreads=16)
    a = MerkleContext(lanes=1)
    b = MerkleContext(lanes=1)
    dev = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")   # b's object: 32 chains of 0.5 s
    b.fill_synthetic_async(dev.data_ptr(), 0, 1 << 30, 77, torch.cuda.current_stream().cuda_stream)
    root_b = torch.zeros(32, dtype=torch.uint8, device="cuda")
    hog = None
    try:
        assert a.root_buffer_ptr(host.ctypes.data, small, CHUNK)[1] == want_small   # a's lane holds ~4 GiB
        torch.cuda.synchronize()
        free, _ = torch.cuda.mem_get_info()
        # ~5 GiB left: below the 6 GiB growth, but with the 4 GiB old block freed there is room
        # for it plus 3 GiB for everything else the call and the HIP runtime allocate
        hog = torch.empty(free - (5 << 30), dtype=torch.uint8, device="cuda")
        free_left, _ = torch.cuda.mem_get_info()
        assert free_left < big < free_left + small
        side = torch.cuda.Stream()
        b.root_device_async(dev.data_ptr(), 1 << 30, CHUNK, root_b.data_ptr(), 0, side.cuda_stream)
        got = a.root_buffer_ptr(host.ctypes.data, big, CHUNK)[1]         # grows 4 -> 6 GiB meanwhile
        torch.cuda.synchronize()
        assert got == want_big
    finally:
        del hog
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        a.close()
        b.close()


def test_last_call_devices_and_lane_default(oracle_lib):
    """dm_last_call_devices: nothing before the first call, then the one GPU a whole call ran on;
    the lane default is sized per GPU: within half the free HBM and, together with
    every live context's claim (dm_keep_claimed), within half of the GPU's HBM."""
    from deoss_amd import MerkleContext
    from test_gpu_parity import expected_default_lanes
    if "DEOSS_LANES" in os.environ:
        pytest.skip("DEOSS_LANES set")
    torch = _torch()
    want = expected_default_lanes(torch)
    before = MerkleContext.keep_claimed(0)
    with MerkleContext() as c:
        assert c.lane_count == want
        assert MerkleContext.keep_claimed(0) == before + want * (16 << 30)
        assert c.last_call_devices() == ([], [], -1)
        data = oracle_lib.splitmix_bytes(3 << 20, 5)
        assert c.root_buffer(data, 1 << 16, want_leaves=False)[1] == oracle_lib.root_buffer(data, 1 << 16)[1]
        devs, ids, lane = c.last_call_devices()
        assert devs == [0] and ids == [0] and 0 <= lane < c.lane_count
    assert MerkleContext.keep_claimed(0) == before


def test_lane_budget_is_per_gpu():
    """default contexts share one keep budget per GPU.  Contexts opened together get
    4, 4, ... lanes until their claims reach half the GPU's HBM, then 1 each; closing one returns
    its claim."""
    from deoss_amd import MerkleContext
    from test_gpu_parity import expected_default_lanes
    if "DEOSS_LANES" in os.environ:
        pytest.skip("DEOSS_LANES set")
    torch = _torch()
    _, total = torch.cuda.mem_get_info()
    base = MerkleContext.keep_claimed(0)          # contexts the session already holds
    held = []
    try:
        for _ in range(5):
            want = expected_default_lanes(torch)
            held.append(MerkleContext())
            assert held[-1].lane_count == want
        claimed = MerkleContext.keep_claimed(0)
        assert claimed == base + sum(c.lane_count for c in held) * (16 << 30)
        assert claimed >= total // 2                         # 5 default contexts reach half of 288 GB
        assert held[-1].lane_count == 1                      # ... so the last one gets a single lane
        last = held.pop()
        last.close()
        assert MerkleContext.keep_claimed(0) == claimed - (16 << 30)
    finally:
        for c in held:
            c.close()


@pytest.mark.parametrize("G", [2, 8])
def test_sharded_call_reports_devices_and_exchange(oracle_lib, G):
    """A sharded call (virtual devices, forced): dm_last_call_devices gives devices 0 .. G-1, and
    with timing on dm_exchange_timing counts one exchange over G devices per call; off, none."""
    c = _context(DEOSS_VIRTUAL_DEVICES=G, DEOSS_FORCE_SHARDED=1)
    try:
        data = oracle_lib.splitmix_bytes(257 * 4096 + 5, 11 + G)
        leaves_w, want = oracle_lib.root_buffer(data, 4096, nthreads=8)
        assert c.root_buffer(data, 4096)[1] == want
        assert c.exchange_timing()[0] == 0          # timing off: not measured
        c.set_timing(True)
        for _ in range(2):
            leaves, root = c.root_buffer(data, 4096, want_leaves=True)
            assert root == want and leaves == leaves_w
        n, us_sum, us_max, last_g = c.exchange_timing()
        assert n == 2 and last_g == G and 0 < us_max <= us_sum
        devs, ids, lane = c.last_call_devices()
        assert devs == list(range(G)) and ids == [0] * G and lane == 0
        c.set_timing(False)
        assert c.exchange_timing() == (0, 0.0, 0.0, 0)
    finally:
        c.close()


def test_rs_create_does_not_wait_for_lane_chains(oracle_lib):
    """dm_rs_create uploads its table on a non-blocking stream: creating a coder on one context
    while another context's 0.5 s chain runs on its lane (a blocking, CU-masked stream) returns long
    before that chain ends -- hipMemcpy on the null stream would wait for it -- and the coder then
    encodes correctly."""
    import threading
    import time
    torch = _torch()
    from deoss_amd import MerkleContext
    from deoss_amd.reedsolomon import New
    with MerkleContext(lanes=1) as a, MerkleContext(lanes=1) as b:
        dev = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
        a.fill_synthetic_async(dev.data_ptr(), 0, 1 << 30, 3, 0)
        torch.cuda.synchronize()
        th = threading.Thread(target=lambda: a.root_device(dev.data_ptr(), 1 << 30, CHUNK))   # 32 chains
        th.start()
        time.sleep(0.05)
        t = time.perf_counter()
        enc = New(b, 4, 8)
        dt = time.perf_counter() - t
        th.join()
        assert dt < 0.25, dt
        shards = [oracle_lib.splitmix_bytes(4096, 40 + j) for j in range(4)]
        assert enc.Encode(shards + [bytes(4096)] * 8)[4:] == oracle_lib.rs_encode(shards, 8)
        enc.close()


def test_context_churn_returns_memory_and_claims(oracle_lib):
    """A long-lived gateway opens and closes contexts and streams: 40 rounds of create -> a
    pageable-buffer root (grows the lane's object buffer), a pinned zero-copy root, a streamed
    upload -> destroy, every result checked.  Afterwards the device's free memory is back within
    256 MiB of where it started (every hipMalloc of the library is matched by a hipFree through
    the one allocator) and the per-GPU keep claims are back to the session's."""
    import numpy as np
    torch = _torch()
    from deoss_amd import MerkleContext, PinnedBuffer
    data = oracle_lib.splitmix_bytes((48 << 20) + 123, 0xC0FFEE)
    _, want = oracle_lib.root_buffer(data, 1 << 20, nthreads=8)
    pin = PinnedBuffer(len(data))
    pin.array()[:] = np.frombuffer(data, dtype=np.uint8)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free0, _ = torch.cuda.mem_get_info()
    claim0 = MerkleContext.keep_claimed(0)
    try:
        for i in range(40):
            with MerkleContext(lanes=2) as c:
                assert c.root_buffer(data, 1 << 20, want_leaves=False)[1] == want
                assert c.root_buffer_ptr(pin.ptr, len(data), 1 << 20)[1] == want
                if i % 4 == 0:
                    s = c.open_stream(1 << 20)
                    for o in range(0, len(data), 5 << 20):
                        s.write(data[o:o + (5 << 20)])
                    assert s.close()[1] == want
        torch.cuda.synchronize()
        free1, _ = torch.cuda.mem_get_info()
        assert abs(free0 - free1) <= (256 << 20), (free0, free1)
        assert MerkleContext.keep_claimed(0) == claim0
    finally:
        pin.free()
