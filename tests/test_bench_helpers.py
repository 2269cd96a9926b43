"""CPU tests of bench.py's host-side helpers (no GPU): percentiles, the step-level roofline the
N = 1 extras carry, and the CPU-baseline legs (the oracle, timed on small inputs)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_percentiles_nearest_rank():
    xs = [i / 1000 for i in range(1, 101)]          # 1 .. 100 ms
    p = bench._pcts(xs)
    assert p["p50_ms"] == 50.0 and p["p99_ms"] == 99.0 and p["min_ms"] == 1.0 and p["max_ms"] == 100.0
    assert p["samples"] == 100
    p = bench._pcts([0.003, 0.001, 0.002])          # below 100 samples p99 is the maximum
    assert p["p50_ms"] == 2.0 and p["p99_ms"] == 3.0


def test_extra_roofline_step_level_and_kernel_level():
    traffic = {"process": {"traffic_bytes_per_step": 52e9, "kernels": {
        "rs_code_kernel": {"launches": 1, "read_bytes": 8.6e9, "write_bytes": 17.2e9},
        "leaf_kernel_quad": {"launches": 1, "read_bytes": 25.9e9, "write_bytes": 1e5},
        "__amd_rocclr_copyBuffer": {"launches": 2, "read_bytes": 0.1e9, "write_bytes": 0.2e9}}}}
    r = {"ms_per_step": 600.0, "roofline": {"bound": "hbm", "achieved": 52.0, "frac": 0.0065, "traffic": None}}
    bench.extra_roofline("FullProcessing", r, traffic, "profiles/extras_traffic.json")
    rf = r["roofline"]
    alg = (8 << 30) * 7
    assert rf["bound"] == "hbm" and rf["algorithmic_bytes_per_step"] == alg
    assert abs(rf["achieved"] - alg / 0.6 / 1e9) < 1e-3 and rf["frac"] == round(rf["achieved"] / 8000.0, 6)
    assert rf["traffic"] == 52e9 and abs(rf["traffic_over_algorithmic"] - 52e9 / alg) < 1e-4
    kern = 8.6e9 + 17.2e9 + 25.9e9 + 1e5           # the product's kernels; the blit copies apart
    assert rf["kernel_traffic"] == round(kern) and rf["copy_traffic"] == round(52e9 - kern)
    assert rf["kernel_traffic_over_design"] == round(kern / rf["design_kernel_bytes_per_step"], 4)
    kl = rf["kernel_level"]             # the workload's own kernel-level line, traffic filled in
    assert kl["traffic"] == 25.9e9 + 1e5 and "leaf_kernel_quad" in kl["traffic_source"]
    # host-memory extras are bound by the PCIe link; an unprofiled extra says so
    r = {"ms_per_step": 200.0}
    bench.extra_roofline("configs[4]_per_gpu_share", r, {}, None)
    assert r["roofline"]["bound"] == "pcie" and r["roofline"]["peak"] == bench.PCIE_PEAK_GBS
    assert r["roofline"]["traffic"] is None and r["roofline"]["traffic_scope"] == "not profiled"
    r = {"error": "x"}
    bench.extra_roofline("FullProcessing", r, traffic, "x")     # no step time: untouched
    assert "roofline" not in r


def test_cpu_baseline_legs_small():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import Oracle
    orc = Oracle()
    a = np.empty(3 << 20, dtype=np.uint8)
    orc.fill_splitmix_ptr(a.ctypes.data, 0, a.size, 5)
    c = bench.cpu_root_baseline(orc, a.ctypes.data, a.size, 1 << 20, "a test buffer", 2 << 20)
    assert c["cores"] == 1 and c["kind"] == "port" and c["value"] > 0
    assert c["parallel"]["cores"] == bench.cpu_share() and c["parallel"]["value"] > 0
    f = bench.cpu_fp_baseline(orc, a.ctypes.data, a.size, 1 << 20, "a test buffer", serial_segs=1, par_segs=3)
    assert f["cores"] == 1 and f["value"] > 0 and "1 segment(s)" in f["sample"]
    assert f["parallel"]["value"] > 0 and "3 segments" in f["parallel"]["sample"]
