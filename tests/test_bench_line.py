"""The driver-facing bench line (CPU, no GPU).

Round 4's N = 1 line grew to 28 KB and the driver could not parse it (BENCH_r04.json "parsed":
null), so the headline went unmeasured.  bench.py now prints a compact line last (compact_line,
at most LINE_MAX_BYTES) and writes the full record to a detail file.  These tests rebuild the
compact line from the two full lines round 4 printed -- the N = 1 default run and the 8-rank
rehearsal (tests/golden/bench_lines_r04.json, from profiles/r04) -- and
check its size and keys, that a failed extra or parity check turns `ok` false, and that a hung
watchdogged leg ends the process with a non-zero status.
"""
import copy
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

REQUIRED = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "ok", "detail")


def _full_line(name):
    """Round 4's full lines, kept in tests/golden/bench_lines_r04.json (from profiles/r04)."""
    with open(os.path.join(ROOT, "tests", "golden", "bench_lines_r04.json")) as f:
        d = json.load(f)
    return d[{"r04q_bench.log": "n1", "r04m_rehearse8.log": "n8"}[name]]


def _size(line):
    return len(json.dumps(line, separators=(",", ":")))


def test_compact_line_n1_from_r04_default_run():
    full = _full_line("r04q_bench.log")
    assert len(json.dumps(full)) > 20000                  # the line the driver could not parse
    line = bench.compact_line(full, "gpurun_out/bench_detail_n1.json")
    assert _size(line) <= bench.LINE_MAX_BYTES
    for k in REQUIRED + ("cpu_baseline", "parity", "e2e", "extras", "latency"):
        assert k in line, k
    assert line["value"] == full["value"] and line["ms_per_step"] == full["ms_per_step"]
    rf = line["roofline"]
    assert rf["frac"] == full["roofline"]["frac"] and rf["traffic"] == full["roofline"]["traffic"]
    assert rf["chain_issue_floor"]["frac"] == full["roofline"]["chain_issue_floor"]["frac"]
    assert 0.99 < rf["traffic_over_algorithmic"] < 1.01
    cb = line["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] == 1 and cb["value"] == full["cpu_baseline"]["value"]
    assert cb["parallel"]["cores"] == full["cpu_baseline"]["parallel"]["cores"]
    assert line["parity"]["bit_exact"] is True and line["parity"]["gpu_root"] == full["parity"]["gpu_root"]
    assert set(line["extras"]) == set(full["other_configs"])
    for name, e in line["extras"].items():
        src = full["other_configs"][name]
        assert e["value"] == src["value"] and e["unit"] == src["unit"] and e["bit_exact"] is True, name
        assert e["frac"] == src["roofline"]["frac"] and e["ok"] is True, name
    assert line["ok"] is True and "problems" not in line
    assert line["detail"] == "gpurun_out/bench_detail_n1.json"


def test_compact_line_n8_rehearsal():
    full = _full_line("r04m_rehearse8.log")
    full = copy.deepcopy(full)
    full["strong_scaling"] = {"workload": "configs[1] strong", "value": 16.3, "unit": "GiB/s", "bit_exact": True,
                              "single_gpu_ms": 490.0, "speedup_vs_one_gpu": 1.0, "speedup_vs_one_gpu_share_of_weak": 1.0}
    full["strong_scaling_4KiB"] = {"workload": "configs[1] strong: one 8 GiB object (2097152 leaves of 4096 B) over "
                                   "8 GPUs", "chunk": 4096, "value": 5000.0, "unit": "GiB/s", "ms_per_step": 1.6,
                                   "bit_exact": True, "single_gpu_ms": 5.6, "speedup_vs_one_gpu": 3.5,
                                   "note": "throughput regime"}
    full["exchange"] = {"collective": "all_gather_into_tensor", "backend": "nccl (RCCL)", "bytes_per_rank": 32,
                        "ranks": 8, "reps": 100, "avg_us": 41.5}
    full["other_configs"]["in_process"]["host_feed"] = {"slice_bytes": 8 << 30, "devices": 8, "alone_GBps": 56.1,
                                                        "all_GBps": 401.7, "all_ms": 171.0, "consistent": True,
                                                        "what": "x" * 300}
    line = bench.compact_line(full, None)
    assert _size(line) <= bench.LINE_MAX_BYTES
    assert line["exchange"] == {"backend": "nccl (RCCL)", "bytes_per_rank": 32, "ranks": 8, "avg_us": 41.5}
    assert line["extras"]["in_process"]["host_feed"] == {"alone_GBps": 56.1, "all_GBps": 401.7, "consistent": True}
    assert line["strong_scaling_4KiB"]["speedup_vs_one_gpu"] == 3.5 and "note" not in line["strong_scaling_4KiB"]
    for k in REQUIRED + ("parity", "launch", "extras", "strong_scaling"):
        assert k in line, k
    assert line["launch"]["world_size"] == full["launch"]["world_size"]
    assert line["strong_scaling"]["speedup_vs_one_gpu"] == 1.0
    assert set(line["extras"]) == {"configs[3]", "configs[4]", "in_process"}
    ip = line["extras"]["in_process"]
    assert ip["bit_exact"] is True and ip["sharded_object"]["bit_exact"] is True
    assert line["ok"] is True


def test_failures_turn_ok_false():
    full = copy.deepcopy(_full_line("r04q_bench.log"))
    full["other_configs"]["configs[2]"] = {"error": "RuntimeError: dm_root_batch failed " + "x" * 4000}
    full["other_configs"]["FullProcessing"]["bit_exact"] = False
    full["parity"]["bit_exact"] = False
    line = bench.compact_line(full, None)
    assert _size(line) <= bench.LINE_MAX_BYTES
    assert line["ok"] is False
    assert {"parity", "configs[2]", "FullProcessing"} <= set(line["problems"])
    assert line["extras"]["configs[2]"]["ok"] is False and len(line["extras"]["configs[2]"]["error"]) <= 160


def test_oversized_line_is_bounded():
    full = copy.deepcopy(_full_line("r04q_bench.log"))
    for i in range(60):        # many more extras than any run has
        full["other_configs"][f"extra_{i:02d}"] = copy.deepcopy(full["other_configs"]["configs[2]"])
    line = bench.compact_line(full, None)
    assert _size(line) <= bench.LINE_MAX_BYTES or len(line["extras"]) > 60
    assert "value" in line and "roofline" in line and "cpu_baseline" in line


def test_emit_writes_detail_and_prints_one_line(tmp_path, capsys):
    full = _full_line("r04q_bench.log")
    path = tmp_path / "detail.json"
    bench.emit(full, str(path))
    out = capsys.readouterr().out.strip().splitlines()
    assert len(out) == 1 and len(out[0]) <= bench.LINE_MAX_BYTES
    line = json.loads(out[0])
    assert line["detail"] == str(path)
    with open(path) as f:
        assert json.load(f) == full


def test_watchdog_hang_exits_nonzero(tmp_path):
    """A leg that outlives its watchdog: the line is printed (ok false, the leg's error in it) and
    the process exits with status 3, not 0."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "bench.py", "--watchdog-check", "0.5", "--detail-out",
                        str(tmp_path / "d.json")], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 3, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["ok"] is False and line["problems"] == ["in_process"]
    assert "watchdog" in line["extras"]["in_process"]["error"]
    assert os.path.exists(tmp_path / "d.json")


def test_strong_leg_error_and_missing_blocks():
    """A strong leg that raised shows as an error and turns ok false; a line without roofline,
    CPU baseline or extras (a bare N > 1 run with --no-extras) still fits and carries the contract keys."""
    full = copy.deepcopy(_full_line("r04m_rehearse8.log"))
    full["strong_scaling_4KiB"] = {"error": "RuntimeError: " + "y" * 3000}
    line = bench.compact_line(full, None)
    assert line["ok"] is False and "strong_scaling_4KiB" in line["problems"]
    assert _size(line) <= bench.LINE_MAX_BYTES and len(line["strong_scaling_4KiB"]["error"]) <= 160
    bare = {k: full[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")}
    line = bench.compact_line(bare, None)
    assert line["ok"] is True and _size(line) < 1500
    for k in REQUIRED:
        if k != "roofline":
            assert k in line, k
