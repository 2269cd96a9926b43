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


def _n8_with_cpu_baseline(tmp_path):
    """Round 4's N = 8 rehearsal line plus the cpu_baseline block an N > 1 run now carries (over
    rank 0's shard: here the N = 1 line's block, the same 8 GiB object), written to a file."""
    full = copy.deepcopy(_full_line("r04m_rehearse8.log"))
    full["cpu_baseline"] = copy.deepcopy(_full_line("r04q_bench.log")["cpu_baseline"])
    full["cpu_baseline"]["shard_root_bit_exact"] = True
    path = tmp_path / "n8.json"
    path.write_text(json.dumps(full))
    return path


def _fake(tmp_path, *extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "DEOSS_BENCH_T0")}
    return [sys.executable, "bench.py", "--fake-legs", *extra, "--fake-line", str(_n8_with_cpu_baseline(tmp_path)),
            "--detail-out", str(tmp_path / "d.json")], env


def test_killed_mid_leg_leaves_a_parseable_line(tmp_path):
    """the line is printed after the headline and after every leg, so a run the
    driver kills in the middle of a leg (SIGKILL: no handler runs) still ends stdout with a whole
    line that carries the headline, its roofline and its CPU baseline, and names the legs it did
    not finish."""
    import signal
    import time
    cmd, env = _fake(tmp_path, "3")
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True,
                         start_new_session=True)
    lines = []
    try:
        t0 = time.time()
        while len(lines) < 2 and time.time() - t0 < 60:     # the headline, then the line after leg 1
            ln = p.stdout.readline()
            if not ln:
                break
            lines.append(ln)
        assert len(lines) == 2, lines
        time.sleep(0.5)                                     # now inside leg 2 (3 s)
    finally:
        os.killpg(p.pid, signal.SIGKILL)
        rest = p.stdout.read()
        p.wait(timeout=30)
    assert p.returncode == -signal.SIGKILL
    lines += [x for x in rest.splitlines(keepends=True) if x.strip()]
    assert len(lines) == 2                                  # nothing was printed after the kill
    for ln in lines:
        assert len(ln.strip()) <= bench.LINE_MAX_BYTES
    last = json.loads(lines[-1])
    for k in REQUIRED + ("cpu_baseline", "legs", "complete"):
        assert k in last, k
    assert last["value"] > 0 and last["roofline"]["frac"] > 0 and last["cpu_baseline"]["cores"] == 1
    assert last["cpu_baseline"]["shard_root_bit_exact"] is True
    assert last["complete"] is False and last["legs"]["done"] == {"strong_scaling": last["legs"]["done"]["strong_scaling"]}
    assert last["legs"]["pending"] == ["strong_scaling_4KiB", "configs[3]", "configs[4]", "in_process"]
    assert last["strong_scaling"]["bit_exact"] is True
    first = json.loads(lines[0])
    assert first["value"] == last["value"] and len(first["legs"]["pending"]) == 5


def test_deadline_skips_legs_that_do_not_fit(tmp_path):
    """--deadline-s: a leg starts only if its estimate fits in what is left; the skipped ones are
    named in `problems` and `legs.skipped`, the run still ends with a complete line and status 0."""
    cmd, env = _fake(tmp_path, "0.6")
    r = subprocess.run(cmd + ["--deadline-s", "2.0"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    out = [json.loads(x) for x in r.stdout.splitlines() if x.strip()]
    assert len(out) == 6                                     # the headline + one line per leg, run or skipped
    last = out[-1]
    assert last["complete"] is True and last["legs"]["pending"] == []
    assert "strong_scaling" in last["legs"]["done"] and "in_process" in last["legs"]["skipped"]
    assert set(last["legs"]["done"]) | set(last["legs"]["skipped"]) == {
        "strong_scaling", "strong_scaling_4KiB", "configs[3]", "configs[4]", "in_process"}
    assert last["ok"] is False and "skipped:in_process" in last["problems"]
    assert "deadline" in last["legs"]["skipped"]["in_process"]
    with open(tmp_path / "d.json") as f:                   # the detail file is rewritten with every line
        assert json.load(f)["legs"]["skipped"].keys() == last["legs"]["skipped"].keys()


def test_leg_estimates_fit_the_default_deadline():
    """The N = 8 legs' estimates plus the headline fit the default deadline, which leaves the
    driver's 600 s a margin; each estimate covers at least 3x the leg's per-rank work measured at
    full size on one MI355X (profiles/r06/n8_legs/times.jsonl, tools/n8_leg_times.sh); the
    in-process watchdog ends before the deadline."""
    n8 = ("strong_scaling", "strong_scaling_4KiB", "configs[3]", "configs[4]", "in_process")
    headline_s = 120.0    # a fresh node's torch import + process group + 25 steps of 0.49 s + parity legs
    assert headline_s + sum(bench.LEG_ESTIMATE_S[k] for k in n8) < bench.DEADLINE_DEFAULT_S < 600
    with open(os.path.join(ROOT, "profiles", "r06", "n8_legs", "times.jsonl")) as f:
        measured = {d["leg"]: d["wall_s"] for d in map(json.loads, f) if d["rc"] == 0}
    covers = {"strong_scaling_4KiB": "strong_4k_8g", "configs[3]": "cfg3_share_128g", "configs[4]": "cfg4_share_12500",
              "in_process": "inprocess_8virt_64g"}
    for leg, m in covers.items():
        assert bench.LEG_ESTIMATE_S[leg] >= 3 * measured[m], (leg, measured[m])
    assert 0 < bench.WATCHDOG_MARGIN_S < bench.LEG_ESTIMATE_S["in_process"]


def test_ranks_follow_rank0_leg_decisions_gloo(tmp_path):
    """N > 1 (2 gloo ranks, no GPU, started by bench.py's own self-launch): rank 0 decides whether
    each leg fits and every rank follows -- here rank 1's own clock says no time is left, yet it
    runs exactly the legs rank 0 runs, so the collectives inside a leg stay matched."""
    cmd, env = _fake(tmp_path, "0.2")
    env["MASTER_ADDR"] = "127.0.0.1"
    r = subprocess.run(cmd[:2] + ["--gpus", "2"] + cmd[2:] + ["--deadline-s", "300"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    last = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert set(last["legs"]["done"]) == {"strong_scaling", "strong_scaling_4KiB", "configs[3]", "configs[4]",
                                         "in_process"} and last["complete"] is True
    with open(tmp_path / "d.json.rank1.json") as f:
        r1 = json.load(f)
    assert set(r1["done"]) == set(last["legs"]["done"]) and not r1["skipped"] and r1["deadline_s"] == 0.0


def _r06(name):
    with open(os.path.join(ROOT, "tests", "golden", "bench_lines_r06.json")) as f:
        return json.load(f)[name]


def test_n_gt_1_line_carries_cpu_baseline_and_traffic():
    """VERDICT r5 item 2, on round 6's real N > 1 records (tests/golden/bench_lines_r06.json): the
    rebuilt line of the 8-rank rehearsal and of the 2-rank full-size run carry `cpu_baseline` (the
    1-thread restatement over rank 0's shard, the job-share rate, the host) and `roofline.traffic`
    (PMC bytes of the same kernel and per-rank launch shape), within 6 KB."""
    for name in ("n8", "n2"):
        full = _r06(name)
        line = bench.compact_line(full, f"gpurun_out/bench_detail_{name}.json")
        assert _size(line) <= bench.LINE_MAX_BYTES, name
        cb = line["cpu_baseline"]
        assert cb["kind"] == "port" and cb["cores"] == 1 and cb["value"] > 1.0, name
        assert cb["parallel"]["cores"] >= 1 and cb["host"] and cb["shard_root_bit_exact"] is True, name
        assert "rank 0's shard" in cb["sample"], name
        rf = line["roofline"]
        assert rf["traffic"] and 0.99 < rf["traffic_over_algorithmic"] < 1.01, name
        assert line["legs"]["pending"] == [] and line["complete"] is True and line["ok"] is True, name
        for k in REQUIRED + ("parity", "launch", "exchange", "strong_scaling", "strong_scaling_4KiB", "vs_cpu_share"):
            assert k in line, (name, k)
    n8 = bench.compact_line(_r06("n8"), None)
    assert set(n8["extras"]) == {"configs[3]", "configs[4]", "in_process"}
    assert n8["extras"]["configs[3]"]["fixture_bit_exact"] is True
    n2 = bench.compact_line(_r06("n2"), None)
    assert n2["parity"]["cpu_root"] == n2["parity"]["sharded_root"] and "weak_n2" in n2["parity"]["cpu_root_source"]
    assert "route_constants" not in n2          # a one-GPU rehearsal's numbers are not a node's


def test_route_constants_from_a_real_line():
    """An N > 1 line over RCCL prints the two measured routing terms as the environment values
    dm_create reads."""
    full = copy.deepcopy(_r06("n8"))
    full.pop("same_device", None)
    full["exchange"]["backend"] = "nccl (RCCL)"
    full["exchange"]["avg_us"] = 41.53
    full["other_configs"]["in_process"]["host_feed"].update(all_GBps=401.7, consistent=True)
    line = bench.compact_line(full, None)
    assert line["route_constants"] == {"DEOSS_ALLGATHER_US": 41.5, "DEOSS_HOST_BYTES_PER_S": 401700000000}
    full["other_configs"]["in_process"]["host_feed"]["consistent"] = False
    assert bench.compact_line(full, None)["route_constants"] == {"DEOSS_ALLGATHER_US": 41.5}
