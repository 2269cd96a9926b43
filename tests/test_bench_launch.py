"""bench.py --gpus N > 1 without a launcher starts its own rank processes (CPU, no GPU).

The driver launches N > 1 through `python -m torch.distributed.run`, which sets WORLD_SIZE; run
bare, `bench.py --gpus N` used to exit with "--gpus N but WORLD_SIZE=1".  Now the parent starts
the N ranks as a child `torch.distributed.run` before anything imports torch, so the parent never
initialises HIP (and never execs).  The hidden --launch-check mode makes the ranks meet over gloo
and print who they are without touching a GPU, so the whole launch runs here.
"""
import json
import os
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PARENT = textwrap.dedent("""
    import json, runpy, sys
    sys.argv = ["bench.py", "--gpus", "{n}", "--launch-check"]
    code = 0
    try:
        runpy.run_path("bench.py", run_name="__main__")
    except SystemExit as e:
        code = e.code
    print("PARENT " + json.dumps({{"torch_imported": "torch" in sys.modules, "code": code,
                                  "pid": __import__("os").getpid()}}), flush=True)
""")


def _run_parent(n):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, "-c", PARENT.format(n=n)], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=600)
    lines = r.stdout.splitlines()
    parent = json.loads(next(x for x in lines if x.startswith("PARENT "))[len("PARENT "):])
    checks = [json.loads(x) for x in lines if x.startswith("{") and "launch_check" in x]
    return r, parent, checks


def test_self_launch_parent_never_imports_torch():
    r, parent, checks = _run_parent(2)
    assert parent["code"] == 0, r.stderr[-3000:]
    assert parent["torch_imported"] is False          # no torch, so no HIP state, in the launcher
    assert len(checks) == 1, r.stdout                  # exactly one line: rank 0's
    c = checks[0]
    assert c["world_size"] == 2 and c["gpus"] == 2
    assert sorted(x["rank"] for x in c["ranks"]) == [0, 1]
    assert sorted(x["local_rank"] for x in c["ranks"]) == [0, 1]
    pids = {x["pid"] for x in c["ranks"]}
    assert len(pids) == 2 and parent["pid"] not in pids   # the ranks are child processes
    assert "self-launch" in c["launcher"]


def test_self_launch_four_ranks():
    r, parent, checks = _run_parent(4)
    assert parent["code"] == 0 and parent["torch_imported"] is False, r.stderr[-3000:]
    assert len(checks) == 1 and checks[0]["world_size"] == 4
    assert sorted(x["rank"] for x in checks[0]["ranks"]) == [0, 1, 2, 3]


def test_external_launcher_is_used_as_is():
    """WORLD_SIZE already set (the driver's torch.distributed.run): bench.py does not launch again."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--launch-check"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    c = json.loads(r.stdout.strip().splitlines()[-1])
    assert c["world_size"] == 1 and c["launcher"].startswith("external")


def _child(code):
    return [sys.executable, "-c", textwrap.dedent(code)]


def test_child_leg_result_crash_and_hang(tmp_path, monkeypatch):
    """run_child_leg (the N = 8 in-process leg's guard): a result, a crash, a crash after the
    result, no result, and a hang whose whole process group is killed."""
    import time
    sys.path.insert(0, ROOT)
    import bench
    r, hung = bench.run_child_leg(_child('print("noise"); print(\'{"in_process": {"bit_exact": true}}\')'),
                                  "in_process", 60)
    assert (r, hung) == ({"bit_exact": True}, False)
    r, hung = bench.run_child_leg(_child("import os; os.abort()"), "in_process", 60)   # SIGABRT, no line
    assert not hung and "without a result" in r["error"] and "-6" in r["error"]
    r, hung = bench.run_child_leg(_child('print(\'{"in_process": {"bit_exact": true}}\'); raise SystemExit(7)'),
                                  "in_process", 60)
    assert not hung and r["bit_exact"] is True and "status 7" in r["error"]
    # the rank environment is not handed to the leg (it would re-form the process group)
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("RANK", "0")
    r, _ = bench.run_child_leg(_child("""
        import json, os
        print(json.dumps({"in_process": {"env": [k for k in ("WORLD_SIZE", "RANK") if k in os.environ]}}))
    """), "in_process", 60)
    assert r == {"env": []}
    # a hang: the leg and a grandchild it started are killed together
    marker = tmp_path / "grandchild.pid"
    t0 = time.monotonic()
    r, hung = bench.run_child_leg(_child(f"""
        import subprocess, sys, time
        g = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(120)"])
        open({str(marker)!r}, "w").write(str(g.pid))
        time.sleep(120)
    """), "in_process", 3)
    assert hung and "watchdog" in r["error"] and time.monotonic() - t0 < 30
    gpid = int(marker.read_text())
    for _ in range(50):                      # the grandchild is gone (reaped by init) soon after the kill
        try:
            os.kill(gpid, 0)
        except ProcessLookupError:
            break
        with open(f"/proc/{gpid}/stat") as f:
            if f.read().split(") ")[1].startswith("Z"):
                break
        time.sleep(0.1)
    else:
        raise AssertionError("grandchild survived the watchdog kill")
