"""CPU guards on the evidence the docs cite: every `profiles/...` path named in DESIGN.md,
INTEGRATION.md and README.md exists, every `profiles/rNN/LOGS.md#name` anchor is a section of that
file, every bare `rNNx_*.log` the docs name is in profiles/rNN/ (or its LOGS.md), and profiles/extras_traffic.json
(read by bench.py for the extras' roofline traffic) covers every extra bench.py reports."""
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ("DESIGN.md", "INTEGRATION.md", "README.md")


def _read(p):
    with open(os.path.join(ROOT, p)) as f:
        return f.read()


def test_profile_paths_exist():
    missing = []
    for doc in DOCS:
        for m in re.finditer(r"`(profiles/[^`\s#()]+)", _read(doc)):
            p = m.group(1).rstrip(".,;:")
            if any(c in p for c in "{*<…"):
                continue
            if not os.path.exists(os.path.join(ROOT, p)):
                missing.append((doc, p))
    assert not missing, missing


def test_logs_anchors_exist():
    bad = []
    for doc in DOCS:
        for m in re.finditer(r"(profiles/r0\d/LOGS\.md)#([A-Za-z0-9_.\-]+)", _read(doc)):
            p, a = m.group(1), m.group(2).rstrip(".,;:")
            if f"## {a}" not in _read(p):
                bad.append((doc, p, a))
    assert not bad, bad


def test_round_logs_named_in_docs_exist():
    """A bare `rNNx_name.log` in the docs is a file of profiles/rNN/ or a section of its LOGS.md."""
    missing = []
    for doc in DOCS:
        for name, rnd in set(re.findall(r"`((r0\d)[a-z]*_[A-Za-z0-9_\-]+\.log)`", _read(doc))):
            d = os.path.join(ROOT, "profiles", rnd)
            logs = os.path.join(d, "LOGS.md")
            if os.path.exists(os.path.join(d, name)):
                continue
            if os.path.exists(logs) and f"## {name}" in _read(os.path.relpath(logs, ROOT)):
                continue
            missing.append((doc, name))
    assert not missing, missing


def test_extras_traffic_covers_every_extra():
    sys.path.insert(0, ROOT)
    import bench
    traffic, src = bench.extras_traffic()
    assert src == "profiles/extras_traffic.json"
    keys = {v[0] for v in bench.EXTRA_ROOF.values()}
    assert keys <= set(traffic), keys - set(traffic)
    for k in keys:
        w = traffic[k]
        assert w["traffic_bytes_per_step"] > 0 and w["kernels"], k
        assert w.get("method", "").startswith("marginal"), (k, w.get("method"))
    raw = json.loads(_read("profiles/extras_traffic.json"))
    assert "FETCH_SIZE" in raw["correction"] and raw["workloads"]
