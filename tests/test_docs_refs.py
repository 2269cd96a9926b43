"""CPU guards on the evidence the docs cite: every `profiles/...` path named in DESIGN.md,
INTEGRATION.md and README.md exists, every `profiles/rNN/LOGS.md#name` anchor is a section of that
file, every bare `r04x_*.log` DESIGN.md names is in profiles/r04/, and profiles/extras_traffic.json
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


def test_round4_logs_named_in_design_exist():
    names = set(re.findall(r"`(r04[a-z]+_[A-Za-z0-9_\-]+\.log)`", _read("DESIGN.md")))
    assert names
    missing = [n for n in names if not os.path.exists(os.path.join(ROOT, "profiles", "r04", n))]
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
