"""Static instruction counts of the compiled K1 loop, for the VALU roofline.

``python -m deoss_amd.isa`` recompiles merkle_capi.hip with ``-save-temps``, finds the block
loop of ``leaf_kernel<false,true>`` (uniform chunks, 16-B aligned: the bench path) and counts its
VALU instructions per 64-byte block; the result is written to ``isa_counts.json`` next to this
file (it travels with the built library).
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
# Issue slots per wave64 instruction relative to v_add_u32, measured on MI355X by
# tools/valu_peak.hip (profiles/r01_valu_peak.json): v_alignbit_b32 and v_add3_u32 run at half
# the v_add_u32 / v_bitop3_b32 rate.
SLOT_WEIGHTS = {"v_alignbit_b32": 2.0, "v_add3_u32": 2.0}
COUNTS = os.path.join(HERE, "isa_counts.json")
K1_SYMBOL = "_ZN2dm11leaf_kernelILb0ELb1EEEvNS_8LeafArgsE"


def _function_body(asm: str, sym: str) -> list:
    lines = asm.splitlines()
    start = None
    for i, ln in enumerate(lines):
        if ln.startswith(sym + ":"):
            start = i
            break
    if start is None:
        raise ValueError(f"{sym} not found in assembly")
    body = []
    for ln in lines[start + 1:]:
        if ln.startswith(".Lfunc_end") or re.match(r"^\s*\.size\s+" + re.escape(sym), ln):
            break
        body.append(ln)
    return body


def analyse(asm: str, sym: str = K1_SYMBOL) -> dict:
    """Find the hottest loop (largest basic-block chain ending in a backward branch)."""
    body = _function_body(asm, sym)
    labels = {}
    insts = []   # (index, text)
    for ln in body:
        s = ln.strip()
        if not s or s.startswith(";") or s.startswith("."):
            m = re.match(r"^(\.LBB[0-9_]+):", s)
            if m:
                labels[m.group(1)] = len(insts)
            continue
        m = re.match(r"^(\.LBB[0-9_]+):", s)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        insts.append(s.split(";")[0].strip())
    best = None
    for i, ins in enumerate(insts):
        m = re.match(r"^s_cbranch_\w+\s+(\.LBB[0-9_]+)", ins) or re.match(r"^s_branch\s+(\.LBB[0-9_]+)", ins)
        if not m or m.group(1) not in labels:
            continue
        tgt = labels[m.group(1)]
        if tgt > i:
            continue
        loop = insts[tgt:i + 1]
        loads = sum(1 for x in loop if x.startswith("global_load_dwordx4"))
        if loads < 4:      # the block loop streams 64 B per iteration (4 x dwordx4)
            continue
        if best is not None and len(loop) >= best["total"]:
            continue
        valu = [x for x in loop if x.startswith("v_")]
        hist = {}
        for x in valu:
            op = x.split()[0]
            hist[op] = hist.get(op, 0) + 1
        per = max(1, loads // 4)   # 64-byte blocks per loop iteration
        slots = sum(SLOT_WEIGHTS.get(x.split()[0], 1.0) for x in valu)
        best = {"valu": round(len(valu) / per, 1), "valu_slots": round(slots / per, 1), "blocks_per_iteration": per,
                "valu_per_iteration": len(valu), "salu": sum(1 for x in loop if x.startswith("s_")),
                "vmem": sum(1 for x in loop if x.startswith(("global_", "buffer_", "flat_"))),
                "total": len(loop), "valu_histogram": dict(sorted(hist.items(), key=lambda kv: -kv[1]))}
    if best is None:
        raise ValueError("no loop found")
    return best


def generate() -> dict:
    from . import build as b
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "lib.so")
        cmd = b.hipcc_cmd(out, extra=("-save-temps",))
        subprocess.run(cmd, check=True, cwd=td, capture_output=True)
        asm_files = [f for f in os.listdir(td) if f.endswith(".s") and "gfx950" in f]
        asm = open(os.path.join(td, asm_files[0])).read()
    res = analyse(asm)
    res["kernel"] = K1_SYMBOL
    res["per"] = "one 64-byte block (loop iteration of absorb_blocks)"
    with open(COUNTS, "w") as f:
        json.dump(res, f, indent=1)
    return res


def valu_per_block():
    """(VALU instructions, full-rate issue slots) per 64-byte block of the K1 loop."""
    try:
        with open(COUNTS) as f:
            d = json.load(f)
            return d["valu"], d["valu_slots"]
    except (OSError, KeyError, ValueError):
        return None, None


if __name__ == "__main__":
    print(json.dumps(generate(), indent=1))
