"""Static instruction counts of the compiled leaf-kernel loops, for the VALU roofline.

``python -m deoss_amd.isa`` recompiles merkle_capi.hip with ``-save-temps`` and, for each
leaf kernel (16-B aligned variants: the bench path), finds its per-block loop in the gfx950
assembly and counts the instructions of one 64-byte block:

* ``wide`` (K1, one lane per leaf): the loop streaming 8 x global_load_dwordx4 per two blocks;
* ``latency`` (K1L) and ``pair`` (K1P): the consumer loop (16 ds_read_b128 of K+W per block)
  and the producer loop (16 ds_write_b128 per block);
* ``quad`` (K1Q): the consumer's whole-stage loop (8 blocks from registers, 32 ds_read_b128:
  each block's words spread over a quad's lanes) and the producer loop.

``lanes`` converts wave-instruction counts into lane-slots per leaf-block: K1 runs one lane per
leaf; per leaf-block K1L spends one consumer + one producer lane, K1P two + two, K1Q eight
consumer lanes + one producer lane (each producer lane schedules its own block).  Results go to
``isa_counts.json`` next to this file (it travels with the built library).
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
COUNTS = os.path.join(HERE, "isa_counts.json")
# Issue slots per wave64 instruction relative to v_add_u32, measured on MI355X by
# tools/valu_peak.hip (profiles/r01/r01_valu_peak.json): v_alignbit_b32 and v_add3_u32 run at half
# the v_add_u32 / v_bitop3_b32 rate.
SLOT_WEIGHTS = {"v_alignbit_b32": 2.0, "v_add3_u32": 2.0, "v_xad_u32": 2.0}
# name: (symbol, (consumer lanes, producer lanes) per leaf-block)
KERNELS = {
    "wide": ("_ZN2dm11leaf_kernelILb0ELb1EEEvNS_8LeafArgsE", (1, 0)),
    "latency": ("_ZN2dm15leaf_kernel_latILb0ELb1EEEvNS_8LeafArgsE", (1, 1)),
    "pair": ("_ZN2dm16leaf_kernel_pairILb0ELb1EEEvNS_8LeafArgsE", (2, 2)),
    "quad": ("_ZN2dm16leaf_kernel_quadILb0ELb1ELb0EEEvNS_8LeafArgsE", (8, 1)),   # wide ring (the headline)
}
K1_SYMBOL = KERNELS["wide"][0]


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


def _loops(body: list):
    """Yield the instruction list of every backward-branch loop."""
    labels, insts = {}, []
    skip = []   # .if <literal> ... .endif from inline asm (DM_QS_ALIGN_MIS): count taken arms only
    for ln in body:
        s = ln.strip()
        m = re.match(r"^\.if\s+(\S+)", s)
        if m:
            skip.append(m.group(1) == "0")
            continue
        if s.startswith(".endif"):
            if skip:
                skip.pop()
            continue
        if any(skip):
            continue
        m = re.match(r"^(\.LBB[0-9_]+):", s)
        if m:
            labels[m.group(1)] = len(insts)
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        insts.append(s.split(";")[0].strip())
    for i, ins in enumerate(insts):
        m = re.match(r"^s_c?branch\w*\s+(\.LBB[0-9_]+)", ins)
        if m and m.group(1) in labels and labels[m.group(1)] <= i:
            yield insts[labels[m.group(1)]:i + 1]


def _summary(loop: list, per: int) -> dict:
    valu = [x for x in loop if x.startswith("v_")]
    hist = {}
    for x in valu:
        op = x.split()[0]
        hist[op] = hist.get(op, 0) + 1
    slots = sum(SLOT_WEIGHTS.get(x.split()[0], 1.0) for x in valu)
    return {"valu": round(len(valu) / per, 1), "valu_slots": round(slots / per, 1),
            "blocks_per_iteration": per, "salu": sum(1 for x in loop if x.startswith("s_")),
            "lds": sum(1 for x in loop if x.startswith("ds_")),
            "vmem": sum(1 for x in loop if x.startswith(("global_", "buffer_", "flat_"))),
            "total": len(loop), "valu_histogram": dict(sorted(hist.items(), key=lambda kv: -kv[1]))}


def _smallest(loops, pred):
    best = None
    for lp in loops:
        if pred(lp) and (best is None or len(lp) < len(best)):
            best = lp
    return best


def analyse(asm: str, sym: str = K1_SYMBOL) -> dict:
    """Per-block counts of the wide kernel's streaming loop.  K1 absorbs two blocks (one 128-B
    line, eight 16-B loads) per iteration, and the second block sits behind a leaf-end branch that
    jumps to the latch, so the iteration is the LARGEST backward-branch region holding the loads
    (the smaller one ends at that branch and holds only the first block's rounds)."""
    loops = [l for l in _loops(_function_body(asm, sym))
             if sum(x.startswith("global_load_dwordx4") for x in l) >= 4]
    if not loops:
        raise ValueError("no block loop found")
    lp = max(loops, key=len)
    loads = sum(x.startswith("global_load_dwordx4") for x in lp)
    return _summary(lp, max(1, loads // 4))


def analyse_split(asm: str, sym: str) -> dict:
    loops = list(_loops(_function_body(asm, sym)))
    # K1Q runs whole ring stages (8 blocks from registers: 8 x 66 steps, each ending in one
    # v_add3_u32; 4 ds_read_b128 per block since the words are spread over a quad's lanes) when
    # every leaf of the wave has them: that loop is the bench path; otherwise the per-block loop
    # (16 reads)
    stage = _smallest(loops, lambda l: sum(x.startswith("v_add3_u32") for x in l) >= 8 * 66
                      and sum(x.startswith("ds_read_b128") for x in l) >= 32)
    if stage is not None:
        prod = _smallest(loops, lambda l: sum(x.startswith("ds_write_b128") for x in l) >= 16)
        if prod is None:
            raise ValueError(f"{sym}: producer loop not found")
        return {"consumer": _summary(stage, 8), "producer": _summary(prod, 1)}
    cons = _smallest(loops, lambda l: sum(x.startswith("ds_read_b128") for x in l) >= 16)
    prod = _smallest(loops, lambda l: sum(x.startswith("ds_write_b128") for x in l) >= 16)
    if cons is None or prod is None:
        raise ValueError(f"{sym}: consumer/producer loop not found")
    return {"consumer": _summary(cons, 1), "producer": _summary(prod, 1)}


def generate(write: bool = True) -> dict:
    """ISA counts of a fresh -save-temps build of the library; written to COUNTS unless write=False."""
    from . import build as b
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "lib.so")
        cmd = b.hipcc_cmd(out, extra=("-save-temps",))
        subprocess.run(cmd, check=True, cwd=td, capture_output=True)
        asm_files = [f for f in os.listdir(td) if f.endswith(".s") and "gfx950" in f]
        asm = open(os.path.join(td, asm_files[0])).read()
    res = {}
    for name, (sym, lanes) in KERNELS.items():
        if name == "wide":
            d = analyse(asm, sym)
            d["lane_slots_per_leaf_block"] = d["valu_slots"]
        else:
            d = analyse_split(asm, sym)
            d["lane_slots_per_leaf_block"] = (d["consumer"]["valu_slots"] * lanes[0] +
                                              d["producer"]["valu_slots"] * lanes[1])
            d["consumer_valu_per_block"] = d["consumer"]["valu"]
        d["kernel"] = sym
        d["lanes_per_leaf_block"] = {"consumer": lanes[0], "producer": lanes[1]}
        res[name] = d
    res["per"] = "one 64-byte block of one leaf"
    if write:
        with open(COUNTS, "w") as f:
            json.dump(res, f, indent=1)
    return res


def kernel_counts(kind: str = "wide"):
    """(VALU instructions per block on the leaf's critical wave, lane-slots per leaf-block)."""
    try:
        with open(COUNTS) as f:
            d = json.load(f)[kind]
    except (OSError, KeyError, ValueError):
        return None, None
    ops = d["valu"] if kind == "wide" else d["consumer_valu_per_block"]
    return ops, d["lane_slots_per_leaf_block"]


def valu_per_block():
    return kernel_counts("wide")


def chain_instructions_per_block(kind: str):
    """All instructions (VALU + LDS + SALU + ...) per block on the leaf's critical wave, from the
    same ISA counts: a wave issues at most one instruction per turn, whatever its type."""
    try:
        with open(COUNTS) as f:
            d = json.load(f)[kind]
    except (OSError, KeyError, ValueError):
        return None
    w = d if kind == "wide" else d.get("consumer", {})
    if "total" not in w or not w.get("blocks_per_iteration"):
        return None
    return w["total"] / w["blocks_per_iteration"]


if __name__ == "__main__":
    print(json.dumps(generate(), indent=1))
