"""The instruction counts bench.py puts into its roofline (deoss_amd/isa_counts.json: VALU and
all instructions per block on each leaf kernel's critical wave) must describe the current
sources: regenerate them from a -save-temps build of the library and compare.  CPU only (hipcc
cross-compiles gfx950 here); about a minute."""
import json

from deoss_amd import isa


def test_isa_counts_match_current_build():
    with open(isa.COUNTS) as f:           # the committed counts, read before anything regenerates them
        committed = json.load(f)
    fresh = isa.generate(write=False)
    for kind in ("wide", "latency", "pair", "quad"):
        a, b = fresh[kind], committed[kind]
        wa = a if kind == "wide" else a["consumer"]
        wb = b if kind == "wide" else b["consumer"]
        for field in ("valu", "valu_slots", "total", "blocks_per_iteration"):
            assert wa[field] == wb[field], (kind, field, wa[field], wb[field])
        assert isa.chain_instructions_per_block(kind) == wb["total"] / wb["blocks_per_iteration"]
    # K1Q's register path: a block's 64 words of -(K+W) spread over a quad's 4 lanes, so the
    # chain's wave issues 4 ds_read_b128 per block (16 before round 3)
    q = fresh["quad"]["consumer"]
    assert q["lds"] == 4 * q["blocks_per_iteration"], q["lds"]
