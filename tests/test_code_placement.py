"""Code placement of the K1Q step streams in the built library (CPU only: reads the gfx950 code
object out of libdeoss_merkle.so and disassembles it).

Every K1Q step instruction is 8 bytes, and on MI355X where the stream sits mod 8 changed the rate
by 15-19 % (profiles/r01/r01f_align_ab.log): the wide kernel (<= 2 workgroups per
CU, the headline) must run at 0 mod 8, the compact kernel (4 per CU) at 4 mod 8.  The kernels
pin this with `.p2align 3` (+ one s_nop for the compact one); this test keeps a later edit from
silently undoing it.
"""
import collections
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "deoss_amd", "libdeoss_merkle.so")
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _disassemble(tmp_path):
    fat = tmp_path / "fat.bin"
    elf = tmp_path / "gfx950.elf"
    # -O binary with an explicit output file: objcopy without one rewrites its input in place,
    # which corrupts the library under any process that has it mapped
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB, str(fat)], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    f"--targets={TARGET}", f"--output={elf}"], check=True)
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", str(elf)], check=True,
                         capture_output=True, text=True)
    return out.stdout


def _step_placement(asm):
    """{kernel symbol: Counter(address mod 8 of its v_xor_b32_dpp step instructions)}"""
    res = {}
    for m in re.finditer(r"^[0-9a-f]+ <(_ZN2dm16leaf_kernel_quad\w+)>:", asm, re.M):
        end = asm.find("\n\n", m.end())
        c = collections.Counter()
        for ln in asm[m.end():end].splitlines():
            if "v_xor_b32_dpp" in ln:
                a = re.search(r"//\s*([0-9A-F]+):", ln)
                c[int(a.group(1), 16) % 8] += 1
        res[m.group(1)] = c
    return res


@pytest.mark.skipif(not os.path.exists(LIB) or shutil.which("objcopy") is None
                    or not os.path.exists(f"{LLVM}/llvm-objdump"),
                    reason="built library or LLVM tools missing")
def test_k1q_step_streams_pinned(tmp_path):
    placement = _step_placement(_disassemble(tmp_path))
    assert len(placement) == 8, sorted(placement)   # TABLE x ALIGNED x COMPACT
    for sym, c in placement.items():
        compact = sym.endswith("ELb1EEEvNS_8LeafArgsE")
        want = 4 if compact else 0
        # the register path (8 blocks per ring stage, 1,056 of these per kernel) is the hot one;
        # the ragged-tail path (quad_block_skewed) is aligned to 0 in both kernels
        assert c[want] >= 1056, (sym, dict(c))
