"""CPU tests of the multi-device dispatch rules (deoss_amd/csrc/shard_plan.hpp): no GPU needed.

1. The partition the library applies (dm_plan_shards) equals deoss_amd.sharding.plan_shards, the
   rule of the one-process-per-GPU path, for G = 1..8 devices and n = 1..600 leaves (+ large n).
2. tests/cpp/test_shard_plan.cpp, built plain and with ASan/UBSan, checks the same table, the
   partition's invariants and that composing per-device k-level subtrees gives the oracle's root.
3. The routing decision table (dm_plan_route): which calls run whole on one device and which are
   sharded, for the shapes DeOSS and the BASELINE configs produce on an 8-GPU node.
"""
import ctypes
import os
import shutil
import subprocess

import pytest

from deoss_amd.sharding import plan_shards

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MiB, GiB = 1 << 20, 1 << 30
SRC = {"device": 0, "pinned": 1, "pageable": 2, "files": 3}
LARGE_N = (1023, 1024, 1025, 4096, 32768, 100000, (1 << 18) + 3)


@pytest.fixture(scope="module")
def lib():
    from deoss_amd import build as b
    b.build(verbose=False)
    from deoss_amd import load_library
    return load_library()


def lib_plan(lib, n, G):
    k = ctypes.c_uint32()
    nb = ctypes.c_uint64()
    lo = (ctypes.c_uint64 * G)()
    hi = (ctypes.c_uint64 * G)()
    assert lib.dm_plan_shards(n, G, ctypes.byref(k), ctypes.byref(nb), lo, hi) == 0
    return k.value, nb.value, list(zip(lo, hi))


def py_plan(n, G):
    p = plan_shards(n, 1, G)
    return p.k, p.n_blocks, [p.leaf_range(r) for r in range(G)]


def test_library_partition_equals_plan_shards(lib):
    for G in range(1, 9):
        for n in list(range(1, 601)) + list(LARGE_N):
            assert lib_plan(lib, n, G) == py_plan(n, G), (G, n)


def test_plan_shards_cpp_plain_and_asan(tmp_path):
    """The C++ partition against plan_shards' table, its invariants and the composed root."""
    table = tmp_path / "plan_table.txt"
    with open(table, "w") as f:
        for G in range(1, 9):
            for n in list(range(1, 601)) + list(LARGE_N):
                k, nb, ranges = py_plan(n, G)
                f.write(f"{G} {n} {k} {nb} " + " ".join(f"{a} {b}" for a, b in ranges) + "\n")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    src = os.path.join(ROOT, "tests", "cpp", "test_shard_plan.cpp")
    oracle_lib = ["-L", os.path.join(ROOT, "oracle"), "-loracle_merkle",
                  "-Wl,-rpath," + os.path.join(ROOT, "oracle")]
    builds = [("plain", ["g++", "-O2", "-std=c++17", "-Wall", "-Werror"])]
    clang = "/opt/rocm/lib/llvm/bin/clang++"
    if os.path.exists(clang):
        builds.append(("asan", [clang, "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                                "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]))
    elif shutil.which("g++"):
        builds.append(("asan", ["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                                "-fno-sanitize-recover=all"]))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    for name, cc in builds:
        exe = str(tmp_path / f"test_shard_plan_{name}")
        subprocess.run(cc + [src, "-o", exe] + oracle_lib, check=True)
        out = subprocess.run([exe, str(table)], capture_output=True, text=True, env=env)
        assert out.returncode == 0, (name, out.stdout, out.stderr)
        assert "shard plan OK" in out.stdout


def route(lib, n, nbytes, leaf_max, src, G=8, cus=256, mode=0, busy=0, by_objects=False):
    est = (ctypes.c_double * G)()
    r = lib.dm_plan_route(n, nbytes, leaf_max, SRC[src], int(by_objects), G, cus, mode, busy, est)
    assert r >= 1
    return r, list(est)


# (what, leaves, bytes, longest leaf, source, expected devices on an 8-GPU node); "batch" = split by objects
DECISIONS = [
    # NewHashTree over DeOSS's 256 x 32 MiB segment files: every chain is resident on one GPU, so the
    # call runs whole on one GPU (~0.5 s either way); concurrent calls go to different GPUs
    ("NewHashTree 256 x 32 MiB files", 256, 8 * GiB, 32 * MiB, "files", 1),
    ("configs[1] 8 GiB @ 32 MiB, pinned host buffer", 256, 8 * GiB, 32 * MiB, "pinned", 1),
    ("configs[1] 8 GiB @ 32 MiB, pageable host buffer", 256, 8 * GiB, 32 * MiB, "pageable", 1),
    ("configs[0] 64 MiB @ 32 MiB", 2, 64 * MiB, 32 * MiB, "pinned", 1),
    ("one 32 MiB segment", 1, 32 * MiB, 32 * MiB, "pinned", 1),
    ("4 MiB object @ 4 KiB chunks (tiny calls never shard)", 1024, 4 * MiB, 4096, "pinned", 1),
    ("device-resident objects never move", 32768, 1 << 40, 32 * MiB, "device", 1),
    # past full-speed residency / PCIe-bound: more devices bring more links and more SIMDs
    ("configs[3] 1 TiB @ 32 MiB from host", 32768, 1 << 40, 32 * MiB, "pinned", 8),
    ("8 GiB @ 1 MiB chunks, pinned (PCIe-bound on one GPU)", 8192, 8 * GiB, MiB, "pinned", 8),
    ("8 GiB @ 4 KiB chunks, pinned", 2 * MiB, 8 * GiB, 4096, "pinned", 8),
    ("configs[4] 100k x 1 MiB batch from host", 100000, 100000 * MiB, MiB, "pinned batch", 8),
    # PCIe-bound up to 5 GPUs; there the 4 MiB chains (63 ms) bound it and more GPUs add nothing
    ("configs[2] 4096 x 4 MiB batch from host", 4096, 16 * GiB, 4 * MiB, "pinned batch", 5),
    ("16 x 1 MiB uploads in one batch call", 16, 16 * MiB, MiB, "pinned batch", 1),
]


@pytest.mark.parametrize("what,n,nbytes,leaf_max,src,want", DECISIONS, ids=[d[0] for d in DECISIONS])
def test_route_decision_table(lib, what, n, nbytes, leaf_max, src, want):
    batch = src.endswith(" batch")
    src = src.split()[0]
    got, est = route(lib, n, nbytes, leaf_max, src, by_objects=batch)
    assert got == want, (what, got, [round(x, 2) for x in est])
    if want == 1 and src != "device":
        assert min(est[1:]) >= 0.95 * est[0]   # no device count is >= 5 % sooner


def route_constants(lib):
    ag, hb = ctypes.c_double(), ctypes.c_double()
    assert lib.dm_route_constants(None, ctypes.byref(ag), ctypes.byref(hb)) == 0
    return ag.value, hb.value


def test_route_constants_from_the_environment(lib, monkeypatch):
    """the N = 8 bench line's measured all-gather and host-feed rates replace
    the model's two estimates without a code change (DEOSS_ALLGATHER_US, DEOSS_HOST_BYTES_PER_S,
    printed by that line as route_constants).  Each override flips the decision it governs."""
    monkeypatch.delenv("DEOSS_ALLGATHER_US", raising=False)
    monkeypatch.delenv("DEOSS_HOST_BYTES_PER_S", raising=False)
    assert route_constants(lib) == (100.0, 500e9)
    cfg3 = (32768, 1 << 40, 32 * MiB, "pinned")             # configs[3] from host: 8 GPUs by default
    small = (2 * MiB, 8 * GiB, 4096, "pinned")             # 8 GiB @ 4 KiB: 8 GPUs by default
    assert route(lib, *cfg3)[0] == 8 and route(lib, *small)[0] == 8
    # a host that feeds all GPUs together no faster than one PCIe link: nothing gains from sharding
    monkeypatch.setenv("DEOSS_HOST_BYTES_PER_S", "50e9")
    assert route_constants(lib) == (100.0, 50e9)
    assert route(lib, *cfg3)[0] == 1
    monkeypatch.delenv("DEOSS_HOST_BYTES_PER_S")
    # an all-gather of 1 s outweighs the 156 ms one GPU takes over PCIe
    monkeypatch.setenv("DEOSS_ALLGATHER_US", "1000000")
    assert route_constants(lib)[0] == 1e6
    assert route(lib, *small)[0] == 1 and route(lib, *cfg3)[0] == 8   # 1 s is nothing against 20 s
    # a measured all-gather of 41.5 us (what a real line would print) changes none of the table's decisions
    monkeypatch.setenv("DEOSS_ALLGATHER_US", "41.5")
    for what, n, nbytes, leaf_max, src, want in DECISIONS:
        batch = src.endswith(" batch")
        assert route(lib, n, nbytes, leaf_max, src.split()[0], by_objects=batch)[0] == want, what
    # malformed, zero or negative values are ignored: the estimates stay
    for bad in ("", "abc", "0", "-5", "1e400", "12us"):
        monkeypatch.setenv("DEOSS_ALLGATHER_US", bad)
        monkeypatch.setenv("DEOSS_HOST_BYTES_PER_S", bad)
        assert route_constants(lib) == (100.0, 500e9), bad


def test_route_never_shards_a_busy_context(lib):
    assert route(lib, 32768, 1 << 40, 32 * MiB, "pinned")[0] == 8
    assert route(lib, 32768, 1 << 40, 32 * MiB, "pinned", busy=1)[0] == 1
    assert route(lib, 32768, 1 << 40, 32 * MiB, "pinned", G=1)[0] == 1


def test_route_picks_fewer_devices_for_mid_sizes(lib):
    """Between 'one device' and 'all devices' the model may take a subset (e.g. 2 or 4)."""
    seen = set()
    for mib in (64, 128, 256, 512, 1024, 4096):
        g, _ = route(lib, mib * 256, mib * MiB, 4096, "pinned")
        seen.add(g)
        assert 1 <= g <= 8
    assert max(seen) == 8 and len(seen) >= 2


def test_route_rejects_bad_arguments(lib):
    assert lib.dm_plan_route(1, 1, 1, 9, 0, 8, 256, 0, 0, None) == -2
    assert lib.dm_plan_route(1, 1, 1, 0, 0, 0, 256, 0, 0, None) == -2
    k = ctypes.c_uint32()
    nb = ctypes.c_uint64()
    assert lib.dm_plan_shards(10, 0, ctypes.byref(k), ctypes.byref(nb), None, None) == -2
