"""BASELINE configs[3]'s root at full size: one 1 TiB object (32,768 leaves of 32 MiB) of the
splitmix64 stream with bench.py's seed, regenerated leaf by leaf by the C oracle
(or_root_synthetic, threads over leaves; no whole-object buffer).  The N = 8 bench line's
configs[3] entry hashes exactly these bytes, so its root must equal this one; the GPU test
tests/test_configs_gpu.py::test_configs3_full_object_shard_by_shard_on_one_gpu reproduces it on
one MI355X shard by shard.  About 3 minutes on 8 cores.
usage: python tests/golden/make_config3_root.py [threads]"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    from bench_common import SEED
    from oracle import Oracle
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 1)
    length, chunk = 1 << 40, 32 << 20
    t0 = time.time()
    leaves, root = Oracle().root_synthetic(length, chunk, SEED, nthreads=threads, want_leaves=True)
    import hashlib
    out = {"name": "config3_1TiB_chunk32MiB", "len": length, "chunk": chunk, "seed": SEED,
           "n_leaves": len(leaves) // 32, "root": root.hex(),
           "leaves_sha256": hashlib.sha256(leaves).hexdigest(),
           "generator": "tests/golden/make_config3_root.py (oracle/merkle_oracle.c or_root_synthetic_at)",
           "pinned": "restatement", "seconds": round(time.time() - t0, 1)}
    # the 8 per-GPU block roots (2^12 leaves each) the sharded path gathers, from the same leaves
    from oracle import py_reduce
    lv = [leaves[32 * i:32 * i + 32] for i in range(len(leaves) // 32)]
    out["shard_roots_k12"] = [b.hex() for b in py_reduce(lv, 12)]
    assert py_reduce([bytes.fromhex(h) for h in out["shard_roots_k12"]])[0] == root
    with open(os.path.join(HERE, "config3_root.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("root", "n_leaves", "seconds")}))


if __name__ == "__main__":
    main()
