"""Full-size roots of the objects the N > 1 bench legs hash, so those legs check their roots
against a committed fixture instead of re-hashing up to 64 GiB on the host CPU inside the
driver's time limit ("make the first real 8-GPU line impossible to lose"):

  weak_n{2,4,8}: the weak-scaling headline at N GPUs, one object of N x 8 GiB at 32 MiB chunks
                 (bench.py --gpus N; the 64 GiB one is also configs[3]'s 64 GiB parity prefix);
  strong_4KiB:   configs[1]'s 8 GiB object at 4 KiB chunks (the strong_scaling_4KiB leg).

All are prefixes of the splitmix64 stream with bench.py's seed (the same bytes the GPU fills at
each rank's byte offset), regenerated leaf by leaf by the C oracle (or_root_synthetic; no
whole-object buffer).  The 8 GiB / 32 MiB object is configs[1]'s fixture in merkle_golden.json
and the 1 TiB one is config3_root.json.  About 30 s on 8 cores.
usage: python tests/golden/make_scale_roots.py [threads]"""
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
    from oracle import Oracle, py_reduce
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 1)
    orc = Oracle()
    out = {"generator": "tests/golden/make_scale_roots.py (oracle/merkle_oracle.c or_root_synthetic_at)",
           "seed": SEED, "pinned": "restatement", "roots": []}
    t0 = time.time()
    chunk = 32 << 20
    leaves, root64 = orc.root_synthetic(64 << 30, chunk, SEED, nthreads=threads, want_leaves=True)
    lv = [leaves[32 * i:32 * i + 32] for i in range(len(leaves) // 32)]
    for n in (2, 4, 8):   # N x 8 GiB = the first N x 256 leaves of the same stream
        r = py_reduce(lv[:256 * n])[0]
        out["roots"].append({"name": f"weak_n{n}", "len": n << 33, "chunk": chunk, "n_leaves": 256 * n,
                             "root": r.hex()})
    assert out["roots"][-1]["root"] == root64.hex()
    assert py_reduce(lv[:256])[0].hex() == "ca268004b8ebf66190268e9909b243c36789f542fdec9b89d9b3ec18753b152f"
    _, r4k = orc.root_synthetic(8 << 30, 4096, SEED, nthreads=threads)
    out["roots"].append({"name": "strong_4KiB", "len": 8 << 30, "chunk": 4096, "n_leaves": (8 << 30) // 4096,
                         "root": r4k.hex()})
    out["seconds"] = round(time.time() - t0, 1)
    with open(os.path.join(HERE, "scale_roots.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
