"""Generate tests/golden/rs_golden.json (Reed-Solomon fragment coding fixtures).

Pins:
* ``klauspost_TestOneEncode``: the known answer of klauspost/reedsolomon's own unit test
  (``reedsolomon_test.go`` TestOneEncode, ported from Backblaze JavaReedSolomon): New(5, 5),
  data shards {0,1} {4,5} {2,3} {6,7} {8,9} -> parity {12,13} {10,11} {14,15} {90,91} {94,95}.
  The module (go.mod:65, v1.12.4) is not vendored under /root/reference; this vector is
  restated from the upstream test, and the restatements below reproduce it.
* everything else is restatement-pinned (pure-Python GF(2^8) arithmetic, no log tables):
  encoding matrices of the shapes DeOSS and the tests use, and parity digests of seeded data.

Run: python tests/golden/make_rs_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
from oracle import py_rs_encode, py_rs_matrix, py_rs_split, splitmix64_bytes  # noqa: E402

OUT = os.path.join(HERE, "rs_golden.json")


def main() -> None:
    kat = {"name": "klauspost_TestOneEncode", "data": 5, "parity": 5,
           "shards": [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]],
           "parity_expected": [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]}
    got = [list(p) for p in py_rs_encode([bytes(s) for s in kat["shards"]], 5)]
    assert got == kat["parity_expected"], got
    matrices = []
    for k, m in [(4, 8), (4, 2), (5, 5), (8, 8), (1, 1), (3, 7)]:
        matrices.append({"data": k, "parity": m, "rows": [bytes(r).hex() for r in py_rs_matrix(k, k + m)]})
    encodes = []
    for k, m, length, seed in [(4, 8, 1, 11), (4, 8, 63, 12), (4, 8, 4096, 13), (4, 8, 100003, 14),
                               (3, 7, 999, 15), (8, 8, 65536, 16), (2, 3, 17, 17)]:
        buf = splitmix64_bytes(length, 0xDE055500 + seed)
        shards = py_rs_split(buf, k)
        par = py_rs_encode(shards, m)
        encodes.append({"data": k, "parity": m, "len": length, "seed": 0xDE055500 + seed,
                        "per_shard": len(shards[0]),
                        "parity_sha256": [hashlib.sha256(p).hexdigest() for p in par]})
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_rs_golden.py", "kat": kat, "matrices": matrices,
                   "encodes": encodes}, f, indent=1)


if __name__ == "__main__":
    main()
