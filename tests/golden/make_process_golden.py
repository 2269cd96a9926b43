"""Generate tests/golden/process_golden.json (FullProcessing and Merkle-proof fixtures).

FullProcessing (cess-go-sdk process.FullProcessing with cipher "", go.mod:8; SDK not vendored):
restated as zero-padded segments -> RS(data, parity) fragments -> SHA-256 names -> fid = hashtree
root over the segments (oracle/process_oracle.c header).  The composition is parity-UNPINNED
(no SDK source or fixture exists offline); its parts are pinned by the hashtree KAT, NIST SHA-256
vectors and klauspost TestOneEncode.  Cases use small segments so the pure-Python restatement
runs in seconds; one case uses the real 32 MiB segment / 4 + 8 shape with a short object.

Merkle proofs (merkletree v0.2.0 GetMerklePath, go.mod:10; not vendored): paths and indices from
the literal Node/Parent restatement (oracle.py py_get_merkle_path), leaf contents chosen to
include duplicates (the reference's hash-equality index rule) and odd counts (the dup leaf).

Inputs are generator parameters (splitmix64 seeds); outputs are hex digests.
Run: python tests/golden/make_process_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
from oracle import (py_full_processing, py_get_merkle_path, py_root_chunks,  # noqa: E402
                    splitmix64_bytes)

OUT = os.path.join(HERE, "process_golden.json")
SEED0 = 0xDE0551000


def proof_chunks(n: int, seed: int):
    """n leaf contents, every third one repeating an earlier one (duplicate digests)."""
    out = []
    for i in range(n):
        if i % 3 == 2:
            out.append(out[i // 2])
        else:
            out.append(splitmix64_bytes(1 + (seed + i) % 97, seed + i))
    return out


def main() -> None:
    process = []
    for length, segment, k, m, seed in [(1, 64, 4, 8, 1), (64, 64, 4, 8, 2), (65, 64, 4, 8, 3),
                                        (1000, 256, 4, 8, 4), (4096, 1024, 4, 8, 5), (5000, 512, 4, 2, 6),
                                        (777, 96, 3, 5, 7), (70000, 4096, 4, 8, 8), (123457, 16384, 8, 8, 9),
                                        (100, 32 << 20, 4, 8, 10)]:
        buf = splitmix64_bytes(length, SEED0 + seed)
        segs, frag_h, fid, frags = py_full_processing(buf, segment, k, m)
        process.append({"len": length, "segment": segment, "data": k, "parity": m, "seed": SEED0 + seed,
                        "segment_hashes": [h.hex() for h in segs],
                        "fragment_hashes": [[h.hex() for h in row] for row in frag_h],
                        "fid": fid.hex()})
    proofs = []
    for n, seed in [(1, 1), (2, 2), (3, 3), (4, 4), (5, 5), (7, 6), (8, 7), (9, 8), (13, 9), (33, 10)]:
        chunks = proof_chunks(n, SEED0 + 100 * seed)
        leaves, root = py_root_chunks(chunks)
        paths = []
        for i in range(n):
            path, index = py_get_merkle_path(chunks, chunks[i])
            paths.append({"leaf": i, "path": [p.hex() for p in path], "index": index})
        proofs.append({"n": n, "seed": SEED0 + 100 * seed, "root": root.hex(),
                       "leaves": [l.hex() for l in leaves], "paths": paths})
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_process_golden.py", "process": process, "proofs": proofs}, f,
                  indent=0)


if __name__ == "__main__":
    main()
