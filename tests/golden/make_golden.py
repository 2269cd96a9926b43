"""Generate tests/golden/merkle_golden.json from the pure-Python hashlib restatement.

Inputs are stored as generator parameters (splitmix64 seeds and lengths) or literal strings;
outputs are hex leaf digests and roots.  The only reference-pinned vector is the 4-leaf KAT of
common/hashtree/hashtree_test.go:20-82 ("content_one".."content_four"), included verbatim
with its expected values recomputed the way that test builds them.  Everything else is
"restatement-pinned" (Python hashlib SHA-256 + merkletree v0.2.0 semantics).

Run: python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
from oracle import py_go_tree, py_root_chunks, split_chunks, splitmix64_bytes  # noqa: E402

OUT = os.path.join(HERE, "merkle_golden.json")


def chunk_bytes(spec):
    if "text" in spec:
        return spec["text"].encode()
    return splitmix64_bytes(spec["len"], spec["seed"])


def splitmix64_np(nbytes: int, seed: int, off: int = 0):
    """Vectorised splitmix64 stream (same function as oracle.splitmix64_bytes, checked against it
    below) so the full-size BASELINE config roots can be generated in seconds."""
    import numpy as np
    i = np.arange(off // 8, (off + nbytes + 7) // 8, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) ^ i) + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").tobytes()[:nbytes]


def synthetic_object_root(length: int, chunk: int, seed: int):
    """Leaf digests + root of bytes [0, length) of the splitmix64 stream, leaf by leaf (hashlib)."""
    piece = 1 << 24
    leaves = []
    for b0 in range(0, length, chunk):
        h = hashlib.sha256()
        end = min(length, b0 + chunk)
        for p in range(b0, end, piece):
            h.update(splitmix64_np(min(piece, end - p), seed, p))
        leaves.append(h.digest())
    from oracle import py_reduce
    return leaves, py_reduce(leaves)[0]


def main() -> None:
    cases = []
    assert splitmix64_np(1000, 12345, 8) == splitmix64_bytes(1000, 12345, 8)
    # 1. reference KAT (hashtree_test.go:20-82), expected values built exactly like the test:
    #    root = SHA256( SHA256(L0||L1) || SHA256(L2||L3) )
    texts = ["content_one", "content_two", "content_three", "content_four"]
    L = [hashlib.sha256(t.encode()).digest() for t in texts]
    h5 = hashlib.sha256(L[0] + L[1]).digest()
    h6 = hashlib.sha256(L[2] + L[3]).digest()
    root = hashlib.sha256(h5 + h6).digest()
    cases.append({"name": "reference_kat_hashtree_test_go", "kind": "chunks",
                  "chunks": [{"text": t} for t in texts],
                  "leaves": [x.hex() for x in L], "root": root.hex(), "pinned": "reference"})
    # 2. leaf counts around powers of two, tiny chunks (odd-node duplication at every level)
    seed = 0xDE0550000
    for n in (1, 2, 3, 4, 5, 6, 7, 8, 9, 15, 16, 17, 31, 33, 255, 256, 257, 511, 513):
        chunks = [{"len": 1 + (i * 37) % 130, "seed": seed + 1000 * n + i} for i in range(n)]
        data = [chunk_bytes(c) for c in chunks]
        leaves, r = py_root_chunks(data)
        golang_leafs, r2 = py_go_tree(data)
        assert r == r2
        cases.append({"name": f"chunks_n{n}", "kind": "chunks", "chunks": chunks,
                      "leaves": [x.hex() for x in leaves], "root": r.hex(), "pinned": "restatement",
                      "go_leafs_len": len(golang_leafs)})
    # 3. SHA-256 padding boundaries (len mod 64 in {0,1,55,56,57,63}), 0-byte chunks
    lens = [0, 1, 3, 4, 55, 56, 57, 63, 64, 65, 119, 120, 121, 127, 128, 129, 1000, 4096, 4097]
    for ln in lens:
        chunks = [{"len": ln, "seed": seed + 7 + ln}]
        data = [chunk_bytes(c) for c in chunks]
        leaves, r = py_root_chunks(data)
        cases.append({"name": f"single_len{ln}", "kind": "chunks", "chunks": chunks,
                      "leaves": [x.hex() for x in leaves], "root": r.hex(), "pinned": "restatement"})
    chunks = [{"len": ln, "seed": seed + 99 + i} for i, ln in enumerate(lens)]
    data = [chunk_bytes(c) for c in chunks]
    leaves, r = py_root_chunks(data)
    cases.append({"name": "mixed_padding_lengths", "kind": "chunks", "chunks": chunks,
                  "leaves": [x.hex() for x in leaves], "root": r.hex(), "pinned": "restatement"})
    # 4. one object split into fixed chunks (short last chunk, aligned and unaligned sizes)
    for (length, chunk) in [(64 << 10, 4096), ((64 << 10) + 1, 4096), (100000, 1000), (100000, 17 * 64),
                            (5000, 1), (3 << 20, 1 << 20), ((3 << 20) - 5, 1 << 20), (1, 64),
                            (64, 64), (65, 64), (777, 100), (1 << 20, 64), (200000, 4093)]:
        s = seed + length + chunk
        buf = splitmix64_bytes(length, s)
        data = split_chunks(buf, chunk)
        leaves, r = py_root_chunks(data)
        case = {"name": f"buffer_{length}_{chunk}", "kind": "buffer", "len": length, "chunk": chunk,
                "seed": s, "n_leaves": len(data), "root": r.hex(), "pinned": "restatement"}
        if len(leaves) <= 600:
            case["leaves"] = [x.hex() for x in leaves]
        else:   # checksum of the concatenated leaf digests keeps the fixture small
            case["leaves_sha256"] = hashlib.sha256(b"".join(leaves)).hexdigest()
        cases.append(case)
    # 5. batch of independent objects (one root each)
    objs = [{"len": ln, "seed": seed + 5000 + i} for i, ln in
            enumerate([1, 64, 100, 4096, 5000, 65536, 70000, 12345, 3, 200000])]
    chunk = 4096
    roots = []
    for o in objs:
        data = split_chunks(splitmix64_bytes(o["len"], o["seed"]), chunk)
        roots.append(py_root_chunks(data)[1].hex())
    cases.append({"name": "batch_10_objects", "kind": "batch", "objects": objs, "chunk": chunk,
                  "roots": roots, "pinned": "restatement"})
    # 6. BASELINE configs at full size (seeds 0xDE0550000 + k):
    #    configs[0] = one 64 MiB object at 32 MiB chunks (2 leaves; the CPU plumbing config),
    #    configs[1] = one 8 GiB object at 32 MiB chunks (256 leaves; the bench headline).
    for k, length in ((0, 64 << 20), (1, 8 << 30)):
        s = seed + k if k == 0 else seed + 2      # bench.py SEED = 0xDE0550002 for configs[1]
        leaves, r = synthetic_object_root(length, 32 << 20, s)
        cases.append({"name": f"config{k}_{length >> 20}MiB_chunk32MiB", "kind": "buffer", "len": length,
                      "chunk": 32 << 20, "seed": s, "n_leaves": len(leaves), "root": r.hex(),
                      "leaves_sha256": hashlib.sha256(b"".join(leaves)).hexdigest(),
                      "pinned": "restatement", "full_size": True})
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py (Python hashlib restatement)",
                   "synthetic": "word[i] = splitmix64(seed ^ i), little-endian", "cases": cases}, f, indent=0)
    print(f"wrote {OUT}: {len(cases)} cases")


if __name__ == "__main__":
    main()
