"""CPU tests of the FullProcessing and Merkle-proof restatements (oracle/, test infrastructure).

FullProcessing (cess-go-sdk, go.mod:8) is a restated composition -- parity UNPINNED against the SDK
itself (absent offline) -- whose parts are pinned: SHA-256 (NIST), the hashtree root
(hashtree_test.go:20-82), the RS coder (klauspost TestOneEncode).  Here: the C restatement
(oracle/process_oracle.c) against the fixtures and the pure-Python restatement, and the
composition's structural properties.  Proofs: merkletree v0.2.0 GetMerklePath restated literally
(Node graph with Parent pointers, oracle.py) against an independent level-array path builder and
the fixtures; every proof folds to the root.
"""
from __future__ import annotations

import hashlib
import json
import os

import pytest

from oracle import (py_fold_path, py_full_processing, py_get_merkle_path, py_reduce, py_root_chunks,
                    py_rs_encode, py_rs_split, py_sha256, splitmix64_bytes)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "process_golden.json")


@pytest.fixture(scope="module")
def pg():
    with open(GOLDEN) as f:
        return json.load(f)


def test_c_full_processing_matches_fixtures(oracle_lib, pg):
    for c in pg["process"]:
        buf = splitmix64_bytes(c["len"], c["seed"])
        seg, frag, fid, _ = oracle_lib.full_processing(buf, c["segment"], c["data"], c["parity"], nthreads=2)
        total = c["data"] + c["parity"]
        assert [seg[i:i + 32].hex() for i in range(0, len(seg), 32)] == c["segment_hashes"]
        rows = [[frag[32 * (s * total + j):32 * (s * total + j) + 32].hex() for j in range(total)]
                for s in range(len(c["segment_hashes"]))]
        assert rows == c["fragment_hashes"]
        assert fid.hex() == c["fid"]


def test_composition_properties(oracle_lib):
    """fid = hashtree root over zero-padded segments; data fragments = the segment in order;
    parity = RS of the data fragments; names = SHA-256 of the fragment bytes."""
    buf = splitmix64_bytes(3000, 77)
    seg_b, frag_b, fid, frags = oracle_lib.full_processing(buf, 1024, 4, 8, want_frags=True)
    padded = buf + bytes(3 * 1024 - len(buf))
    segs = [padded[i * 1024:(i + 1) * 1024] for i in range(3)]
    assert fid == py_root_chunks(segs)[1]
    for s in range(3):
        row = [frags[(s * 12 + j) * 256:(s * 12 + j + 1) * 256] for j in range(12)]
        assert b"".join(row[:4]) == segs[s]
        assert row[4:] == py_rs_encode(py_rs_split(segs[s], 4), 8)
        for j in range(12):
            assert frag_b[32 * (s * 12 + j):32 * (s * 12 + j + 1)] == hashlib.sha256(row[j]).digest()
        assert seg_b[32 * s:32 * s + 32] == py_sha256(segs[s])


def test_c_and_python_restatements_agree(oracle_lib):
    for length, segment in [(1, 64), (640, 64), (641, 128), (9999, 2048)]:
        buf = splitmix64_bytes(length, length)
        segs, frag_h, fid, frags = py_full_processing(buf, segment)
        s, f, fi, fr = oracle_lib.full_processing(buf, segment, want_frags=True)
        assert s == b"".join(segs) and f == b"".join(sum(frag_h, [])) and fi == fid
        assert fr == b"".join(sum(frags, []))


def test_empty_object_is_an_error(oracle_lib):
    with pytest.raises(ValueError):
        oracle_lib.full_processing(b"", 64)
    with pytest.raises(ValueError):
        py_full_processing(b"", 64)


def _level_paths(leaves, i):
    """Independent path builder over level arrays (the kernels' rule)."""
    path, bits, lev, p = [], [], list(leaves), i
    while True:
        c = len(lev)
        j = p // 2
        left, right = lev[2 * j], lev[min(2 * j + 1, c - 1)]
        if left == lev[p]:
            path.append(right)
            bits.append(1)
        else:
            path.append(left)
            bits.append(0)
        lev = [py_sha256(lev[2 * k] + lev[min(2 * k + 1, c - 1)]) for k in range((c + 1) // 2)]
        p = j
        if len(lev) == 1:
            return path, bits


def test_proof_fixtures_match_literal_and_level_rules(pg):
    for case in pg["proofs"]:
        n = case["n"]
        leaves = [bytes.fromhex(h) for h in case["leaves"]]
        root = bytes.fromhex(case["root"])
        assert py_reduce(leaves)[0] == root
        for p in case["paths"]:
            path = [bytes.fromhex(h) for h in p["path"]]
            i = p["leaf"]
            # the first leaf with the same digest gets the path (merkletree scans with Equals)
            first = leaves.index(leaves[i])
            assert _level_paths(leaves, first) == (path, p["index"])
            assert py_fold_path(leaves[i], path, p["index"]) == root
            assert len(path) == max(1, (n - 1).bit_length())


@pytest.mark.parametrize("n", list(range(1, 70)) + [127, 128, 129, 255, 256, 257])
def test_literal_get_merkle_path_equals_level_rule(n):
    chunks = [bytes([i % 5, i % 3]) for i in range(n)]   # many duplicate contents
    leaves, root = py_root_chunks(chunks)
    for i in range(n):
        first = chunks.index(chunks[i])
        path, index = py_get_merkle_path(chunks, chunks[i])
        assert (path, index) == _level_paths(leaves, first)
        assert py_fold_path(leaves[i], path, index) == root


def test_get_merkle_path_missing_content():
    assert py_get_merkle_path([b"a", b"b"], b"c") == (None, None)
