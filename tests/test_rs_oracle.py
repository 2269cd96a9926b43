"""CPU tests of the Reed-Solomon restatement (oracle/rs_oracle.c + oracle/oracle.py py_rs_*).

The module it restates (klauspost/reedsolomon v1.12.4, go.mod:65) is not vendored: the pins are
the upstream library's own TestOneEncode known answer (tests/golden/rs_golden.json "kat") and
two independent restatements agreeing with each other and with the fixtures.
"""
from __future__ import annotations

import hashlib
import itertools
import json
import os
import random

import pytest

from oracle import py_rs_code, py_rs_encode, py_rs_matrix, py_rs_split, splitmix64_bytes

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "rs_golden.json")


@pytest.fixture(scope="module")
def rs_golden():
    with open(GOLDEN) as f:
        return json.load(f)


def test_klauspost_one_encode_kat(oracle_lib, rs_golden):
    kat = rs_golden["kat"]
    shards = [bytes(s) for s in kat["shards"]]
    assert [list(p) for p in oracle_lib.rs_encode(shards, kat["parity"])] == kat["parity_expected"]
    assert [list(p) for p in py_rs_encode(shards, kat["parity"])] == kat["parity_expected"]


def test_matrices_match_fixtures(oracle_lib, rs_golden):
    for m in rs_golden["matrices"]:
        k, t = m["data"], m["data"] + m["parity"]
        rows = [bytes(r).hex() for r in oracle_lib.rs_matrix(k, t)]
        assert rows == m["rows"]
        # systematic: the top square is the identity
        assert rows[:k] == [bytes(int(i == j) for j in range(k)).hex() for i in range(k)]


def test_encodes_match_fixtures(oracle_lib, rs_golden):
    for e in rs_golden["encodes"]:
        shards = py_rs_split(splitmix64_bytes(e["len"], e["seed"]), e["data"])
        assert len(shards[0]) == e["per_shard"]
        par = oracle_lib.rs_encode(shards, e["parity"], nthreads=2)
        assert [hashlib.sha256(p).hexdigest() for p in par] == e["parity_sha256"]


@pytest.mark.parametrize("k,m", [(4, 8), (4, 2), (6, 3), (1, 5), (8, 8)])
def test_c_and_python_restatements_agree(oracle_lib, k, m):
    rng = random.Random(k * 100 + m)
    shards = [bytes(rng.randrange(256) for _ in range(333)) for _ in range(k)]
    assert oracle_lib.rs_encode(shards, m) == py_rs_encode(shards, m)


def test_every_erasure_pattern_reconstructs_4_8(oracle_lib):
    """Any 4 of the 12 fragments rebuild all 12 (all C(12, 8) + smaller erasure sets)."""
    rng = random.Random(5)
    data = [bytes(rng.randrange(256) for _ in range(48)) for _ in range(4)]
    full = data + oracle_lib.rs_encode(data, 8)
    for nmiss in range(1, 9):
        for miss in itertools.combinations(range(12), nmiss):
            if nmiss < 8 and rng.random() > 0.05:
                continue   # all 495 maximal patterns, a sample of the smaller ones
            got = oracle_lib.rs_reconstruct(4, 8, [None if i in miss else s for i, s in enumerate(full)], 48)
            assert got == full, miss


def test_too_few_shards(oracle_lib):
    data = [bytes(16)] * 4
    full = data + oracle_lib.rs_encode(data, 8)
    with pytest.raises(ValueError, match="too few"):
        oracle_lib.rs_reconstruct(4, 8, [None] * 9 + full[9:], 16)


def test_linearity(oracle_lib):
    """encode(a ^ b) == encode(a) ^ encode(b): the code is GF(2)-linear."""
    rng = random.Random(9)
    a = [bytes(rng.randrange(256) for _ in range(64)) for _ in range(4)]
    b = [bytes(rng.randrange(256) for _ in range(64)) for _ in range(4)]
    x = [bytes(p ^ q for p, q in zip(u, v)) for u, v in zip(a, b)]
    pa, pb, px = (oracle_lib.rs_encode(s, 8) for s in (a, b, x))
    assert px == [bytes(p ^ q for p, q in zip(u, v)) for u, v in zip(pa, pb)]


def test_code_rows_identity():
    rows = py_rs_matrix(4, 12)
    shards = [bytes([i] * 8) for i in range(4)]
    assert py_rs_code(rows[:4], shards) == shards
