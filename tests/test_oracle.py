"""CPU: pin the oracle (oracle/) to the crate's published known answers,
FIPS 180-4 / hashlib, an independent pure-Python GF restatement, and the
committed golden fixtures.  No GPU."""
from __future__ import annotations

import hashlib
import itertools

import numpy as np
import pytest

import oracle
from helpers import data_for, sha_vector_inputs

# ---- independent pure-Python restatement (small sizes only) ---------------


def _py_tables():
    exp, log = [0] * 510, [0] * 256
    b = 1
    for i in range(255):
        exp[i] = exp[i + 255] = b
        log[b] = i
        b <<= 1
        if b & 0x100:
            b ^= 0x11D
    return exp, log


EXP, LOG = _py_tables()


def py_mul(a, b):
    return 0 if a == 0 or b == 0 else EXP[LOG[a] + LOG[b]]


def py_inv_matrix(m):
    n = len(m)
    w = [row[:] + [1 if i == r else 0 for i in range(n)] for r, row in enumerate(m)]
    for c in range(n):
        p = next(r for r in range(c, n) if w[r][c])
        w[c], w[p] = w[p], w[c]
        inv = EXP[(255 - LOG[w[c][c]]) % 255]
        w[c] = [py_mul(inv, x) for x in w[c]]
        for r in range(n):
            if r != c and w[r][c]:
                s = w[r][c]
                w[r] = [x ^ py_mul(s, y) for x, y in zip(w[r], w[c])]
    return [row[n:] for row in w]


def py_matrix(k, m):
    v = [[1 if c == 0 else (0 if r == 0 else EXP[(LOG[r] * c) % 255]) for c in range(k)] for r in range(k + m)]
    ti = py_inv_matrix(v[:k])
    out = []
    for row in v:
        o = []
        for c in range(k):
            acc = 0
            for i in range(k):
                acc ^= py_mul(row[i], ti[i][c])
            o.append(acc)
        out.append(o)
    return out


# ---- known answers ------------------------------------------------------------


def test_galois_known_answers(golden):
    kat = golden("rs_kat.json")
    for a, b, want in kat["gf_mul"]:
        assert oracle.gf_mul(a, b) == want
    for a, b, want in kat["gf_div"]:
        assert oracle.gf_div(a, b) == want
    for a, n, want in kat["gf_exp"]:
        assert oracle.gf_exp(a, n) == want


def test_gf_tables_match_pure_python():
    for a in range(256):
        for b in range(0, 256, 7):
            assert oracle.gf_mul(a, b) == py_mul(a, b)


def test_one_encode_crate_vector(golden):
    kat = golden("rs_kat.json")["one_encode"]
    parity = oracle.encode([bytes(d) for d in kat["data"]], kat["m"])
    assert [p.tolist() for p in parity] == kat["parity"]


def test_parity_rows_fixture(golden):
    rows = golden("rs_kat.json")["parity_rows"]
    for key, want in rows.items():
        k, m = map(int, key.split("+"))
        assert oracle.matrix(k, m)[k:].tolist() == want
    # SURVEY.md §8(c) listed these rows from a separate throwaway restatement.
    assert rows["4+2"] == [[27, 28, 18, 20], [28, 27, 20, 18]]
    assert rows["1+2"] == [[1], [1]]


@pytest.mark.parametrize("k,m", [(1, 1), (2, 3), (4, 2), (5, 5), (8, 4), (10, 4), (13, 7)])
def test_matrix_matches_pure_python(k, m):
    assert oracle.matrix(k, m).tolist() == py_matrix(k, m)


@pytest.mark.parametrize("k,m", [(1, 2), (8, 4), (64, 4), (128, 127), (253, 2)])
def test_matrix_is_systematic(k, m):
    mat = oracle.matrix(k, m)
    assert np.array_equal(mat[:k], np.eye(k, dtype=np.uint8))


def test_rs_new_errors():
    assert oracle.rs_check(0, 1) == -3      # TooFewDataShards
    assert oracle.rs_check(1, 0) == -5      # TooFewParityShards
    assert oracle.rs_check(200, 57) == -2   # TooManyShards (> 256)
    assert oracle.rs_check(200, 56) == 0


# ---- SHA-256 ---------------------------------------------------------------------


def test_sha256_vectors(golden):
    sv = golden("sha256_vectors.json")
    assert oracle.sha256(b"").hex() == sv["empty"]
    lens = [c["len"] for c in sv["cases"]]
    for data, case in zip(sha_vector_inputs(sv["seed"], lens), sv["cases"]):
        assert oracle.sha256(data).hex() == case["sha256"]
        assert oracle.sha256(data, fast=True).hex() == case["sha256"]
        assert hashlib.sha256(data).hexdigest() == case["sha256"]


def test_sha256_boundaries_vs_hashlib():
    rng = np.random.default_rng(1)
    for n in list(range(0, 200)) + [4095, 4096, 4097]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.sha256(b) == hashlib.sha256(b).digest()


# ---- encode / reconstruct -------------------------------------------------------


def test_encode_vectors(golden):
    for case in golden("encode_vectors.json")["cases"]:
        data = data_for(case["seed"], case["k"], case["shard_size"], case["last_len"])
        parity, digests, rc = oracle.compute_parity(data, case["m"], case["shard_size"])
        assert rc == 0
        assert [hashlib.sha256(p.tobytes()).hexdigest() for p in parity] == case["parity_sha256"]
        assert [d.hex() for d in digests] == case["chunk_sha256"]


def test_reconstruct_vectors(golden):
    for case in golden("reconstruct_vectors.json")["cases"]:
        k, m, s = case["k"], case["m"], case["shard_size"]
        data = data_for(case["seed"], k, s)
        shards = data + oracle.encode(data, m, s)
        assert [hashlib.sha256(x.tobytes()).hexdigest() for x in shards] == case["shard_sha256"]
        for pat in case["erasure_patterns"]:
            inp = [None if i in pat else shards[i] for i in range(k + m)]
            out, present, rc = oracle.reconstruct(inp, k, m, s)
            assert rc == 0 and present.all()
            assert all(np.array_equal(out[i], shards[i]) for i in range(k + m))
            out, present, rc = oracle.reconstruct(inp, k, m, s, data_only=True)
            assert rc == 0
            assert all(np.array_equal(out[i], shards[i]) for i in range(k))
            for i in pat:
                if i >= k:
                    assert present[i] == 0  # reconstruct_data leaves parity alone


def test_reconstruct_too_few():
    data = data_for(7, 4, 32)
    shards = data + oracle.encode(data, 2, 32)
    for pat in itertools.combinations(range(6), 3):
        inp = [None if i in pat else shards[i] for i in range(6)]
        _, _, rc = oracle.reconstruct(inp, 4, 2, 32)
        assert rc == -10  # TooFewShardsPresent


def test_compute_parity_guard_255():
    data = [np.zeros(4, np.uint8)] * 250
    _, _, rc = oracle.compute_parity(data, 6, 4)
    assert rc == -20  # filesystem.rs:1095 "too many shards"


def test_try_reconstruct_semantics():
    k, m, s = 4, 2, 100
    body = bytes([0xEF]) * 350
    data = [body[o:o + s] for o in range(0, 350, s)]
    parity, dig, rc = oracle.compute_parity(data, m, s)
    shards = [bytes(d) for d in data] + [p.tobytes() for p in parity]
    sizes = [100, 100, 100, 50, 100, 100]
    corrupt = list(shards)
    corrupt[1] = bytes(100)                        # integration.rs:3228 zeroed chunk
    out, rc, npres = oracle.try_reconstruct_data_chunk(corrupt, k, m, s, dig, sizes, 1)
    assert rc == 0 and out == shards[1] and npres == 5
    missing = list(shards)
    missing[0] = None                              # :3252 deleted chunk
    out, rc, _ = oracle.try_reconstruct_data_chunk(missing, k, m, s, dig, sizes, 0)
    assert rc == 0 and out == shards[0]
    three = [None, None, None] + shards[3:]        # :3276 three deleted
    out, rc, npres = oracle.try_reconstruct_data_chunk(three, k, m, s, dig, sizes, 0)
    assert rc == -10 and npres == 3
    out, rc, _ = oracle.try_reconstruct_data_chunk(shards, k, m, s, dig, sizes, 3)
    assert rc == 0 and out == shards[3] and len(out) == 50


def test_k1_parity_is_copy():
    """BASELINE config 1 (k=1, m=2): parity rows are [1], parity == data."""
    d = data_for(3, 1, 4096)
    parity = oracle.encode(d, 2)
    assert all(np.array_equal(p, d[0]) for p in parity)


def test_expected_layout_helper_matches_golden_scenarios(golden):
    """tests/helpers.expected_ec_object (the reference layout the driver tests
    compare against) reproduces every committed reference scenario: file
    names, sizes, parity bytes and the to_string_pretty manifest text."""
    from helpers import expected_ec_object, scenario_body

    for name, sc in golden("reference_scenarios.json").items():
        if not isinstance(sc, dict):
            continue  # "source" note
        body = scenario_body(sc["body"])
        files, manifest = expected_ec_object(body, sc["chunk_size"], sc["parity_shards"])
        assert manifest == sc["manifest"], name
        assert sorted(files) == sorted(sc["files"]), name
        for fname, meta in sc["files"].items():
            assert len(files[fname]) == meta["size"], (name, fname)
            if "hex" in meta:
                assert files[fname].hex() == meta["hex"], (name, fname)
