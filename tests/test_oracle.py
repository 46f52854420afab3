"""CPU: the oracle is pinned before it is trusted.

1. Known-answer tests the reference's own suites hold (CRC check values,
   empty delta size, magic, prime sizes of SURVEY.md §8 table).
2. Every golden vector in tests/golden/golden.json (minted from the
   reference's src/c by tests/golden/make_golden.py).
3. Where the reference build exists (oracle/_ref), a randomised differential
   run of oracle vs reference, both algorithms.
"""
from __future__ import annotations

import hashlib
import json
import os

import pytest

from cases import random_cases, small_cases

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))


def _sha(b):
    return hashlib.sha256(b).hexdigest()


def test_crc_kat(orc):
    for msg, h in GOLDEN["crc_kat"].items():
        assert orc.crc64_xz(msg.encode()).hex() == h


def test_mod_mersenne_values(orc):
    # src/cpp/tests/test_hash.cpp:15-20 style values
    M = (1 << 61) - 1
    for x in (0, 1, M - 1, M, M + 1, 2 * M, (1 << 64) - 1, (1 << 100) + 12345, M * M):
        assert orc.mod_mersenne(x) == x % M


def test_rolling_equals_direct(orc):
    # src/cpp/tests/test_hash.cpp:34-47: rolling == direct at every offset
    import random
    data = random.Random(3).randbytes(300)
    M, B, p = (1 << 61) - 1, 263, 16
    for off in range(0, 300 - p):
        h = 0
        for b in data[off:off + p]:
            h = (h * B + b) % M
        assert orc.fingerprint(data, off, p) == h


def test_primes(orc):
    # src/cpp/tests/test_hash.cpp:51-109 (primes, Carmichael numbers)
    for n in (2, 3, 5, 7, 1009, 4099, 16411, 65537, 1048573, 1073741827):
        assert orc.is_prime(n)
    for n in (0, 1, 4, 561, 1105, 1729, 2465, 2821, 6601, 8911, 1048575):
        assert not orc.is_prime(n)
    assert orc.next_prime(1000) == 1009
    # SURVEY.md §8 table (reference's own _next_prime)
    assert orc.onepass_q(65536, 16, 1) == 4099
    assert orc.onepass_q(262144, 16, 1) == 16411
    assert orc.onepass_q(1 << 20, 16, 1) == 65537
    assert orc.onepass_q(65536, 16, 1048573) == 1048573
    # (SURVEY.md §8 lists m=16 here; the reference formula correcting.c:129 gives 17)
    assert orc.correcting_params(65536, 16, 1) == (8191, 131059, 17)
    assert orc.correcting_params(262144, 16, 1) == (32771, 524261, 16)
    assert orc.correcting_params(1 << 20, 16, 1) == (131071, 2097131, 16)


def test_empty_delta_is_26_bytes(orc):
    # src/python/test_delta.py:180-191
    d = orc.encode(1, b"hello", b"")
    assert len(d) == 26 and d[:4] == b"DLT\x03"


@pytest.mark.parametrize("case", GOLDEN["cases"], ids=lambda c: f"{c['name']}-a{c['algo']}")
def test_golden(orc, case):
    kind = case["kind"]
    if kind == "small":
        m = {c[0]: c for c in small_cases()}
        _, R, V, p, q = m[case["name"]]
    elif kind == "synth_edits":
        R, V = orc.synth_pair(case["seed"], case["pair_len"], case["n_edits"])
    elif kind == "synth_transpose":
        R, V = orc.synth_transpose(case["seed"], case["num_blocks"], case["mean"], case["pct"])
    elif kind == "synth_random":
        R, V = orc.synth_random(case["r_seed"], 1 << 20), orc.synth_random(case["v_seed"], 1 << 20)
    elif kind == "synth_shift":
        R, V = orc.synth_shift(case["seed"], case["pair_len"], case["n_edits"], case["indel_pct"])
    else:
        raise AssertionError(kind)
    assert _sha(R) == case["r_sha256"] and _sha(V) == case["v_sha256"], "input generator drifted"
    d = orc.encode(case["algo"], R, V, p=case["p"], q=case["q"])
    assert len(d) == case["delta_len"]
    assert _sha(d) == case["delta_sha256"]
    if "delta_hex" in case:
        assert d.hex() == case["delta_hex"]
    rc, out = orc.decode(R, d)
    assert rc == 0 and out == V


def test_oracle_vs_reference_random(orc, ref):
    for algo in (1, 2):
        for name, R, V, p, q in random_cases(400, seed=algo * 77):
            if algo == 2 and len(V) >= p and len(V) // 2 + p > len(V):
                continue   # reference reads past |V| (correcting.c:133-136)
            assert orc.encode(algo, R, V, p=p, q=q) == ref.encode(algo, R, V, p=p, q=q), name


def test_oracle_vs_reference_small(orc, ref):
    for name, R, V, p, q in small_cases():
        for algo in (1, 2):
            if algo == 2 and len(V) >= p and len(V) // 2 + p > len(V):
                continue
            for bc in (256, 1, 2):
                assert orc.encode(algo, R, V, p=p, q=q, buf_cap=bc) == \
                    ref.encode(algo, R, V, p=p, q=q, buf_cap=bc), (name, algo, bc)


def test_decode_errors(orc):
    R, V = b"A" * 100, b"A" * 50 + b"B" * 10
    d = orc.encode(1, R, V, p=4)
    assert orc.decode(R, d)[1] == V
    assert orc.decode(b"C" * 100, d)[0] == 9
    bad = bytearray(d)
    bad[20] ^= 1
    assert orc.decode(R, bytes(bad))[0] == 10
    assert orc.decode(R, bytes(bad), ignore_hash=True)[1] == V
    assert orc.decode(R, b"NOPE" + d[4:])[0] == 8
    assert orc.decode(R, d[:30])[0] == 8


# ── in-place deltas (main.c encode --inplace), minted from the reference ──

GOLDEN_INPLACE = json.load(open(os.path.join(HERE, "golden", "golden_inplace.json")))["cases"]


def inplace_inputs(orc, case):
    kind = case["kind"]
    if kind == "small":
        m = {c[0]: c for c in small_cases()}
        base = case["name"].rsplit("_pol", 1)[0]
        return m[base][1], m[base][2]
    if kind == "synth_edits":
        return orc.synth_pair(case["seed"], case["pair_len"], case["n_edits"])
    return orc.synth_transpose(case["seed"], case["num_blocks"], case["mean"], case["pct"])


@pytest.mark.parametrize("case", GOLDEN_INPLACE, ids=lambda c: c["name"])
def test_golden_inplace_oracle_decode(orc, case):
    """The oracle's decode (apply.c:253-284 in-place replay) rebuilds V from
    every reference in-place delta, CRCs checked."""
    R, V = inplace_inputs(orc, case)
    assert _sha(R) == case["r_sha256"] and _sha(V) == case["v_sha256"]
    d = bytes.fromhex(case["delta_hex"])
    assert d[4] == 1, "in-place flag"
    rc, out = orc.decode(R, d)
    assert rc == 0 and out == V
