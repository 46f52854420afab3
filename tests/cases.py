"""Deterministic parity cases, modelled on the reference's own tests.

Each case is (name, R, V, p, q).  The sources are cited per case; sizes are
small enough that the CPU oracle finishes in well under a second.
"""
from __future__ import annotations

import random

DEFAULT_Q = 1048573


def _rnd(rng, n):
    return bytes(rng.getrandbits(8) for _ in range(n))


def small_cases():
    cases = []
    # paper example, src/python/test_delta.py:63-76
    R, V = b"ABCDEFGHIJKLMNOP", b"QWIJKLMNOBCDEFGHZDEFGHIJKL"
    for q in (1, 7, DEFAULT_Q):
        cases.append(("paper_p2_q%d" % q, R, V, 2, q))
    # identical, test_delta.py:79-90
    data = b"The quick brown fox jumps over the lazy dog." * 10
    cases.append(("identical_p2", data, data, 2, DEFAULT_Q))
    cases.append(("identical_p16", data, data, 16, DEFAULT_Q))
    # completely different, test_delta.py:93-103
    cases.append(("different_p2", bytes(range(256)) * 2, bytes(range(255, -1, -1)) * 2, 2, DEFAULT_Q))
    # empty version / reference, test_delta.py:106-128 and test_delta.sh:115-128
    cases.append(("empty_version", b"hello", b"", 2, DEFAULT_Q))
    cases.append(("empty_reference", b"", b"hello world", 2, DEFAULT_Q))
    cases.append(("both_empty", b"", b"", 16, DEFAULT_Q))
    # |V| < p and |R| < p
    cases.append(("short_version", b"ABCDEFGHIJKLMNOPQRSTUVWXYZ", b"ABCDEFG", 16, DEFAULT_Q))
    cases.append(("short_reference", b"ABCDEFG", b"ABCDEFGHIJKLMNOPQRSTUVWXYZ", 16, DEFAULT_Q))
    cases.append(("exactly_p", b"0123456789abcdef", b"0123456789abcdef", 16, DEFAULT_Q))
    # binary round trip, test_delta.py:131-141
    R = b"ABCDEFGHIJKLMNOPQRSTUVWXYZ" * 100
    V = b"0123EFGHIJKLMNOPQRS456ABCDEFGHIJKL789" * 100
    for q in (1, 101, DEFAULT_Q):
        cases.append(("binary_rt_p4_q%d" % q, R, V, 4, q))
    # block transposition, test_delta.py:239-251
    X, Y = b"FIRST_BLOCK_DATA_" * 10, b"SECOND_BLOCK_DATA" * 10
    cases.append(("transposition_p4", X + Y, Y + X, 4, DEFAULT_Q))
    # scattered modifications, test_delta.py:254-270
    rng = random.Random(42)
    R = _rnd(rng, 2000)
    Vb = bytearray(R)
    for _ in range(100):
        Vb[rng.randint(0, len(Vb) - 1)] = rng.getrandbits(8)
    for p, q in ((4, DEFAULT_Q), (16, DEFAULT_Q), (16, 1), (4, 7)):
        cases.append(("scattered_p%d_q%d" % (p, q), R, bytes(Vb), p, q))
    # checkpointing-style inputs, test_delta.py:916-952
    R = b"ABCDEFGHIJKLMNOP" * 20
    cases.append(("insert_p16_q7", R, R[:160] + b"XXXXYYYY" + R[160:], 16, 7))
    R = bytes(range(256)) * 40
    cases.append(("insertion_10k_p16_q31", R, R[:5000] + b"X" * 100 + R[5000:], 16, 31))
    # small alphabet (many fingerprint/slot collisions), rotations
    rng = random.Random(7)
    for i, (n, q, p) in enumerate(((700, 1, 4), (1500, 2, 16), (3000, 13, 16), (4000, 1, 2))):
        R = bytes(65 + rng.getrandbits(2) for _ in range(n))
        V = bytes(65 + rng.getrandbits(2) for _ in range(n + 37))
        cases.append(("alphabet4_%d" % i, R, V, p, q))
    R = _rnd(rng, 3001)
    cases.append(("rotation", R, R[1234:] + R[:1234], 16, 1))
    cases.append(("rotation_default_q", R, R[1234:] + R[:1234], 16, DEFAULT_Q))
    # long unmatched stretch: exercises the table tier (epochs > 512 steps)
    R = _rnd(rng, 6000)
    V = _rnd(rng, 3000) + R[100:2100] + _rnd(rng, 900) + R[:700]
    for q in (1, 257, DEFAULT_Q):
        cases.append(("long_epoch_q%d" % q, R, V, 16, q))
    # long epoch where |V| runs out first and R keeps scanning (can_v false)
    R = _rnd(rng, 5000)
    V = _rnd(rng, 1500) + R[4000:4100]
    cases.append(("r_outlasts_v", R, V, 16, 1))
    # repeated bytes (first-writer-wins within a version)
    cases.append(("runs", b"\x00" * 3000 + b"\x01" * 50, b"\x00" * 1500 + b"\x02" + b"\x00" * 2000, 16, 1))
    # general p
    R = _rnd(rng, 2500)
    Vb = bytearray(R)
    for _ in range(60):
        Vb[rng.randrange(len(Vb))] = rng.getrandbits(8)
    for p in (1, 3, 31, 64):
        cases.append(("scattered_p%d" % p, R, bytes(Vb), p, 1))
    return cases


def random_cases(n, seed=1234, max_len=5000):
    """Randomised mix in the style of tests used to pin the oracle."""
    rng = random.Random(seed)
    out = []
    for i in range(n):
        kind = rng.randrange(5)
        L = rng.choice([0, 1, 15, 16, 17, 100, 700, 2000, max_len])
        R = _rnd(rng, L)
        if kind == 0:
            V = _rnd(rng, rng.choice([0, 5, 300, 2000]))
        elif kind == 1:
            Vb = bytearray(R)
            for _ in range(rng.randrange(0, 1 + L // 20)):
                if Vb:
                    Vb[rng.randrange(len(Vb))] = rng.getrandbits(8)
            V = bytes(Vb)
        elif kind == 2:
            k = rng.randrange(0, L + 1)
            V = R[k:] + R[:k]
        elif kind == 3:
            V = R[L // 3:] + _rnd(rng, rng.randrange(50)) + R[:L // 3]
        else:
            V = R
        p = rng.choice([2, 4, 16, 16, 16])
        q = rng.choice([1, 7, 101, 4099, DEFAULT_Q])
        out.append(("rand%d" % i, R, V, p, q))
    return out
