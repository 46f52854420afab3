"""CPU: the speculative diagonal-member onepass (oracle/spec_model.c, the
model the HIP kernels implement) gives command-for-command the oracle's
onepass (src/c/onepass.c:32-297) on adversarial inputs: substitutions at
every density, low-entropy and periodic data (off-diagonal repeats), block
moves, insertions/deletions (diagonal changes), unequal lengths, tiny and
default table sizes (slot collisions)."""
from __future__ import annotations

import ctypes as C
import random

import pytest

ONEPASS = 1


class Stats(C.Structure):
    _fields_ = [("members", C.c_uint64), ("verified", C.c_uint64), ("exact_epochs", C.c_uint64),
                ("resyncs", C.c_uint64)]


@pytest.fixture(scope="module")
def sm(orc):
    L = orc.L
    L.sm_diff_onepass_spec.restype = C.c_size_t
    u8p = C.POINTER(C.c_uint8)
    L.sm_diff_onepass_spec.argtypes = [u8p, C.c_size_t, u8p, C.c_size_t, C.c_size_t, C.c_size_t,
                                       C.c_void_p, C.POINTER(Stats)]
    return L


def _buf(b):
    return C.cast(C.c_char_p(b), C.POINTER(C.c_uint8)) if b else None


def spec(orc, sm, R, V, q):
    from oracle import _Cmd
    ptr = C.POINTER(_Cmd)()
    st = Stats()
    n = sm.sm_diff_onepass_spec(_buf(R), len(R), _buf(V), len(V), 16, q, C.byref(ptr), C.byref(st))
    return orc._cmds(ptr, n), st


def _cases(seed, n):
    rng = random.Random(seed)
    for i in range(n):
        kind = i % 9
        L = rng.choice([0, 5, 16, 17, 40, 300, 2000, 9000])
        if kind == 0:      # substitutions, any density
            R = rng.randbytes(L)
            V = bytearray(R)
            for _ in range(int(L * rng.choice([0.001, 0.01, 0.05, 0.1, 0.3]))):
                V[rng.randrange(L)] = rng.randrange(256)
            V = bytes(V)
        elif kind == 1:    # low entropy
            a = rng.choice([1, 2, 3, 4])
            R = bytes(rng.randrange(a) for _ in range(L))
            V = bytearray(R)
            for _ in range(L // 20):
                V[rng.randrange(L)] = rng.randrange(a)
            V = bytes(V)
        elif kind == 2:    # periodic with substitutions (off-diagonal equal windows)
            per = rng.choice([3, 8, 16, 17, 31, 64])
            unit = rng.randbytes(per)
            R = (unit * (L // per + 1))[:L]
            V = bytearray(R)
            for _ in range(L // 50 if L else 0):
                V[rng.randrange(L)] = rng.randrange(256)
            V = bytes(V[:L])
        elif kind == 3:    # insertion / deletion (diagonal changes)
            R = rng.randbytes(L)
            a = rng.randrange(L + 1)
            V = R[:a] + rng.randbytes(rng.randrange(1, 40)) + R[a + rng.randrange(0, 30):]
        elif kind == 4:    # block moves
            R = rng.randbytes(L)
            cut = sorted(rng.sample(range(L + 1), 3)) if L >= 3 else [0, 0, L]
            V = R[cut[1]:cut[2]] + R[:cut[1]] + R[cut[2]:]
        elif kind == 5:    # unequal lengths
            R = rng.randbytes(L)
            V = bytearray(R + rng.randbytes(rng.randrange(0, 100)))
            for _ in range(L // 30):
                V[rng.randrange(len(V))] = rng.randrange(256)
            V = bytes(V)
            if rng.random() < 0.5:
                R, V = V, R
        elif kind == 6:    # long members (dense edits), diag repeats within a member
            R = rng.randbytes(L)
            V = bytearray(R)
            for j in range(0, L, rng.choice([5, 9, 13])):
                V[j] ^= 0x5A
            V = bytes(V)
        elif kind == 7:    # zeros with sparse edits
            R = bytes(L)
            V = bytearray(R)
            for _ in range(L // 100 + 1):
                if L:
                    V[rng.randrange(L)] = 1
            V = bytes(V)
        else:              # identical / empty / totally different
            R = rng.randbytes(L)
            V = rng.choice([R, rng.randbytes(L), b"", R[: L // 2]])
        q = rng.choice([1, 7, 97, 1031, 1048573])
        yield i, R, V, q


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_spec_model_equals_onepass(orc, sm, seed):
    tot = Stats()
    for i, R, V, q in _cases(seed, 700):
        got, st = spec(orc, sm, R, V, q)
        assert got == orc.diff_onepass(R, V, p=16, q=q), (seed, i, len(R), len(V), q)
        for f, _ in Stats._fields_:
            setattr(tot, f, getattr(tot, f) + getattr(st, f))
    assert tot.members > 1000 and tot.verified > 0 and tot.resyncs > 0


def test_spec_model_c2_c3_pairs(orc, sm):
    """The benchmark geometries: nearly every member verifies."""
    for seed, L, ne in [(0xC2000000, 65536, 655), (0xC3000000, 262144, 26214)]:
        for i in range(3):
            R, V = orc.synth_pair(seed + i, L, ne)
            got, st = spec(orc, sm, R, V, 1)
            assert got == orc.diff_onepass(R, V, p=16, q=1)
            assert st.verified >= st.members * 0.99, (st.members, st.verified)
