"""dg_encode_pipelined (the pipelined host-to-host path):
bit-exact against the oracle across chunk boundaries, for pinned and pageable
arenas, aligned and unaligned layouts, both algorithms; plan reuse across
calls; the capacity error."""
from __future__ import annotations

import random

import pytest

from cases import DEFAULT_Q

pytestmark = pytest.mark.gpu

ONEPASS, CORRECTING = 1, 2


def _pairs(seed, n):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        L = rng.choice([0, 5, 16, 17, 300, 4096, 20000, 65536])
        R = rng.randbytes(L)
        V = bytearray(R)
        for _ in range(rng.randrange(0, 1 + L // 50)):
            V[rng.randrange(L)] = rng.randrange(256)
        if i % 5 == 0:
            V = bytes(V) + rng.randbytes(rng.randrange(0, 300))
        out.append((R, bytes(V)))
    return out


@pytest.mark.parametrize("pinned", [True, False])
@pytest.mark.parametrize("align", [16, 1])
def test_pipelined_onepass(dg, orc, pinned, align):
    pairs = _pairs(11 + align, 96)
    got = dg.encode_pipelined(pairs, "onepass", p=16, q=97, chunk_bytes=64 << 10, pinned=pinned, align=align)
    for i, ((R, V), d) in enumerate(zip(pairs, got)):
        assert d == orc.encode(ONEPASS, R, V, p=16, q=97), i
    # the same layout again: the slots' plans are reused
    got2 = dg.encode_pipelined(pairs, "onepass", p=16, q=97, chunk_bytes=64 << 10, pinned=pinned, align=align)
    assert got2 == got


def test_pipelined_correcting_and_default_q(dg, orc):
    pairs = _pairs(5, 40)
    got = dg.encode_pipelined(pairs, "correcting", p=16, q=DEFAULT_Q, chunk_bytes=100 << 10)
    for i, ((R, V), d) in enumerate(zip(pairs, got)):
        assert d == orc.encode(CORRECTING, R, V, p=16, q=DEFAULT_Q), i


def test_pipelined_capacity(dg):
    pairs = _pairs(3, 8)
    with pytest.raises(dg.DeltaError) as e:
        dg.encode_pipelined(pairs, "onepass", q=97, out_cap=100)
    assert e.value.code == 7
