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


def test_pipelined_capacity(dg, orc):
    pairs = _pairs(3, 8)
    with pytest.raises(dg.DeltaError) as e:
        dg.encode_pipelined(pairs, "onepass", q=97, out_cap=100)
    assert e.value.code == 7
    # through the C ABI: the chunks that fit are written and marked DG_OK; every
    # pair of the chunk that overflowed and of later chunks gets
    # DG_ERR_CAPACITY and offsets equal to the bytes written so far
    import ctypes as C
    L = dg._lib
    ctx = dg.default_context()
    pairs = [(bytes(range(256)) * 64, bytes(range(255, -1, -1)) * 64) for _ in range(6)]   # 16 KiB each
    want = [orc.encode(ONEPASS, R, V, p=16, q=97) for R, V in pairs]
    n = len(pairs)
    lay = [(i * 16384, 16384, i * 16384, 16384) for i in range(n)]
    hr = (C.c_uint8 * (n * 16384)).from_buffer_copy(b"".join(R for R, _ in pairs))
    hv = (C.c_uint8 * (n * 16384)).from_buffer_copy(b"".join(V for _, V in pairs))
    cap = len(want[0]) + len(want[1]) + 10          # room for the first chunk (2 pairs) only
    ho = (C.c_uint8 * cap)()
    pa = (L.Pair * n)(*[L.Pair(*x) for x in lay])
    offs = (C.c_uint64 * (n + 1))(*([12345] * (n + 1)))
    st = (C.c_int32 * n)(*([0] * n))
    o = L.DiffOptions.make(q=97)
    rc = dg.lib.dg_encode_pipelined(ctx.handle, ONEPASS, C.addressof(hr), C.addressof(hv), pa, n, C.byref(o),
                                   2 * 32768, C.addressof(ho), cap, offs, st)
    assert rc == 7
    written = len(want[0]) + len(want[1])
    assert list(st) == [0, 0] + [7] * (n - 2)
    assert list(offs) == [0, len(want[0]), written] + [written] * (n - 2)
    assert bytes(ho[:written]) == want[0] + want[1]


def test_pipelined_limits_invalidate_cached_plans(dg, orc):
    """Context limits changed between calls with the same layout: each call
    builds its plans under the current limits (the cached plans key on them)
    and the output stays the oracle's in every chain mode (periodic data with
    q = 97 breaks many verified members)."""
    ctx = dg.Context(0)
    pairs = [(bytes(range(256)) * 1024, bytes(range(256)) * 1023 + bytes(256)) for _ in range(3)]
    want = [orc.encode(ONEPASS, R, V, p=16, q=97) for R, V in pairs]
    for mode in (dg.MEMBERS_OFF, dg.MEMBERS_ON, dg.MEMBERS_OFF):
        ctx.set_limit(dg.LIMIT_ONEPASS_MEMBERS, mode)
        assert dg.encode_pipelined(pairs, "onepass", q=97, pinned=True, ctx=ctx) == want
    ctx.close()


@pytest.mark.parametrize("n_dev", [2, 3])
@pytest.mark.parametrize("algo", ["onepass", "correcting"])
def test_pipelined_multi_device(dg, orc, n_dev, algo):
    """dg_encode_pipelined_multi: pair ranges balanced by bytes over several
    contexts (the one-GPU box: contexts on device 0, each with its own
    streams, plans and staging, driven by its own host thread), deltas packed
    in pair order exactly as the one-device call packs them."""
    pairs = _pairs(40 + n_dev, 70)
    ctxs = [dg.Context(0) for _ in range(n_dev)]
    try:
        got = dg.encode_pipelined(pairs, algo, p=16, q=97, chunk_bytes=96 << 10, pinned=True, ctxs=ctxs)
        one = dg.encode_pipelined(pairs, algo, p=16, q=97, chunk_bytes=96 << 10, pinned=True, ctx=ctxs[0])
        assert got == one
        a = ONEPASS if algo == "onepass" else CORRECTING
        for i, ((R, V), d) in enumerate(zip(pairs, got)):
            assert d == orc.encode(a, R, V, p=16, q=97), i
        # a tight h_out: the ranges that fit are packed, the rest report DG_ERR_CAPACITY
        total = sum(len(d) for d in got)
        with pytest.raises(dg.DeltaError) as e:
            dg.encode_pipelined(pairs, algo, p=16, q=97, pinned=True, ctxs=ctxs, out_cap=total // 2)
        assert e.value.code == 7
    finally:
        for c in ctxs:
            c.close()


def test_pipelined_multi_tight_capacity(dg, orc):
    """under a tight out_cap the multi-device call packs the pairs
    up to the first that does not fit; it and every later pair (also in later
    ranges with smaller deltas) report DG_ERR_CAPACITY at the bytes written."""
    import ctypes as C
    L = dg._lib
    n = 9
    # delta sizes differ per pair: pair i's V differs from R in a block of i KiB
    pairs = []
    for i in range(n):
        R = bytes((7 * k + i) & 0xFF for k in range(16384))
        V = bytearray(R)
        for k in range(1024 * (i % 4) + 16):
            V[100 + k] ^= 0x5A
        pairs.append((R, bytes(V)))
    want = [orc.encode(ONEPASS, R, V, p=16, q=97) for R, V in pairs]
    lay = [(i * 16384, 16384, i * 16384, 16384) for i in range(n)]
    hr = (C.c_uint8 * (n * 16384)).from_buffer_copy(b"".join(R for R, _ in pairs))
    hv = (C.c_uint8 * (n * 16384)).from_buffer_copy(b"".join(V for _, V in pairs))
    first = 3   # pairs 0..2 fit, pair 3 (the largest delta) does not; pair 4 alone would
    cap = sum(len(w) for w in want[:first]) + len(want[first]) - 1
    ho = (C.c_uint8 * cap)()
    pa = (L.Pair * n)(*[L.Pair(*x) for x in lay])
    offs = (C.c_uint64 * (n + 1))(*([12345] * (n + 1)))
    st = (C.c_int32 * n)(*([0] * n))
    o = L.DiffOptions.make(q=97)
    ctxs = [dg.Context(0) for _ in range(3)]
    try:
        hs = (C.c_void_p * 3)(*[c.handle for c in ctxs])
        rc = dg.lib.dg_encode_pipelined_multi(hs, 3, ONEPASS, C.addressof(hr), C.addressof(hv), pa, n, C.byref(o),
                                              1 << 20, C.addressof(ho), cap, offs, st)
    finally:
        for c in ctxs:
            c.close()
    assert rc == 7
    written = sum(len(w) for w in want[:first])
    assert list(st) == [0] * first + [7] * (n - first)
    exp = [0]
    for w in want[:first]:
        exp.append(exp[-1] + len(w))
    assert list(offs) == exp + [written] * (n - first)
    assert bytes(ho[:written]) == b"".join(want[:first])


def test_pipelined_multi_range_failure_wins_over_status(dg, orc):
    """a range that fails as a whole (here: plan creation refuses a
    pair of >= 4 GiB, DG_ERR_TOO_LARGE, before any byte is read) makes the
    multi-device call return that code even when a status array is passed, as
    the one-device call does; its pairs carry the code, the other range's
    pairs are written and DG_OK.  The caller's current device is unchanged."""
    import ctypes as C
    import torch
    L = dg._lib
    n = 6
    pairs = [(bytes((5 * k + i) & 0xFF for k in range(4096)),) * 2 for i in range(n)]
    pairs = [(R, R[:100] + bytes(16) + R[116:]) for (R, _) in pairs]
    want = [orc.encode(ONEPASS, R, V, p=16, q=97) for R, V in pairs]
    huge = n - 2   # R of 5 GiB (never read: the plan refuses it first)
    lay = [(i * 4096, 4096, i * 4096, 4096) for i in range(n)]
    lay[huge] = (0, 5 << 30, huge * 4096, 4096)
    hr = (C.c_uint8 * (n * 4096)).from_buffer_copy(b"".join(R for R, _ in pairs))
    hv = (C.c_uint8 * (n * 4096)).from_buffer_copy(b"".join(V for _, V in pairs))
    cap = 1 << 20
    ho = (C.c_uint8 * cap)()
    pa = (L.Pair * n)(*[L.Pair(*x) for x in lay])
    offs = (C.c_uint64 * (n + 1))(*([12345] * (n + 1)))
    st = (C.c_int32 * n)(*([0] * n))
    o = L.DiffOptions.make(q=97)
    ctxs = [dg.Context(0) for _ in range(2)]
    dev0 = torch.cuda.current_device()
    try:
        hs = (C.c_void_p * 2)(*[c.handle for c in ctxs])
        rc = dg.lib.dg_encode_pipelined_multi(hs, 2, ONEPASS, C.addressof(hr), C.addressof(hv), pa, n, C.byref(o),
                                              1 << 20, C.addressof(ho), cap, offs, st)
    finally:
        for c in ctxs:
            c.close()
    assert rc == 3   # DG_ERR_TOO_LARGE
    assert torch.cuda.current_device() == dev0
    assert list(st[:huge]) == [0] * huge
    assert all(s == 3 for s in st[huge:])
    written = sum(len(w) for w in want[:huge])
    assert bytes(ho[:written]) == b"".join(want[:huge])
    assert offs[huge] == written
