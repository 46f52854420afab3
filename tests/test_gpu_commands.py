"""dg_diff — the command-list entry (delta_diff + delta_place_commands) on the
GPU, against the oracle's delta_diff restatement (or_diff_onepass /
or_diff_correcting), command for command.
"""
from __future__ import annotations

import random

import pytest

from cases import random_cases, small_cases

pytestmark = pytest.mark.gpu


def oracle_placed(dg, cmds, V):
    out = []
    for c in cmds:
        if c[0] == "COPY":
            out.append(dg.PlacedCopy(c[2], c[1], c[3]))
        else:
            out.append(dg.PlacedAdd(c[1], V[c[1]:c[1] + c[2]]))
    return out


@pytest.mark.parametrize("case", small_cases(), ids=lambda c: c[0])
def test_diff_onepass_small(dg, ctx, orc, case):
    name, R, V, p, q = case
    got = dg.diff_placed(R, V, "onepass", p=p, q=q, ctx=ctx)
    assert got == oracle_placed(dg, orc.diff_onepass(R, V, p=p, q=q), V)
    cmds = dg.diff_onepass(R, V, p=p, q=q, ctx=ctx)
    assert dg.place_commands(cmds) == got and dg.output_size(cmds) == len(V)


def test_diff_random_both_algorithms(dg, ctx, orc):
    for i, (name, R, V, p, q) in enumerate(random_cases(60, seed=31)):
        got = dg.diff_placed(R, V, "onepass", p=p, q=q, ctx=ctx)
        assert got == oracle_placed(dg, orc.diff_onepass(R, V, p=p, q=q), V), name
        if len(R) >= p and i % 2 == 0:
            bc = 1 + i % 256
            got = dg.diff_placed(R, V, "correcting", p=p, q=q, buf_cap=bc, ctx=ctx)
            exp = orc.diff_correcting(R, V, p=p, q=q, buf_cap=bc)
            assert got == oracle_placed(dg, exp, V), name


def test_diff_then_encode_matches_encode(dg, ctx):
    """diff -> place -> encode_delta with the device CRCs == dg_encode (the
    chain of main.c:257-292 split at the command list, HOWTO.md:426-464)."""
    rng = random.Random(4)
    R = rng.randbytes(200000)
    V = bytearray(R)
    for _ in range(300):
        V[rng.randrange(len(V))] = rng.randrange(256)
    V = bytes(V[5000:] + V[:5000])
    for algo in ("onepass", "correcting"):
        cmds = dg.diff(R, V, algo, ctx=ctx)
        d = dg.encode_delta(dg.place_commands(cmds), version_size=len(V),
                            src_crc=dg.crc64_xz(R, ctx=ctx), dst_crc=dg.crc64_xz(V, ctx=ctx))
        assert d == dg.encode(R, V, algo, ctx=ctx)
        assert dg.decode(R, d, ctx=ctx) == V
    # the in-place flag does not leak into the algorithm's list
    o = dg.DiffOptions.make(flags=1 << dg._lib.OPT_INPLACE)
    import ctypes as C
    cl = dg._lib.Commands()
    ctx.check(dg.lib.dg_diff(ctx.handle, 1, dg._lib._u8(R), len(R), dg._lib._u8(V), len(V), C.byref(o),
                             C.byref(cl)), "dg_diff")
    try:
        assert dg._lib._placed_list(cl) == dg.diff_placed(R, V, "onepass", ctx=ctx)
    finally:
        dg.lib.dg_commands_free(C.byref(cl))
