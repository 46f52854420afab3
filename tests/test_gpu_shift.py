"""Onepass where matches leave diagonal 0, on the device.

* Shift pairs (C3s: substitutions, insertions and deletions; or_synth_shift):
  the device generator equals the oracle's, and onepass over a device batch
  is bit-exact against the reference-minted goldens (pairs 0..2 of the C3s
  seed) and the oracle, in both chain modes, every pair decoding back to V.
* C4's transposition pairs under onepass (c4o): the same checks.
Both are the workloads of bench.py's c3s / c3s_chain / c4o / c4o_chain lines.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import json
import os

import pytest

pytestmark = pytest.mark.gpu

ONEPASS = 1
HERE = os.path.dirname(os.path.abspath(__file__))


def _golden(name):
    cases = json.load(open(os.path.join(HERE, "golden", "golden.json")))["cases"]
    return {c["name"]: c for c in cases}[name]


def _shift_batch(dg, ctx, torch, seed, n, L, n_edits, pct):
    pairs = (dg._lib.Pair * n)()
    rb, vb = C.c_uint64(), C.c_uint64()
    ctx.check(dg.lib.dg_synth_shift_pairs_device(ctx.handle, seed, n, L, n_edits, pct, pairs, C.byref(rb),
                                                 C.byref(vb), None, None, None), "layout")
    ref = torch.empty(max(rb.value, 16), dtype=torch.uint8, device="cuda")
    ver = torch.empty(max(vb.value, 16), dtype=torch.uint8, device="cuda")
    ctx.check(dg.lib.dg_synth_shift_pairs_device(ctx.handle, seed, n, L, n_edits, pct, pairs, C.byref(rb),
                                                 C.byref(vb), ref.data_ptr(), ver.data_ptr(), None), "synth")
    torch.cuda.synchronize()
    return ref, ver, [(p.r_off, p.r_len, p.v_off, p.v_len) for p in pairs]


def _transpose_batch(dg, ctx, torch, seed, n, target):
    pairs = (dg._lib.Pair * n)()
    rb, vb = C.c_uint64(), C.c_uint64()
    ctx.check(dg.lib.dg_synth_transpose_pairs_device(ctx.handle, seed, n, target, 50, pairs, C.byref(rb),
                                                     C.byref(vb), None, None, None), "layout")
    ref = torch.empty(rb.value, dtype=torch.uint8, device="cuda")
    ver = torch.empty(vb.value, dtype=torch.uint8, device="cuda")
    ctx.check(dg.lib.dg_synth_transpose_pairs_device(ctx.handle, seed, n, target, 50, pairs, C.byref(rb),
                                                     C.byref(vb), ref.data_ptr(), ver.data_ptr(), None), "synth")
    torch.cuda.synchronize()
    return ref, ver, [(p.r_off, p.r_len, p.v_off, p.v_len) for p in pairs]


def _encode_and_check(dg, ctx, torch, ref, ver, lay, samples, want):
    """Onepass (q floor 1) over the batch; samples bit-exact; all decode back."""
    n = len(lay)
    plan = dg.EncodePlan(ctx, "onepass", lay, q=1)
    out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    try:
        plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), off.data_ptr(), st.data_ptr(),
                 ctx.stream)
        torch.cuda.synchronize()
        members = plan.members
    finally:
        plan.close()
    assert int((st != 0).sum()) == 0, st.unique().tolist()
    offs = off.cpu().tolist()
    for i in samples:
        assert bytes(out[offs[i]:offs[i + 1]].cpu().numpy()) == want(i), i
    descs = (dg._lib.DecodeDesc * n)(*[dg._lib.DecodeDesc(lay[i][0], lay[i][1], offs[i], offs[i + 1] - offs[i],
                                                          lay[i][2], max(lay[i][3], 1)) for i in range(n)])
    dec = torch.zeros(ver.numel(), dtype=torch.uint8, device="cuda")
    dlen = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.check(dg.lib.dg_decode_batch_device(ctx.handle, ref.data_ptr(), out.data_ptr(), descs, n, 0,
                                            dec.data_ptr(), dlen.data_ptr(), dst.data_ptr(), None), "decode")
    torch.cuda.synchronize()
    assert int(dst.abs().sum()) == 0
    assert dlen.cpu().tolist() == [x[3] for x in lay]
    for i in range(n):   # the arena's padding between pairs is not part of V
        e = lay[i][2] + lay[i][3]
        ver[e:(e + 15) // 16 * 16] = 0
    assert bool(torch.equal(dec, ver))
    return members


@pytest.mark.parametrize("pct", [0, 5, 67, 100])
def test_shift_generator_matches_oracle(dg, ctx, orc, torch_cuda, pct):
    torch = torch_cuda
    for L, ne in ((262144, 26214), (65536, 300), (1000, 999), (40, 7), (16, 40)):
        seed = 0xC3500000 + 17 * L + pct
        ref, ver, lay = _shift_batch(dg, ctx, torch, seed, 3, L, ne, pct)
        for i, (ro, rl, vo, vl) in enumerate(lay):
            R, V = orc.synth_shift(seed + i, L, ne, pct)
            assert bytes(ref[ro:ro + rl].cpu().numpy()) == R, (L, i)
            assert vl == len(V) and bytes(ver[vo:vo + vl].cpu().numpy()) == V, (L, i)


def test_c3s_batch(dg, ctx_mode, orc, torch_cuda):
    """512 C3s pairs (the bench's seeds): goldens of pairs 0..2, an oracle
    sample, every pair decoded back, in both chain modes."""
    torch = torch_cuda
    seed, n, L, ne = 0xC3500000, 512, 262144, 26214
    ref, ver, lay = _shift_batch(dg, ctx_mode, torch, seed, n, L, ne, 67)
    gold = {i: _golden(f"c3s_{i}") for i in range(3)}

    def want(i):
        if i in gold:
            return None
        R, V = orc.synth_shift(seed + i, L, ne, 67)
        return orc.encode(ONEPASS, R, V, p=16, q=1)

    plan = dg.EncodePlan(ctx_mode, "onepass", lay, q=1)
    out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    try:
        plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), off.data_ptr(), st.data_ptr(),
                 ctx_mode.stream)
        torch.cuda.synchronize()
    finally:
        plan.close()
    assert int((st != 0).sum()) == 0
    offs = off.cpu().tolist()
    for i, g in gold.items():
        assert hashlib.sha256(bytes(out[offs[i]:offs[i + 1]].cpu().numpy())).hexdigest() == g["delta_sha256"], i
    _encode_and_check(dg, ctx_mode, torch, ref, ver, lay, [5, 100, 311, n - 1], want)


def test_c4o_batch(dg, ctx_mode, orc, torch_cuda):
    """Onepass over 256 of C4's transposition pairs: the goldens of pairs 0..3
    (minted from the reference's onepass), an oracle sample, all decoded back."""
    torch = torch_cuda
    seed, n, target = 0xC4000000, 256, 262144
    ref, ver, lay = _transpose_batch(dg, ctx_mode, torch, seed, n, target)

    def want(i):
        nb = 8 + (i % 57)
        R, V = orc.synth_transpose(seed + i, nb, target // nb, 50)
        return orc.encode(ONEPASS, R, V, p=16, q=1)

    gold = [_golden(f"c4_onepass_{i}") for i in range(4)]
    plan = dg.EncodePlan(ctx_mode, "onepass", lay, q=1)
    out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    try:
        plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), off.data_ptr(), st.data_ptr(),
                 ctx_mode.stream)
        torch.cuda.synchronize()
    finally:
        plan.close()
    offs = off.cpu().tolist()
    for i, g in enumerate(gold):
        assert hashlib.sha256(bytes(out[offs[i]:offs[i + 1]].cpu().numpy())).hexdigest() == g["delta_sha256"], i
    _encode_and_check(dg, ctx_mode, torch, ref, ver, lay, [7, 57, 130, n - 1], want)
