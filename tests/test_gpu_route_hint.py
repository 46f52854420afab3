"""Automatic member mode's per-plan routing hint (dg_host.cpp, dg_encode_plan_run).

The routed plain chain counts the pairs it takes and scan_sizes_kernel hands
the count to a host-mapped word.  The plan's next runs read it:

* every pair routed: the run goes as a plain plan (no member kernel, the
  plain serialiser), except every 16th run, a member-mode probe;
* more pairs routed than 16 per CU: the routed chain waits for the CRC pass.

Neither may change a byte of the output, so each test runs one plan many
times and checks every run against the first, oracle samples and a full
decode.  Both batches route more than 16 x 256 pairs, so the probes and the
mixed batch's runs take the CRC-join path too.
"""
from __future__ import annotations

import ctypes as C

import pytest

pytestmark = pytest.mark.gpu

ONEPASS = 1
L_SHIFT, NE_SHIFT, PCT = 131072, 13107, 67


def _shift(dg, ctx, torch, seed, n):
    pairs = (dg._lib.Pair * n)()
    rb, vb = C.c_uint64(), C.c_uint64()
    args = (ctx.handle, seed, n, L_SHIFT, NE_SHIFT, PCT, pairs, C.byref(rb), C.byref(vb))
    ctx.check(dg.lib.dg_synth_shift_pairs_device(*args, None, None, None), "layout")
    ref = torch.empty((rb.value + 15) // 16 * 16, dtype=torch.uint8, device="cuda")
    ver = torch.empty((vb.value + 15) // 16 * 16, dtype=torch.uint8, device="cuda")
    ctx.check(dg.lib.dg_synth_shift_pairs_device(*args, ref.data_ptr(), ver.data_ptr(), None), "synth")
    return ref, ver, [(p.r_off, p.r_len, p.v_off, p.v_len) for p in pairs]


def _runs(dg, ctx, torch, ref, ver, lay, n_runs):
    """n_runs runs of one plan; returns the plan's member flag, the first
    run's output and offsets, and asserts every later run equals it."""
    n = len(lay)
    plan = dg.EncodePlan(ctx, "onepass", lay, q=1)
    out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    first = None
    try:
        for r in range(n_runs):
            out.fill_(0xEE)
            st.fill_(-1)
            torch.cuda.synchronize()
            plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), off.data_ptr(), st.data_ptr(),
                     ctx.stream)
            torch.cuda.synchronize()
            assert int((st != 0).sum()) == 0, (r, st.unique().tolist())
            total = int(off[n])
            if first is None:
                first = (out[:total].clone(), off.clone())
            else:
                assert torch.equal(off, first[1]), r
                assert torch.equal(out[:total], first[0]), r
        members = plan.members
        modes = plan.run_modes
    finally:
        plan.close()
    return members, modes, first[0], first[1].cpu().tolist()


def _decode_all(dg, ctx, torch, ref, ver, lay, delta, offs):
    n = len(lay)
    descs = (dg._lib.DecodeDesc * n)(*[dg._lib.DecodeDesc(lay[i][0], lay[i][1], offs[i], offs[i + 1] - offs[i],
                                                          lay[i][2], max(lay[i][3], 1)) for i in range(n)])
    dec = torch.zeros(ver.numel(), dtype=torch.uint8, device="cuda")
    dlen = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.check(dg.lib.dg_decode_batch_device(ctx.handle, ref.data_ptr(), delta.data_ptr(), descs, n, 0,
                                            dec.data_ptr(), dlen.data_ptr(), dst.data_ptr(), None), "decode")
    torch.cuda.synchronize()
    assert int(dst.abs().sum()) == 0
    assert dlen.cpu().tolist() == [x[3] for x in lay]
    for ro, rl, vo, vl in lay:
        assert torch.equal(dec[vo:vo + vl], ver[vo:vo + vl]), vo


def test_all_routed_batch_runs_plain_between_probes(dg, orc, torch_cuda):
    """4160 shift pairs of 128 KiB, automatic mode: run 1 in member mode (no
    hint yet), runs 2-16 as a plain plan, run 17 a member probe with the
    routed chain after the CRC pass, then plain again: 20 identical outputs."""
    torch = torch_cuda
    ctx = dg.Context(0)
    ctx.set_limit(dg.LIMIT_ONEPASS_MEMBERS, dg.MEMBERS_AUTO)
    seed, n = 0xC3510000, 4160
    ref, ver, lay = _shift(dg, ctx, torch, seed, n)
    members, modes, delta, offs = _runs(dg, ctx, torch, ref, ver, lay, 20)
    assert members
    assert modes == (2, 18)   # runs 1 and 17 in member mode
    for i in (0, 1, 2047, n - 1):
        R, V = orc.synth_shift(seed + i, L_SHIFT, NE_SHIFT, PCT)
        assert bytes(delta[offs[i]:offs[i + 1]].cpu().numpy()) == orc.encode(ONEPASS, R, V, p=16, q=1), i
    _decode_all(dg, ctx, torch, ref, ver, lay, delta, offs)


def test_mixed_batch_routed_chain_after_crc(dg, orc, torch_cuda):
    """4160 shift pairs then 192 substitution pairs (1 % edits, verified
    members): some pairs stay on the member chain, so every run is a member
    run, and from run 2 on the routed chain waits for the CRC pass."""
    torch = torch_cuda
    ctx = dg.Context(0)
    ctx.set_limit(dg.LIMIT_ONEPASS_MEMBERS, dg.MEMBERS_AUTO)
    seed, n1, n2, L2 = 0xC3520000, 4160, 192, 131072
    sref, sver, slay = _shift(dg, ctx, torch, seed, n1)
    eref = torch.empty(n2 * L2, dtype=torch.uint8, device="cuda")
    ever = torch.empty(n2 * L2, dtype=torch.uint8, device="cuda")
    ne2 = int(0.01 * L2 + 0.5)
    ctx.check(dg.lib.dg_synth_edit_pairs_device(ctx.handle, eref.data_ptr(), ever.data_ptr(), n2, L2, seed + n1,
                                                ne2, None), "synth")
    ref = torch.cat([sref, eref])
    ver = torch.cat([sver, ever])
    r0, v0 = sref.numel(), sver.numel()
    lay = slay + [(r0 + i * L2, L2, v0 + i * L2, L2) for i in range(n2)]
    n = n1 + n2
    members, modes, delta, offs = _runs(dg, ctx, torch, ref, ver, lay, 6)
    assert members
    assert modes == (6, 0)
    for i in (0, n1 - 1):
        R, V = orc.synth_shift(seed + i, L_SHIFT, NE_SHIFT, PCT)
        assert bytes(delta[offs[i]:offs[i + 1]].cpu().numpy()) == orc.encode(ONEPASS, R, V, p=16, q=1), i
    for j in (0, n2 - 1):
        R, V = orc.synth_pair(seed + n1 + j, L2, ne2)
        i = n1 + j
        assert bytes(delta[offs[i]:offs[i + 1]].cpu().numpy()) == orc.encode(ONEPASS, R, V, p=16, q=1), i
    _decode_all(dg, ctx, torch, ref, ver, lay, delta, offs)
