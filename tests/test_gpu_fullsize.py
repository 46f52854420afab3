"""GPU parity at BASELINE's full sizes.

* C3 per GPU: the whole 8192 x 256 KiB, 10%-edit device batch the bench
  times — every status checked, sampled pairs bit-exact against the oracle,
  the reference-minted golden deltas of pairs 0..3, and every pair decoded
  back to V on the device (src/dst CRCs verified there).
* C5: 1024 in-place deltas (device onepass encode of C2 pairs, converted by
  dg_make_inplace(localmin)) — sampled deltas byte-identical to the
  reference's own `encode --inplace` chain, all of them decoded on the device
  in one plan and checked against V.
* C4: the whole 4096-pair transposition batch the bench times, encoded by
  the correcting plan, sampled pairs bit-exact against the oracle and every
  pair decoded back to V on the device.
* C5o: 1024 in-place deltas of C4 transposition pairs (moving COPYs, so the
  replay order matters): sampled deltas equal to the reference's own
  `encode correcting --inplace` chain, all decoded on the device in one plan.
* Work-table pool contention: more long-epoch pairs than pool tables (a
  4-table pool at the default --table-size), every pair checked against the
  oracle.
"""
from __future__ import annotations

import hashlib
import json
import os
import random

import pytest

from cases import DEFAULT_Q

pytestmark = pytest.mark.gpu

ONEPASS = 1
HERE = os.path.dirname(os.path.abspath(__file__))


def _golden(name):
    cases = json.load(open(os.path.join(HERE, "golden", "golden.json")))["cases"]
    return {c["name"]: c for c in cases}[name]


def _synth(dg, ctx, torch, n, L, n_edits, seed):
    ref = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    ver = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    ctx.check(dg.lib.dg_synth_edit_pairs_device(ctx.handle, ref.data_ptr(), ver.data_ptr(), n, L, seed,
                                                n_edits, None), "synth")
    return ref, ver


def _encode(dg, ctx, torch, ref, ver, layout, q, algo="onepass"):
    plan = dg.EncodePlan(ctx, algo, layout, q=q)
    out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
    off = torch.empty(len(layout) + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(len(layout), dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), off.data_ptr(),
             st.data_ptr(), ctx.stream)
    torch.cuda.synchronize()
    plan.close()
    return out, off, st


def test_c3_full_batch(dg, ctx_mode, orc, torch_cuda):
    torch = torch_cuda
    ctx = ctx_mode
    n, L, seed, ne = 8192, 262144, 0xC3000000, 26214
    ref, ver = _synth(dg, ctx, torch, n, L, ne, seed)
    layout = [(i * L, L, i * L, L) for i in range(n)]
    out, off, st = _encode(dg, ctx, torch, ref, ver, layout, q=1)
    assert int((st != 0).sum()) == 0, st.unique().tolist()
    offs = off.cpu().tolist()
    assert offs[0] == 0 and all(offs[i] < offs[i + 1] for i in range(n))

    def delta(i):
        return bytes(out[offs[i]:offs[i + 1]].cpu().numpy())

    # the reference's own bytes for pairs 0..3 (tests/golden, minted from src/c)
    for i in range(4):
        g = _golden(f"c3_{i}")
        assert g["seed"] == seed + i and g["n_edits"] == ne
        assert hashlib.sha256(delta(i)).hexdigest() == g["delta_sha256"], i
    # a spread sample against the oracle (inputs regenerated on the host)
    for i in [5, 1023, 2048, 4095, 4096, 6000, 7777, n - 1]:
        R, V = orc.synth_pair(seed + i, L, ne)
        assert bytes(ref[i * L:(i + 1) * L].cpu().numpy()) == R
        assert delta(i) == orc.encode(ONEPASS, R, V, p=16, q=1), i
    # every pair decodes back to V on the device, CRCs verified there
    descs = (dg._lib.DecodeDesc * n)(*[
        dg._lib.DecodeDesc(i * L, L, offs[i], offs[i + 1] - offs[i], i * L, L) for i in range(n)])
    del st
    dec = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    dlen = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.check(dg.lib.dg_decode_batch_device(ctx.handle, ref.data_ptr(), out.data_ptr(), descs, n, 0,
                                            dec.data_ptr(), dlen.data_ptr(), dst.data_ptr(), None),
              "decode batch")
    torch.cuda.synchronize()
    assert int(dst.abs().sum()) == 0
    assert bool((dlen == L).all())
    assert bool(torch.equal(dec, ver))
    del ref, ver, out, dec
    torch.cuda.empty_cache()


def _decode_all_back(dg, ctx, torch, ref, ver, out, offs, n, L):
    """Every pair's delta decoded back to V in one device batch (CRCs checked there)."""
    descs = (dg._lib.DecodeDesc * n)(*[
        dg._lib.DecodeDesc(i * L, L, offs[i], offs[i + 1] - offs[i], i * L, L) for i in range(n)])
    dec = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    dlen = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.check(dg.lib.dg_decode_batch_device(ctx.handle, ref.data_ptr(), out.data_ptr(), descs, n, 0,
                                            dec.data_ptr(), dlen.data_ptr(), dst.data_ptr(), None),
              "decode batch")
    torch.cuda.synchronize()
    assert int(dst.abs().sum()) == 0
    assert bool((dlen == L).all())
    assert bool(torch.equal(dec, ver))


def test_c6_full_batch(dg, ctx_mode, orc, torch_cuda):
    """The north star's upper pair size: the whole
    1024 x 1 MiB, 1%-edit batch the bench's c6 line times, at --table-size 1
    (q = next_prime(65536) = 65537, onepass.c:61-62), in both chain modes:
    pairs 0..3 equal the reference-minted goldens, a spread sample equals
    the oracle, every pair decodes back to V on the device."""
    torch = torch_cuda
    ctx = ctx_mode
    n, L, seed, ne = 1024, 1 << 20, 0xC6000000, 10486
    ref, ver = _synth(dg, ctx, torch, n, L, ne, seed)
    layout = [(i * L, L, i * L, L) for i in range(n)]
    plan = dg.EncodePlan(ctx, "onepass", layout, q=1)
    assert plan.table_size(0) == 65537
    plan.close()
    out, off, st = _encode(dg, ctx, torch, ref, ver, layout, q=1)
    assert int((st != 0).sum()) == 0, st.unique().tolist()
    offs = off.cpu().tolist()
    assert offs[0] == 0 and all(offs[i] < offs[i + 1] for i in range(n))

    def delta(i):
        return bytes(out[offs[i]:offs[i + 1]].cpu().numpy())

    for i in range(4):
        g = _golden(f"c6_{i}")
        assert g["seed"] == seed + i and g["n_edits"] == ne and g["q"] == 1
        assert hashlib.sha256(delta(i)).hexdigest() == g["delta_sha256"], i
    for i in [5, 511, 512, 777, n - 1]:
        R, V = orc.synth_pair(seed + i, L, ne)
        assert delta(i) == orc.encode(ONEPASS, R, V, p=16, q=1), i
    _decode_all_back(dg, ctx, torch, ref, ver, out, offs, n, L)
    del ref, ver, out
    torch.cuda.empty_cache()


def test_c2_default_q_full_batch(dg, ctx, orc, torch_cuda):
    """C2 at the CLI's default --table-size (q = 1048573, delta.h:21): the
    whole 4096-pair batch of the bench's c2_defq line, the reference-minted
    goldens of pairs 0..1, an oracle sample, every pair decoded back."""
    torch = torch_cuda
    n, L, seed, ne = 4096, 65536, 0xC2000000, 655
    ref, ver = _synth(dg, ctx, torch, n, L, ne, seed)
    layout = [(i * L, L, i * L, L) for i in range(n)]
    out, off, st = _encode(dg, ctx, torch, ref, ver, layout, q=DEFAULT_Q)
    assert int((st != 0).sum()) == 0, st.unique().tolist()
    offs = off.cpu().tolist()

    def delta(i):
        return bytes(out[offs[i]:offs[i + 1]].cpu().numpy())

    for i in range(2):
        g = _golden(f"c2_default_q_{i}")
        assert g["q"] == DEFAULT_Q
        assert hashlib.sha256(delta(i)).hexdigest() == g["delta_sha256"], i
    for i in [7, 1000, 2049, n - 1]:
        R, V = orc.synth_pair(seed + i, L, ne)
        assert delta(i) == orc.encode(ONEPASS, R, V, p=16, q=DEFAULT_Q), i
    _decode_all_back(dg, ctx, torch, ref, ver, out, offs, n, L)
    del ref, ver, out
    torch.cuda.empty_cache()


def test_c5_inplace_full_batch(dg, ctx, orc, torch_cuda):
    import oracle as O
    torch = torch_cuda
    n, L, seed, ne = 1024, 65536, 0xC2000000, 655
    ref, ver = _synth(dg, ctx, torch, n, L, ne, seed)
    layout = [(i * L, L, i * L, L) for i in range(n)]
    out, off, st = _encode(dg, ctx, torch, ref, ver, layout, q=1)
    assert int(st.abs().sum()) == 0
    offs = off.cpu().tolist()
    std = out[:offs[-1]].cpu().numpy().tobytes()
    ref_h = ref.cpu().numpy().tobytes()
    deltas, commands = [], 0
    for i in range(n):
        d = dg.make_inplace(ref_h[i * L:(i + 1) * L], std[offs[i]:offs[i + 1]], policy="localmin")
        assert d[4] == 1
        deltas.append(d)
        commands += dg.info(d)["num_commands"]
    assert commands > 1_000_000              # ~1.1 M commands
    if O.reference_available():              # the reference's own encode --inplace chain
        refc = O.Reference()
        for i in range(0, n, 97):
            R, V = orc.synth_pair(seed + i, L, ne)
            assert deltas[i] == refc.encode_inplace(ONEPASS, R, V, p=16, q=1, policy=0), i
    d_offs = [0]
    for d in deltas:
        d_offs.append(d_offs[-1] + len(d))
    d_dev = torch.frombuffer(bytearray(b"".join(deltas)), dtype=torch.uint8).to("cuda")
    descs = [(i * L, L, d_offs[i], len(deltas[i]), i * L, L) for i in range(n)]
    plan = dg.DecodePlan(ctx, descs)
    dec = torch.zeros(n * L, dtype=torch.uint8, device="cuda")
    dlen = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int32, device="cuda")
    for _ in range(2):   # the plan is reusable
        dec.zero_()
        torch.cuda.synchronize()
        plan.run(ref.data_ptr(), d_dev.data_ptr(), dec.data_ptr(), dlen.data_ptr(), dst.data_ptr(),
                 ctx.stream)
        torch.cuda.synchronize()
        assert int(dst.abs().sum()) == 0
        assert bool((dlen == L).all())
        assert bool(torch.equal(dec, ver))
    plan.close()


def test_c4_full_batch(dg, ctx, orc, torch_cuda):
    import ctypes as C
    torch = torch_cuda
    n, target, seed = 4096, 262144, 0xC4000000
    pairs = (dg._lib.Pair * n)()
    rb, vb = C.c_uint64(), C.c_uint64()
    ctx.check(dg.lib.dg_synth_transpose_pairs_device(ctx.handle, seed, n, target, 50, pairs,
                                                     C.byref(rb), C.byref(vb), None, None, None), "layout")
    ref = torch.empty(rb.value, dtype=torch.uint8, device="cuda")
    ver = torch.empty(vb.value, dtype=torch.uint8, device="cuda")
    ctx.check(dg.lib.dg_synth_transpose_pairs_device(ctx.handle, seed, n, target, 50, pairs,
                                                     C.byref(rb), C.byref(vb), ref.data_ptr(),
                                                     ver.data_ptr(), None), "synth")
    lay = [(p.r_off, p.r_len, p.v_off, p.v_len) for p in pairs]
    out, off, st = _encode(dg, ctx, torch, ref, ver, lay, q=1, algo="correcting")
    assert int((st != 0).sum()) == 0, st.unique().tolist()
    offs = off.cpu().tolist()
    assert offs[0] == 0 and all(offs[i] < offs[i + 1] for i in range(n))
    for i in [0, 1, 56, 57, 1000, 2047, 3001, n - 1]:
        nb = 8 + (i % 57)
        R, V = orc.synth_transpose(seed + i, nb, target // nb, 50)
        got = bytes(out[offs[i]:offs[i + 1]].cpu().numpy())
        assert got == orc.encode(2, R, V, p=16, q=1), i
    descs = (dg._lib.DecodeDesc * n)(*[
        dg._lib.DecodeDesc(lay[i][0], lay[i][1], offs[i], offs[i + 1] - offs[i], lay[i][2],
                           max(lay[i][1], lay[i][3])) for i in range(n)])
    dec = torch.zeros(int(vb.value), dtype=torch.uint8, device="cuda")
    dlen = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.check(dg.lib.dg_decode_batch_device(ctx.handle, ref.data_ptr(), out.data_ptr(), descs, n, 0,
                                            dec.data_ptr(), dlen.data_ptr(), dst.data_ptr(), None),
              "decode batch")
    torch.cuda.synchronize()
    assert int(dst.abs().sum()) == 0
    assert dlen.cpu().tolist() == [x[3] for x in lay]
    for i in range(n):   # the arena's 16-byte padding between pairs is not part of V
        e = lay[i][2] + lay[i][3]
        ver[e:(e + 15) // 16 * 16] = 0
    assert bool(torch.equal(dec, ver))
    del ref, ver, out, dec
    torch.cuda.empty_cache()


def test_c5o_ordered_full_batch(dg, ctx, orc, torch_cuda):
    import ctypes as C
    import oracle as O
    torch = torch_cuda
    n, target, seed = 1024, 262144, 0xC4000000
    pairs = (dg._lib.Pair * n)()
    rb, vb = C.c_uint64(), C.c_uint64()
    ctx.check(dg.lib.dg_synth_transpose_pairs_device(ctx.handle, seed, n, target, 50, pairs,
                                                     C.byref(rb), C.byref(vb), None, None, None), "layout")
    ref = torch.empty(rb.value, dtype=torch.uint8, device="cuda")
    ver = torch.empty(vb.value, dtype=torch.uint8, device="cuda")
    ctx.check(dg.lib.dg_synth_transpose_pairs_device(ctx.handle, seed, n, target, 50, pairs,
                                                     C.byref(rb), C.byref(vb), ref.data_ptr(),
                                                     ver.data_ptr(), None), "synth")
    lay = [(p.r_off, p.r_len, p.v_off, p.v_len) for p in pairs]
    out, off, st = _encode(dg, ctx, torch, ref, ver, lay, q=1, algo="correcting")
    assert int(st.abs().sum()) == 0
    offs = off.cpu().tolist()
    std = out[:offs[-1]].cpu().numpy().tobytes()
    ref_h = ref.cpu().numpy().tobytes()
    deltas, moving = [], 0
    for i, (ro, rl, vo, vl) in enumerate(lay):
        d = dg.make_inplace(ref_h[ro:ro + rl], std[offs[i]:offs[i + 1]], policy="localmin")
        deltas.append(d)
        moving += sum(1 for c in dg.decode_delta(d)[0] if isinstance(c, dg.PlacedCopy) and c.src != c.dst)
    assert moving > 10 * n      # most COPYs move
    if O.reference_available():              # the reference's own encode --inplace chain
        refc = O.Reference()
        for i in range(0, n, 131):
            nb = 8 + (i % 57)
            R, V = orc.synth_transpose(seed + i, nb, target // nb, 50)
            assert deltas[i] == refc.encode_inplace(2, R, V, p=16, q=1, policy=0), i
    d_offs = [0]
    for d in deltas:
        d_offs.append(d_offs[-1] + len(d))
    d_dev = torch.frombuffer(bytearray(b"".join(deltas)), dtype=torch.uint8).to("cuda")
    descs = [(ro, rl, d_offs[i], len(deltas[i]), vo, max(rl, vl)) for i, (ro, rl, vo, vl) in enumerate(lay)]
    plan = dg.DecodePlan(ctx, descs)
    dec = torch.zeros(int(vb.value), dtype=torch.uint8, device="cuda")
    dlen = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int32, device="cuda")
    for i in range(n):   # the arena's padding between pairs is not part of V
        e = lay[i][2] + lay[i][3]
        ver[e:(e + 15) // 16 * 16] = 0
    try:
        for _ in range(2):   # the plan is reusable
            dec.zero_()
            torch.cuda.synchronize()
            plan.run(ref.data_ptr(), d_dev.data_ptr(), dec.data_ptr(), dlen.data_ptr(), dst.data_ptr(),
                     ctx.stream)
            torch.cuda.synchronize()
            assert int(dst.abs().sum()) == 0, dst.unique().tolist()
            assert dlen.cpu().tolist() == [x[3] for x in lay]
            assert bool(torch.equal(dec, ver))
    finally:
        plan.close()


@pytest.mark.parametrize("mode", ["members", "chain"])
def test_table_pool_contention(dg, orc, torch_cuda, mode):
    """256 pairs whose epochs run far past the register history (phase C)
    share a pool of 4 work tables at the default --table-size: waves wait for
    tables, every pair completes with status 0 and the oracle's bytes."""
    torch = torch_cuda
    ctx = dg.Context(0)
    ctx.set_limit(dg.LIMIT_TABLE_POOL_BYTES, 4 * 16 * DEFAULT_Q)
    ctx.set_limit(dg.LIMIT_ONEPASS_MEMBERS, dg.MEMBERS_ON if mode == "members" else dg.MEMBERS_OFF)
    with pytest.raises(dg.DeltaError):
        ctx.set_limit(99, 1)
    rng = random.Random(77)
    pairs = []
    for i in range(256):
        R = rng.randbytes(65536)
        if i % 2:
            V = rng.randbytes(65536)                          # one epoch over the whole pair
        else:
            a = rng.randrange(1000, 60000)
            V = R[:a] + rng.randbytes(rng.choice([600, 3000, 9000])) + R[a:]   # long epoch, then a match
        pairs.append((R, V))
    got = dg.encode_batch(pairs, "onepass", p=16, q=DEFAULT_Q, ctx=ctx)
    for i, ((R, V), d) in enumerate(zip(pairs, got)):
        assert d == orc.encode(ONEPASS, R, V, p=16, q=DEFAULT_Q), i
    ctx.close()


def test_table_tag_wrap(dg, orc, torch_cuda):
    """The table tier's 16-bit epoch tags run out and the tables are cleared:
    one plan reused 60 times over 64 pairs of ~156 epochs of ~380 steps each
    (every epoch in the table tier) with an 8-table pool (one table per XCD
    partition) passes 65535 tags per table; every run's deltas equal the
    oracle's."""
    torch = torch_cuda
    rng = random.Random(4242)
    pairs = []
    for _ in range(64):
        R = rng.randbytes(65536)
        V, c = bytearray(), 0
        while c + 340 <= len(R):
            V += rng.randbytes(380) + R[c + 300:c + 340]   # matched at step ~380 of its epoch
            c += 340
        pairs.append((R, bytes(V)))
    ctx = dg.Context(0)
    ctx.set_limit(dg.LIMIT_TABLE_POOL_BYTES, 8 * 16 * DEFAULT_Q)
    ctx.set_limit(dg.LIMIT_ONEPASS_MEMBERS, dg.MEMBERS_OFF)
    want = [orc.encode(ONEPASS, R, V, p=16, q=DEFAULT_Q) for R, V in pairs]
    rb = b"".join(R for R, _ in pairs)
    vb = b"".join(V for _, V in pairs)
    layout, ro, vo = [], 0, 0
    for R, V in pairs:
        layout.append((ro, len(R), vo, len(V)))
        ro += len(R)
        vo += len(V)
    ref = torch.frombuffer(bytearray(rb), dtype=torch.uint8).cuda()
    ver = torch.frombuffer(bytearray(vb), dtype=torch.uint8).cuda()
    plan = dg.EncodePlan(ctx, "onepass", layout, q=DEFAULT_Q)
    try:
        out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
        off = torch.empty(len(layout) + 1, dtype=torch.int64, device="cuda")
        st = torch.empty(len(layout), dtype=torch.int32, device="cuda")
        for run in range(60):
            plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), off.data_ptr(),
                     st.data_ptr(), ctx.stream)
            torch.cuda.synchronize()
            assert int(st.abs().sum()) == 0, (run, st.unique().tolist())
            if run % 10 == 9 or run < 2:
                o = off.cpu().tolist()
                blob = out[:o[-1]].cpu().numpy().tobytes()
                for i, w in enumerate(want):
                    assert blob[o[i]:o[i + 1]] == w, (run, i)
    finally:
        plan.close()
        ctx.close()


def test_decode_many_streams_queued_blocks(dg, ctx, orc, torch_cuda):
    """C5's "many streams" reading (VERDICT r5 missing #4): 65,536 delta
    streams in one decode batch, 64 times C5's count, so decode_kernel's
    blocks queue behind each other instead of all being resident at once
    (apply.c:271-284, main.c:341-385).  Standard deltas of 4 KiB 1%-edit
    pairs all decode back to V with both CRCs checked on the device; 8192
    of them converted in place (localmin) decode back too."""
    torch = torch_cuda
    n, L, seed, ne = 65536, 4096, 0x5A000000, 41
    ref, ver = _synth(dg, ctx, torch, n, L, ne, seed)
    layout = [(i * L, L, i * L, L) for i in range(n)]
    out, off, st = _encode(dg, ctx, torch, ref, ver, layout, q=1)
    assert int((st != 0).sum()) == 0, st.unique().tolist()
    offs = off.cpu().tolist()
    for i in [0, 1, 4097, n - 1]:   # a sample against the oracle
        R, V = orc.synth_pair(seed + i, L, ne)
        assert bytes(out[offs[i]:offs[i + 1]].cpu().numpy()) == orc.encode(ONEPASS, R, V, p=16, q=1), i
    _decode_all_back(dg, ctx, torch, ref, ver, out, offs, n, L)
    # in place: the first 8192 streams
    m = 8192
    std = out[:offs[m]].cpu().numpy().tobytes()
    ref_h = ref[:m * L].cpu().numpy().tobytes()
    deltas = [dg.make_inplace(ref_h[i * L:(i + 1) * L], std[offs[i]:offs[i + 1]], policy="localmin")
              for i in range(m)]
    d_offs = [0]
    for d in deltas:
        d_offs.append(d_offs[-1] + len(d))
    d_dev = torch.frombuffer(bytearray(b"".join(deltas)), dtype=torch.uint8).to("cuda")
    plan = dg.DecodePlan(ctx, [(i * L, L, d_offs[i], len(deltas[i]), i * L, L) for i in range(m)])
    dec = torch.zeros(m * L, dtype=torch.uint8, device="cuda")
    dlen = torch.empty(m, dtype=torch.int64, device="cuda")
    dst = torch.empty(m, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    plan.run(ref.data_ptr(), d_dev.data_ptr(), dec.data_ptr(), dlen.data_ptr(), dst.data_ptr(), ctx.stream)
    torch.cuda.synchronize()
    assert int(dst.abs().sum()) == 0
    assert bool((dlen == L).all())
    assert bool(torch.equal(dec, ver[:m * L]))
    plan.close()
    del ref, ver, out, dec
    torch.cuda.empty_cache()
