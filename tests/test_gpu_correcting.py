"""GPU parity of the correcting path (src/c/correcting.c:81-495) against the
oracle, bit for bit, through the C ABI (dg_encode / dg_encode_batch /
dg_encode_plan_*).  Includes the reference-minted golden vectors (c4_*,
the SURVEY edge cases) and lookback-buffer sizes that force the ring to emit
and the tail correction (6b) to run.
"""
from __future__ import annotations

import hashlib
import json
import os

import pytest

from cases import DEFAULT_Q, random_cases, small_cases

pytestmark = pytest.mark.gpu

CORRECTING = 2
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("case", small_cases(), ids=lambda c: c[0])
def test_correcting_small_cases(dg, ctx, orc, case):
    name, R, V, p, q = case
    got = dg.encode(R, V, "correcting", p=p, q=q, ctx=ctx)
    assert got == orc.encode(CORRECTING, R, V, p=p, q=q)


@pytest.mark.parametrize("buf_cap", [1, 2, 5, 256])
def test_correcting_random_batch(dg, ctx, orc, buf_cap):
    cs = random_cases(200, seed=1234 + buf_cap)
    by_pq = {}
    for name, R, V, p, q in cs:
        by_pq.setdefault((p, q), []).append((name, R, V))
    for (p, q), items in by_pq.items():
        got = dg.encode_batch([(R, V) for _, R, V in items], "correcting", p=p, q=q,
                              buf_cap=buf_cap, ctx=ctx)
        for (name, R, V), g in zip(items, got):
            assert g == orc.encode(CORRECTING, R, V, p=p, q=q, buf_cap=buf_cap), (name, buf_cap)


def test_correcting_golden_on_device(dg, ctx, orc):
    from test_gpu_parity import _golden_inputs
    cases = [c for c in json.load(open(os.path.join(HERE, "golden", "golden.json")))["cases"]
             if c["algo"] == CORRECTING]
    assert cases
    groups = {}
    for c in cases:
        groups.setdefault((c["p"], c["q"]), []).append(c)
    for (p, q), cs in groups.items():
        ins = [_golden_inputs(orc, c) for c in cs]
        outs = dg.encode_batch(ins, "correcting", p=p, q=q, ctx=ctx)
        for c, d in zip(cs, outs):
            assert len(d) == c["delta_len"], c["name"]
            assert hashlib.sha256(d).hexdigest() == c["delta_sha256"], c["name"]


def test_correcting_c4_sample(dg, ctx, orc):
    """C4 geometry: gen_transpositions-style pairs (8..64 blocks, 50% moved,
    ~256 KiB), --table-size 1; every pair bit-exact and decodable."""
    pairs = []
    for i in range(24):
        nb = 8 + (i % 57)
        pairs.append(orc.synth_transpose(0xC4000000 + i, nb, 262144 // nb, 50))
    outs = dg.encode_batch(pairs, "correcting", p=16, q=1, ctx=ctx)
    for i, ((R, V), d) in enumerate(zip(pairs, outs)):
        assert d == orc.encode(CORRECTING, R, V, p=16, q=1), i
        assert dg.decode(R, d, ctx=ctx) == V


def _low_entropy_cases(n, seed):
    """Repetitive inputs: many seed collisions, backward extensions into
    already-encoded V and hence tail corrections (correcting.c:364-445)."""
    import random
    rng = random.Random(seed)
    out = []
    for i in range(n):
        alpha = rng.choice([2, 3, 4, 16])
        L = rng.choice([200, 1000, 3000])
        R = bytes(65 + rng.randrange(alpha) for _ in range(L))
        unit = bytes(65 + rng.randrange(alpha) for _ in range(rng.randrange(5, 60)))
        V = bytearray()
        while len(V) < L:
            pick = rng.randrange(3)
            if pick == 0:
                a = rng.randrange(L)
                V += R[a:a + rng.randrange(10, 200)]
            elif pick == 1:
                V += unit * rng.randrange(1, 5)
            else:
                V += bytes(65 + rng.randrange(alpha) for _ in range(rng.randrange(1, 30)))
        out.append((f"lowent{i}", R, bytes(V), rng.choice([2, 4, 16]), rng.choice([1, 7, 101])))
    return out


@pytest.mark.parametrize("buf_cap", [1, 3, 256])
def test_correcting_low_entropy(dg, ctx, orc, buf_cap):
    cs = _low_entropy_cases(120, seed=77 + buf_cap)
    by_pq = {}
    for name, R, V, p, q in cs:
        by_pq.setdefault((p, q), []).append((name, R, V))
    for (p, q), items in by_pq.items():
        got = dg.encode_batch([(R, V) for _, R, V in items], "correcting", p=p, q=q,
                              buf_cap=buf_cap, ctx=ctx)
        for (name, R, V), g in zip(items, got):
            assert g == orc.encode(CORRECTING, R, V, p=p, q=q, buf_cap=buf_cap), (name, buf_cap)


def test_correcting_c4_device_batch(dg, ctx, orc, torch_cuda):
    """C4 batch generated on the device (dg_synth_transpose_pairs_device) equals
    the oracle's generator; encoded through the plan API, sampled pairs are
    bit-exact and the rest are checked by status."""
    import ctypes as C
    torch = torch_cuda
    n, target, seed = 128, 262144, 0xC4000000
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
    plan = dg.EncodePlan(ctx, "correcting", lay, q=1)
    out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), off.data_ptr(),
             st.data_ptr(), ctx.stream)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0
    offs = off.cpu().tolist()
    refc, verc, outc = ref.cpu(), ver.cpu(), out.cpu()
    for i in list(range(0, n, 9)) + [n - 1]:
        nb = 8 + (i % 57)
        R, V = orc.synth_transpose(seed + i, nb, target // nb, 50)
        ro, rl, vo, vl = lay[i]
        assert bytes(refc[ro:ro + rl].numpy()) == R
        assert bytes(verc[vo:vo + vl].numpy()) == V
        assert bytes(outc[offs[i]:offs[i + 1]].numpy()) == orc.encode(CORRECTING, R, V, p=16, q=1), i


@pytest.mark.parametrize("build", ["lds", "global"])
def test_correcting_build_paths(dg, ctx, orc, build):
    """Both R-index builds (one block's LDS per pair, or memory-side atomicMin
    over a (pair, chunk) grid) give the oracle's bytes.  The plan picks the
    LDS build when every pair's index fits one block's LDS: q = 1 keeps the
    indexes small enough; the default --table-size (q = 1048573) does not
    fit and takes the global build."""
    q = 1 if build == "lds" else DEFAULT_Q
    cs = [c for c in random_cases(120, seed=4242) if c[3] == 16]
    got = dg.encode_batch([(R, V) for _, R, V, _, _ in cs], "correcting", p=16, q=q, ctx=ctx)
    for (name, R, V, _, _), g in zip(cs, got):
        assert g == orc.encode(CORRECTING, R, V, p=16, q=q), (name, build)
