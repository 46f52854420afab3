"""GPU parity: the HIP path against the oracle, bit for bit.

Every comparison here is exact (integer/byte work).  The oracle is the CPU
restatement in oracle/ (itself pinned to the reference in tests/test_oracle.py
and tests/golden/).
"""
from __future__ import annotations

import os
import random

import pytest

from cases import DEFAULT_Q, random_cases, small_cases

pytestmark = pytest.mark.gpu

ONEPASS, CORRECTING = 1, 2


# ── CRC-64/XZ ────────────────────────────────────────────────────────────

def test_crc_known_answers(dg, ctx):
    # src/python/test_delta.py:970-977, src/cpp/tests/test_hash.cpp:124-136
    assert dg.crc64_xz(b"123456789", ctx=ctx).hex() == "995dc9bbdf1939fa"
    assert dg.crc64_xz(b"", ctx=ctx) == bytes(8)


@pytest.mark.parametrize("n", [1, 7, 8, 9, 15, 16, 17, 1000, 65535, 65536, 65537, 200001, 1 << 20])
def test_crc_lengths(dg, ctx, orc, n):
    data = random.Random(n).randbytes(n)
    assert dg.crc64_xz(data, ctx=ctx) == orc.crc64_xz(data)


def test_crc_batch_alignments(dg, ctx, orc, torch_cuda):
    torch = torch_cuda
    rng = random.Random(5)
    blob = rng.randbytes(300000)
    spans, exp = [], []
    for i in range(200):
        off = rng.randrange(0, 200000)
        ln = rng.choice([0, 3, 8, 31, 64, 1000, 4097, 65536 + rng.randrange(64), 90000])
        spans.append((off, ln))
        exp.append(int.from_bytes(orc.crc64_xz(blob[off:off + ln]), "big"))
    d = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    out = torch.zeros(len(spans), dtype=torch.int64, device="cuda")
    import ctypes as C
    arr = (dg._lib.Span * len(spans))(*[dg._lib.Span(o, l) for o, l in spans])
    torch.cuda.synchronize()
    ctx.check(dg.lib.dg_crc64_xz_batch_device(ctx.handle, d.data_ptr(), arr, len(spans),
                                              out.data_ptr(), None), "crc batch")
    got = [v & (2**64 - 1) for v in out.cpu().tolist()]
    assert got == exp


# ── onepass encode ───────────────────────────────────────────────────────

@pytest.mark.parametrize("case", small_cases(), ids=lambda c: c[0])
def test_onepass_small_cases(dg, ctx_mode, orc, case):
    name, R, V, p, q = case
    got = dg.encode(R, V, "onepass", p=p, q=q, ctx=ctx_mode)
    assert got == orc.encode(ONEPASS, R, V, p=p, q=q)


def test_onepass_random_batch(dg, ctx_mode, orc):
    ctx = ctx_mode
    cs = random_cases(300, seed=99)
    by_pq = {}
    for name, R, V, p, q in cs:
        by_pq.setdefault((p, q), []).append((name, R, V))
    for (p, q), items in by_pq.items():
        got = dg.encode_batch([(R, V) for _, R, V in items], "onepass", p=p, q=q, ctx=ctx)
        for (name, R, V), g in zip(items, got):
            assert g == orc.encode(ONEPASS, R, V, p=p, q=q), name


def _device_batch(dg, ctx, torch, n, L, rate, seed, algo="onepass", q=1, check=64):
    ref = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    ver = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    n_edits = int(rate * L + 0.5)
    ctx.check(dg.lib.dg_synth_edit_pairs_device(ctx.handle, ref.data_ptr(), ver.data_ptr(), n, L,
                                                seed, n_edits, None), "synth")
    plan = dg.EncodePlan(ctx, algo, [(i * L, L, i * L, L) for i in range(n)], q=q)
    out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
    off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), off.data_ptr(),
             st.data_ptr(), ctx.stream)
    torch.cuda.synchronize()
    return plan, ref, ver, out, off, st, n_edits


def test_onepass_c2_batch_sample(dg, ctx_mode, orc, torch_cuda):
    """C2 geometry (64 KiB pairs, 1% edits, --table-size 1): device-generated
    inputs equal the oracle's generator; sampled pairs bit-exact."""
    torch = torch_cuda
    ctx = ctx_mode
    n, L, seed = 256, 65536, 0xC2000000
    plan, ref, ver, out, off, st, ne = _device_batch(dg, ctx, torch, n, L, 0.01, seed)
    stc = st.cpu()
    assert int(stc.abs().sum()) == 0
    offs = off.cpu().tolist()
    outc = out.cpu()
    refc, verc = ref.cpu(), ver.cpu()
    for i in list(range(0, n, 17)) + [n - 1]:
        R, V = orc.synth_pair(seed + i, L, ne)
        assert bytes(refc[i * L:(i + 1) * L].numpy()) == R
        assert bytes(verc[i * L:(i + 1) * L].numpy()) == V
        got = bytes(outc[offs[i]:offs[i + 1]].numpy())
        assert got == orc.encode(ONEPASS, R, V, p=16, q=1), i


# ── decode ───────────────────────────────────────────────────────────────

@pytest.mark.parametrize("case", small_cases()[:24], ids=lambda c: c[0])
def test_decode_roundtrip(dg, ctx, orc, case):
    name, R, V, p, q = case
    delta = orc.encode(ONEPASS, R, V, p=p, q=q)
    assert dg.decode(R, delta, ctx=ctx) == V


def test_decode_crc_errors(dg, ctx, orc):
    R = random.Random(1).randbytes(3000)
    V = R[:1000] + b"xyz" + R[1000:]
    delta = orc.encode(ONEPASS, R, V, p=16, q=DEFAULT_Q)
    with pytest.raises(dg.DeltaError) as e:
        dg.decode(R[:-1] + b"\x00", delta, ctx=ctx)
    assert e.value.code == 9
    bad = bytearray(delta)
    bad[17] ^= 1
    with pytest.raises(dg.DeltaError) as e:
        dg.decode(R, bytes(bad), ctx=ctx)
    assert e.value.code == 10
    assert dg.decode(R, bytes(bad), ignore_hash=True, ctx=ctx) == V
    with pytest.raises(dg.DeltaError) as e:
        dg.decode(R, b"XLT\x03" + delta[4:], ctx=ctx)
    assert e.value.code == 8


# ── golden fixtures (minted from the reference) on the device ─────────────

def _golden():
    import json
    here = os.path.dirname(os.path.abspath(__file__))
    return json.load(open(os.path.join(here, "golden", "golden.json")))["cases"]


def _golden_inputs(orc, case):
    kind = case["kind"]
    if kind == "small":
        m = {c[0]: c for c in small_cases()}
        return m[case["name"]][1], m[case["name"]][2]
    if kind == "synth_edits":
        return orc.synth_pair(case["seed"], case["pair_len"], case["n_edits"])
    if kind == "synth_transpose":
        return orc.synth_transpose(case["seed"], case["num_blocks"], case["mean"], case["pct"])
    if kind == "synth_shift":
        return orc.synth_shift(case["seed"], case["pair_len"], case["n_edits"], case["indel_pct"])
    return orc.synth_random(case["r_seed"], 1 << 20), orc.synth_random(case["v_seed"], 1 << 20)


def test_golden_onepass_on_device(dg, ctx_mode, orc):
    import hashlib
    ctx = ctx_mode
    groups = {}
    for c in _golden():
        if c["algo"] != ONEPASS:
            continue
        groups.setdefault((c["p"], c["q"]), []).append(c)
    for (p, q), cs in groups.items():
        ins = [_golden_inputs(orc, c) for c in cs]
        outs = dg.encode_batch(ins, "onepass", p=p, q=q, ctx=ctx)
        for c, d in zip(cs, outs):
            assert len(d) == c["delta_len"], c["name"]
            assert hashlib.sha256(d).hexdigest() == c["delta_sha256"], c["name"]


# ── full C2 batch: every pair decodes back to V on the device ─────────────

def test_c2_full_batch_roundtrip(dg, ctx_mode, orc, torch_cuda):
    torch = torch_cuda
    ctx = ctx_mode
    n, L, seed = 4096, 65536, 0xC2000000
    plan, ref, ver, out, off, st, ne = _device_batch(dg, ctx, torch, n, L, 0.01, seed)
    assert int(st.abs().sum()) == 0
    offs = off.cpu()
    import ctypes as C
    descs = (dg._lib.DecodeDesc * n)(*[
        dg._lib.DecodeDesc(i * L, L, int(offs[i]), int(offs[i + 1] - offs[i]), i * L, L)
        for i in range(n)])
    dec = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    dlen = torch.empty(n, dtype=torch.int64, device="cuda")
    dst = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    ctx.check(dg.lib.dg_decode_batch_device(ctx.handle, ref.data_ptr(), out.data_ptr(), descs, n, 0,
                                            dec.data_ptr(), dlen.data_ptr(), dst.data_ptr(), None),
              "decode batch")
    torch.cuda.synchronize()
    assert int(dst.abs().sum()) == 0          # src and dst CRC verified on device
    assert bool(torch.equal(dec, ver))        # every V reproduced
    # the first pairs equal the reference-minted golden deltas
    import hashlib
    gold = {c["name"]: c for c in _golden()}
    outc = out.cpu()
    for i in range(8):
        d = bytes(outc[int(offs[i]):int(offs[i + 1])].numpy())
        assert hashlib.sha256(d).hexdigest() == gold[f"c2_{i}"]["delta_sha256"]


# ── CLI: same bytes and report lines as the reference CLI ─────────────────

def test_cli_encode_decode_vs_reference(tmp_path, orc):
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    cli = os.path.join(os.path.dirname(here), "delta-compression_amd", "bin", "delta")
    ref_cli = os.path.join(os.path.dirname(here), "oracle", "_ref", "delta")
    R = orc.synth_random(1, 1 << 20)
    V = orc.synth_random(2, 1 << 20)
    rp, vp = tmp_path / "r.bin", tmp_path / "v.bin"
    rp.write_bytes(R)
    vp.write_bytes(V)
    a = subprocess.run([cli, "encode", "onepass", str(rp), str(vp), str(tmp_path / "d")],
                       capture_output=True, text=True)
    assert a.returncode == 0, a.stderr
    d = (tmp_path / "d").read_bytes()
    assert len(d) == 1048611                  # C1: one ADD
    assert d == orc.encode(ONEPASS, R, V)
    if os.path.exists(ref_cli):
        b = subprocess.run([ref_cli, "encode", "onepass", str(rp), str(vp), str(tmp_path / "d_ref")],
                           capture_output=True, text=True)
        assert (tmp_path / "d_ref").read_bytes() == d
        strip = lambda s: [l for l in s.splitlines() if not l.startswith(("Time:", "Delta:"))]
        assert strip(a.stdout) == strip(b.stdout)
    c = subprocess.run([cli, "decode", str(rp), str(tmp_path / "d"), str(tmp_path / "out")],
                       capture_output=True, text=True)
    assert c.returncode == 0, c.stderr
    assert (tmp_path / "out").read_bytes() == V
    bad = subprocess.run([cli, "decode", str(vp), str(tmp_path / "d"), str(tmp_path / "out2")],
                         capture_output=True, text=True)
    assert bad.returncode == 1 and "source file does not match delta" in bad.stderr


def test_cli_decode_failures_vs_reference(tmp_path, orc):
    """decode with a wrong R and with a corrupted dst_crc, with and without
    --ignore-hash: stderr, exit code and the output file as the reference CLI
    (main.c:341-385: the source check exits before writing; the output check
    fails after the file is written; --ignore-hash prints the two warnings)."""
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    cli = os.path.join(os.path.dirname(here), "delta-compression_amd", "bin", "delta")
    ref_cli = os.path.join(os.path.dirname(here), "oracle", "_ref", "delta")
    if not os.path.exists(ref_cli):
        pytest.skip("oracle/_ref/delta not built")
    rng = random.Random(5)
    R = rng.randbytes(50000)
    V = R[:20000] + rng.randbytes(300) + R[20000:]
    d = orc.encode(ONEPASS, R, V, p=16, q=97)
    wrong_r = bytearray(R)
    wrong_r[100] ^= 1          # same length: decodes to V except one byte
    bad_dst = bytearray(d)
    bad_dst[17] ^= 0x40        # dst_crc byte (header: magic 4, flags 1, size 4, src_crc 8)
    files = {"r": bytes(R), "wr": bytes(wrong_r), "d": d, "bd": bytes(bad_dst)}
    for k, v in files.items():
        (tmp_path / k).write_bytes(v)
    cases = [("wr", "d", []), ("r", "bd", []), ("wr", "d", ["--ignore-hash"]), ("r", "bd", ["--ignore-hash"]),
             ("wr", "bd", ["--ignore-hash"])]
    for i, (r, dd, extra) in enumerate(cases):
        res = []
        for tool in (cli, ref_cli):
            out = tmp_path / f"o_{i}_{os.path.basename(os.path.dirname(os.path.dirname(tool)))}"
            p = subprocess.run([tool, "decode", str(tmp_path / r), str(tmp_path / dd), str(out)] + extra,
                               capture_output=True, text=True)
            res.append((p.returncode, p.stderr, out.read_bytes() if out.exists() else None))
        assert res[0] == res[1], (r, dd, extra, res[0][:2], res[1][:2])
    # the cases do what they are meant to
    assert res[0][0] == 0 and res[0][1].count("warning") == 2


# ── in-place deltas minted by the reference (delta_make_inplace) ─────────

def test_golden_inplace_decode_on_device(dg, ctx, orc):
    """Every reference in-place delta (tests/golden/golden_inplace.json,
    both cycle policies, onepass and correcting) replays on the device into
    a max(|R|, |V|) buffer in command order (apply.c:253-284) and passes the
    on-device src/dst CRC checks."""
    import json
    from test_oracle import inplace_inputs
    here = os.path.dirname(os.path.abspath(__file__))
    cases = json.load(open(os.path.join(here, "golden", "golden_inplace.json")))["cases"]
    for c in cases:
        R, V = inplace_inputs(orc, c)
        d = bytes.fromhex(c["delta_hex"])
        assert dg.decode(R, d, ctx=ctx) == V, c["name"]


def test_decode_plan_batch_mixed(dg, ctx, orc, torch_cuda):
    """dg_decode_plan over a batch mixing standard and in-place deltas with
    corrupted ones: per-stream status precedence malformed > src CRC > dst CRC
    (main.c:335-385), good streams reconstructed exactly, run twice (the plan
    is reusable and needs no host synchronisation between its kernels)."""
    import json
    torch = torch_cuda
    from test_oracle import inplace_inputs
    here = os.path.dirname(os.path.abspath(__file__))
    ip = json.load(open(os.path.join(here, "golden", "golden_inplace.json")))["cases"][:12]
    items = []   # (R, delta, expected V or None, expected status)
    for c in ip:
        R, V = inplace_inputs(orc, c)
        items.append((R, bytes.fromhex(c["delta_hex"]), V, 0))
    rng = random.Random(11)
    for k in range(12):
        R = rng.randbytes(rng.choice([0, 10, 5000, 70000]))
        V = R[: len(R) // 2] + rng.randbytes(300) + R[len(R) // 2:]
        d = orc.encode(ONEPASS, R, V, p=16, q=DEFAULT_Q)
        items.append((R, d, V, 0))
        if k % 3 == 0:
            items.append((R + b"!", d, None, 9))                      # wrong source
        if k % 3 == 1:
            bad = bytearray(d); bad[17] ^= 0x40
            items.append((R, bytes(bad), None, 10))                  # wrong dst CRC
        if k % 3 == 2:
            items.append((R, d[:25] + b"\x07" + d[26:], None, 8))     # bad command tag
            items.append((R + b"!", b"DLT\x02" + d[4:], None, 8))    # magic beats src CRC
    up = lambda x: (x + 15) // 16 * 16
    r_off, d_off, o_off, descs = 0, 0, 0, []
    for R, d, V, _ in items:
        vs = int.from_bytes(d[5:9], "big") if len(d) >= 9 else 0
        cap = max(vs, len(R), 1)
        descs.append((r_off, len(R), d_off, len(d), o_off, cap))
        r_off += up(len(R)); d_off += len(d); o_off += up(cap)
    ref = torch.zeros(max(r_off, 16), dtype=torch.uint8)
    dl = torch.zeros(max(d_off, 16), dtype=torch.uint8)
    for (R, d, _, _), (ro, rl, do, dln, _, _) in zip(items, descs):
        if rl:
            ref[ro:ro + rl] = torch.frombuffer(bytearray(R), dtype=torch.uint8)
        dl[do:do + dln] = torch.frombuffer(bytearray(d), dtype=torch.uint8)
    ref, dl = ref.cuda(), dl.cuda()
    out = torch.zeros(max(o_off, 16), dtype=torch.uint8, device="cuda")
    olen = torch.zeros(len(items), dtype=torch.int64, device="cuda")
    st = torch.zeros(len(items), dtype=torch.int32, device="cuda")
    plan = dg.DecodePlan(ctx, descs)
    for _ in range(2):
        out.zero_()
        torch.cuda.synchronize()
        plan.run(ref.data_ptr(), dl.data_ptr(), out.data_ptr(), olen.data_ptr(), st.data_ptr(),
                 ctx.stream)
        torch.cuda.synchronize()
        stc, oc, lc = st.cpu().tolist(), out.cpu(), olen.cpu().tolist()
        for i, ((R, d, V, want), ds) in enumerate(zip(items, descs)):
            assert stc[i] == want, (i, stc[i], want)
            if want == 0:
                assert lc[i] == len(V)
                assert bytes(oc[ds[4]:ds[4] + len(V)].numpy()) == V, i


def test_decode_plan_rejects_overlapping_arenas(dg, ctx, orc, torch_cuda):
    """An output arena overlapping the reference (a one-buffer in-place decode)
    or the delta bytes is refused before anything is written: the
    kernel writes the output image before it reads R for the source CRC."""
    torch = torch_cuda
    R = bytes(range(256)) * 16
    V = R[:2000] + b"xyz" + R[2000:]
    d = orc.encode(ONEPASS, R, V, p=16, q=97)
    buf = torch.zeros(16384, dtype=torch.uint8, device="cuda")
    buf[:len(R)] = torch.frombuffer(bytearray(R), dtype=torch.uint8).cuda()
    dl = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    olen = torch.zeros(1, dtype=torch.int64, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    plan = dg.DecodePlan(ctx, [(0, len(R), 0, len(d), 0, len(V))])
    before = buf.clone()
    try:
        for out_ptr in (buf.data_ptr(),            # out == ref
                        buf.data_ptr() + 2048,     # out starts inside ref
                        dl.data_ptr()):            # out == delta
            with pytest.raises(dg.DeltaError) as e:
                plan.run(buf.data_ptr(), dl.data_ptr(), out_ptr, olen.data_ptr(), st.data_ptr(), ctx.stream)
            assert e.value.code == 1
        torch.cuda.synchronize()
        assert torch.equal(buf, before)
        # right after R in the same allocation: disjoint, so it decodes
        plan.run(buf.data_ptr(), dl.data_ptr(), buf.data_ptr() + len(R), olen.data_ptr(), st.data_ptr(),
                 ctx.stream)
        torch.cuda.synchronize()
        assert int(st.item()) == 0 and bytes(buf[len(R):len(R) + len(V)].cpu().numpy()) == V
    finally:
        plan.close()


def test_decode_plan_interleaved_arenas(dg, ctx, orc, torch_cuda):
    """References and outputs interleaved in ONE allocation at disjoint
    offsets: the arenas' extents overlap but no output byte a
    descriptor names is a reference byte, so the run decodes; moving one
    output onto a reference is refused."""
    torch = torch_cuda
    rng = random.Random(77)
    R0, R1 = rng.randbytes(4096), rng.randbytes(4096)
    V0, V1 = R0[:100] + b"ab" + R0[100:4000], R1[:3000] + b"Z" * 50 + R1[3000:]
    d0 = orc.encode(ONEPASS, R0, V0, p=16, q=97)
    d1 = orc.encode(ONEPASS, R1, V1, p=16, q=97)
    # [R0 | out0 | R1 | out1], each region 8 KiB
    buf = torch.zeros(32768, dtype=torch.uint8, device="cuda")
    buf[0:4096] = torch.frombuffer(bytearray(R0), dtype=torch.uint8).cuda()
    buf[16384:16384 + 4096] = torch.frombuffer(bytearray(R1), dtype=torch.uint8).cuda()
    dl = torch.frombuffer(bytearray(d0 + d1), dtype=torch.uint8).cuda()
    olen = torch.zeros(2, dtype=torch.int64, device="cuda")
    st = torch.zeros(2, dtype=torch.int32, device="cuda")
    descs = [(0, 4096, 0, len(d0), 8192, 8192), (16384, 4096, len(d0), len(d1), 24576, 8192)]
    plan = dg.DecodePlan(ctx, descs)
    try:
        plan.run(buf.data_ptr(), dl.data_ptr(), buf.data_ptr(), olen.data_ptr(), st.data_ptr(), ctx.stream)
        torch.cuda.synchronize()
        assert st.cpu().tolist() == [0, 0]
        assert bytes(buf[8192:8192 + len(V0)].cpu().numpy()) == V0
        assert bytes(buf[24576:24576 + len(V1)].cpu().numpy()) == V1
    finally:
        plan.close()
    bad = dg.DecodePlan(ctx, [descs[0], (16384, 4096, len(d0), len(d1), 14336, 8192)])   # out1 over R1
    try:
        with pytest.raises(dg.DeltaError) as e:
            bad.run(buf.data_ptr(), dl.data_ptr(), buf.data_ptr(), olen.data_ptr(), st.data_ptr(), ctx.stream)
        assert e.value.code == 1
    finally:
        bad.close()


def test_encode_inplace_vs_reference_golden(dg, ctx, orc):
    """dg_encode with DG_OPT_INPLACE (device encode + host CRWI conversion)
    reproduces every reference in-place delta (main.c encode --inplace)."""
    import json
    from test_oracle import inplace_inputs
    here = os.path.dirname(os.path.abspath(__file__))
    pol = {0: "localmin", 1: "constant"}
    for c in json.load(open(os.path.join(here, "golden", "golden_inplace.json")))["cases"]:
        R, V = inplace_inputs(orc, c)
        algo = "onepass" if c["algo"] == ONEPASS else "correcting"
        got = dg.encode(R, V, algo, p=16, q=c["q"], inplace=True, policy=pol[c["policy"]], ctx=ctx)
        assert got == bytes.fromhex(c["delta_hex"]), c["name"]


def test_cli_encode_inplace_vs_reference(tmp_path, orc):
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    cli = os.path.join(os.path.dirname(here), "delta-compression_amd", "bin", "delta")
    ref_cli = os.path.join(os.path.dirname(here), "oracle", "_ref", "delta")
    R, V = orc.synth_transpose(0xC4000001, 9, 4000, 50)
    (tmp_path / "r").write_bytes(R)
    (tmp_path / "v").write_bytes(V)
    for pol in ([], ["--policy", "constant"]):
        args = ["encode", "correcting", str(tmp_path / "r"), str(tmp_path / "v")]
        a = subprocess.run([cli] + args + [str(tmp_path / "d"), "--inplace", "--table-size", "1"] + pol,
                           capture_output=True, text=True)
        assert a.returncode == 0, a.stderr
        d = (tmp_path / "d").read_bytes()
        assert d[4] == 1
        c = subprocess.run([cli, "decode", str(tmp_path / "r"), str(tmp_path / "d"), str(tmp_path / "o")],
                           capture_output=True, text=True)
        assert c.returncode == 0 and (tmp_path / "o").read_bytes() == V
        if os.path.exists(ref_cli):
            b = subprocess.run([ref_cli] + args + [str(tmp_path / "d_ref"), "--inplace", "--table-size", "1"]
                               + pol, capture_output=True, text=True)
            assert (tmp_path / "d_ref").read_bytes() == d
            strip = lambda s: [l for l in s.splitlines() if not l.startswith(("Time:", "Delta:"))]
            assert strip(a.stdout) == strip(b.stdout)
