"""In-place conversion (dg_make_inplace, host code in libdeltagpu.so) against
the reference's delta_make_inplace, byte for byte — CPU only, no GPU call.

Pinned by tests/golden/golden_inplace.json (minted from src/c by
make_golden.py, both cycle policies) and, where oracle/_ref exists, by a
randomised comparison with the reference on inputs with many CRWI cycles.
"""
from __future__ import annotations

import json
import os
import random

import pytest

from test_oracle import inplace_inputs

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = json.load(open(os.path.join(HERE, "golden", "golden_inplace.json")))["cases"]
POL = {0: "localmin", 1: "constant"}


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_make_inplace_matches_reference_golden(dg, orc, case):
    R, V = inplace_inputs(orc, case)
    std = orc.encode(case["algo"], R, V, p=16, q=case["q"])
    got = dg.make_inplace(R, std, POL[case["policy"]])
    assert got == bytes.fromhex(case["delta_hex"])
    rc, out = orc.decode(R, got)
    assert rc == 0 and out == V


def test_make_inplace_passthrough_and_errors(dg, orc):
    R = random.Random(2).randbytes(5000)
    V = R[2500:] + R[:2500]
    std = orc.encode(1, R, V, p=16, q=1)
    ip, st = dg.make_inplace(R, std, stats=True)
    assert st["already_inplace"] == 0 and ip[4] == 1
    again, st2 = dg.make_inplace(R, ip, stats=True)
    assert again == ip and st2["already_inplace"] == 1
    with pytest.raises(dg.DeltaError) as e:
        dg.make_inplace(R, b"XLT\x03" + std[4:])
    assert e.value.code == 8
    with pytest.raises(dg.DeltaError):
        dg.make_inplace(R, std[:30])


def _cyclic_pairs(n, seed):
    """Block permutations and swaps: CRWI graphs full of cycles."""
    rng = random.Random(seed)
    out = []
    for i in range(n):
        nb = rng.randrange(2, 24)
        blk = rng.randrange(20, 300)
        R = rng.randbytes(nb * blk)
        blocks = [R[k * blk:(k + 1) * blk] for k in range(nb)]
        rng.shuffle(blocks)
        if rng.random() < 0.5:
            blocks = blocks[::-1]
        V = b"".join(blocks)
        if rng.random() < 0.3:
            V = V[: len(V) // 2] + rng.randbytes(rng.randrange(1, 50)) + V[len(V) // 2:]
        out.append((R, V, rng.choice([1, 2]), rng.choice([4, 16]), rng.choice([1, 101, 1048573])))
    return out


def test_make_inplace_random_vs_reference(dg, orc, ref):
    for R, V, algo, p, q in _cyclic_pairs(150, 5):
        std = orc.encode(algo, R, V, p=p, q=q)
        for pol in (0, 1):
            want = ref.encode_inplace(algo, R, V, p=p, q=q, policy=pol)
            assert dg.make_inplace(R, std, POL[pol]) == want


def test_cli_inplace_subcommand_vs_reference(tmp_path, dg, orc):
    """`delta inplace ref delta_in delta_out [--policy P]` (main.c:427-480):
    same output file and stdout lines (Time excepted) as the reference CLI;
    host-only, so it runs without a GPU."""
    import subprocess
    root = os.path.dirname(HERE)
    cli = os.path.join(root, "delta-compression_amd", "bin", "delta")
    ref_cli = os.path.join(root, "oracle", "_ref", "delta")
    R, V, algo, p, q = _cyclic_pairs(1, 9)[0]
    (tmp_path / "r").write_bytes(R)
    (tmp_path / "d").write_bytes(orc.encode(algo, R, V, p=p, q=q))
    strip = lambda s: [l.replace("o_ref ", "o ") for l in s.splitlines() if not l.startswith("Time:")]
    for pol in ([], ["--policy", "constant"]):
        a = subprocess.run([cli, "inplace", str(tmp_path / "r"), str(tmp_path / "d"), str(tmp_path / "o")]
                           + pol, capture_output=True, text=True)
        assert a.returncode == 0, a.stderr
        mine = (tmp_path / "o").read_bytes()
        assert mine == dg.make_inplace(R, (tmp_path / "d").read_bytes(),
                                             "constant" if pol else "localmin")
        if os.path.exists(ref_cli):
            b = subprocess.run([ref_cli, "inplace", str(tmp_path / "r"), str(tmp_path / "d"),
                                str(tmp_path / "o_ref")] + pol, capture_output=True, text=True)
            assert b.returncode == 0
            assert (tmp_path / "o_ref").read_bytes() == mine
            assert strip(a.stdout) == strip(b.stdout) and strip(a.stdout)
        # already in-place: copied unchanged
        c = subprocess.run([cli, "inplace", str(tmp_path / "r"), str(tmp_path / "o"), str(tmp_path / "o2")],
                           capture_output=True, text=True)
        assert c.returncode == 0 and "already in-place" in c.stdout
        assert (tmp_path / "o2").read_bytes() == mine
