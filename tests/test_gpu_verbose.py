"""`delta encode ... --verbose`: the reference's diagnostic lines on stderr
(onepass.c:64-69, 277-285; correcting.c:137-152, 200-214, 470-485,
523-576), from the device's counters and the delta, line for line against the
reference CLI built from src/c (oracle/_ref/delta)."""
from __future__ import annotations

import os
import random
import subprocess

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CLI = os.path.join(os.path.dirname(HERE), "delta-compression_amd", "bin", "delta")
REF = os.path.join(os.path.dirname(HERE), "oracle", "_ref", "delta")


def _cases(orc):
    rng = random.Random(7)
    R, V = orc.synth_pair(0xC2000000, 65536, 655)                      # C2 pair
    yield "onepass", R, V, []
    yield "onepass", R, V, ["--table-size", "1"]
    ins = R[:30000] + rng.randbytes(777) + R[30000:]                   # insertion: off-diagonal matches
    yield "onepass", R, ins, ["--table-size", "97"]
    yield "onepass", rng.randbytes(5000), rng.randbytes(7000), []      # no matches
    yield "onepass", b"", rng.randbytes(100), []                       # |R| < p
    blocks = [R[i:i + 4096] for i in range(0, 65536, 4096)]
    rng.shuffle(blocks)
    T = b"".join(blocks)                                               # block transposition
    yield "correcting", R, T, []
    yield "correcting", R, T, ["--table-size", "97"]
    yield "correcting", R, V, ["--table-size", "1"]
    low = bytes(rng.choice(b"ab") for _ in range(20000))               # low entropy: collisions
    yield "correcting", low, low[::-1], []
    yield "correcting", rng.randbytes(3000), rng.randbytes(3000), []


@pytest.mark.skipif(not os.path.exists(REF), reason="reference CLI not built (oracle/_ref)")
def test_verbose_lines_match_reference(tmp_path, orc):
    for k, (algo, R, V, extra) in enumerate(_cases(orc)):
        rp, vp = tmp_path / f"r{k}", tmp_path / f"v{k}"
        rp.write_bytes(R)
        vp.write_bytes(V)
        ours = subprocess.run([CLI, "encode", algo, str(rp), str(vp), str(tmp_path / f"d{k}"), "--verbose"] + extra,
                              capture_output=True, text=True)
        ref = subprocess.run([REF, "encode", algo, str(rp), str(vp), str(tmp_path / f"e{k}"), "--verbose"] + extra,
                             capture_output=True, text=True)
        assert ours.returncode == 0 and ref.returncode == 0, (ours.stderr, ref.stderr)
        assert (tmp_path / f"d{k}").read_bytes() == (tmp_path / f"e{k}").read_bytes(), k
        assert ours.stderr.splitlines() == ref.stderr.splitlines(), (k, algo, extra, ours.stderr, ref.stderr)
