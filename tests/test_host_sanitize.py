"""The library's host-only code under AddressSanitizer + UBSan (CPU, no GPU).

dg_format.cpp (dg_delta_info / dg_delta_decode / dg_encode_commands) and
dg_inplace.cpp (dg_make_inplace) contain no HIP, so they are compiled here
with g++ -fsanitize=address,undefined together with tests/sanitize/
host_fuzz.cpp and driven over a corpus of reference-minted deltas
(tests/golden/*.json), oracle-encoded pairs with many CRWI cycles, and every
truncation plus seeded byte mutations of each (see host_fuzz.cpp).  The
oracle only makes inputs here.
"""
from __future__ import annotations

import json
import os
import random
import shutil
import struct
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "delta-compression_amd", "csrc")


def _corpus(orc) -> bytes:
    from test_oracle import inplace_inputs
    out = bytearray()

    def rec(R: bytes, d: bytes):
        out.extend(struct.pack("<I", len(R)) + R + struct.pack("<I", len(d)) + d)

    g = json.load(open(os.path.join(HERE, "golden", "golden.json")))["cases"]
    for c in g:   # the small cases carry their bytes; R for them is not needed by the walk
        if "delta_hex" in c and len(c["delta_hex"]) < 40000:
            rec(b"", bytes.fromhex(c["delta_hex"]))
    for c in json.load(open(os.path.join(HERE, "golden", "golden_inplace.json")))["cases"][:12]:
        R, V = inplace_inputs(orc, c)
        rec(R, orc.encode(c["algo"], R, V, p=16, q=c["q"]))     # standard: converted both ways
        rec(R, bytes.fromhex(c["delta_hex"]))                    # reference in-place: passthrough
    rng = random.Random(7)
    for i in range(24):   # block permutations: CRWI graphs full of cycles
        nb, blk = rng.randrange(2, 20), rng.randrange(20, 200)
        R = rng.randbytes(nb * blk)
        blocks = [R[k * blk:(k + 1) * blk] for k in range(nb)]
        rng.shuffle(blocks)
        V = b"".join(blocks)
        if i % 3 == 0:
            V = V[:len(V) // 2] + rng.randbytes(40) + V[len(V) // 2:]
        rec(R, orc.encode(1 + (i & 1), R, V, p=4 + (i % 3) * 4, q=1 if i % 4 == 0 else 4099))
    return bytes(out)


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_host_code_under_asan_ubsan(orc, tmp_path):
    exe = tmp_path / "host_fuzz"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           os.path.join(HERE, "sanitize", "host_fuzz.cpp"),
           os.path.join(CSRC, "dg_format.cpp"), os.path.join(CSRC, "dg_inplace.cpp"),
           "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    corpus = tmp_path / "corpus.bin"
    corpus.write_bytes(_corpus(orc))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    p = subprocess.run([str(exe), str(corpus)], capture_output=True, text=True, env=env, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "failures 0" in p.stdout
