"""The command-list level of the ABI on the CPU: dg_delta_decode,
dg_encode_commands and the Python mirror's place/unplace (no GPU call).

Pinned by the reference-minted deltas in tests/golden/ (decode -> encode
reproduces every one byte for byte), by oracle-encoded deltas, and by a
restatement of delta.py:967-999's walk written here.  The error cases follow
encoding.c:111-178 (the reference exits; the library returns
DG_ERR_MALFORMED = 8).
"""
from __future__ import annotations

import json
import os
import random
import struct

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden.json")))["cases"]
GOLD_IP = json.load(open(os.path.join(HERE, "golden", "golden_inplace.json")))["cases"]
DELTAS = [c for c in GOLD + GOLD_IP if "delta_hex" in c]


def walk(data: bytes):
    """delta.py:967-999 / encoding.c:111-178, as plain tuples."""
    assert data[:4] == b"DLT\x03"
    pos, out = 25, []
    while pos < len(data):
        t = data[pos]
        pos += 1
        if t == 0:
            break
        if t == 1:
            out.append(("copy",) + struct.unpack_from(">III", data, pos))
            pos += 12
        else:
            dst, n = struct.unpack_from(">II", data, pos)
            out.append(("add", dst, data[pos + 8:pos + 8 + n]))
            pos += 8 + n
    return out, bool(data[4] & 1), struct.unpack_from(">I", data, 5)[0], data[9:17], data[17:25]


def as_tuples(dg, cmds):
    return [("copy", c.src, c.dst, c.length) if isinstance(c, dg.PlacedCopy) else ("add", c.dst, c.data)
            for c in cmds]


@pytest.mark.parametrize("case", DELTAS, ids=lambda c: c["name"])
def test_decode_encode_golden(dg, case):
    d = bytes.fromhex(case["delta_hex"])
    cmds, inplace, vsize, sc, dc = dg.decode_delta(d)
    w = walk(d)
    assert as_tuples(dg, cmds) == w[0] and (inplace, vsize, sc, dc) == w[1:]
    again = dg.encode_delta(cmds, inplace=inplace, version_size=vsize, src_crc=sc, dst_crc=dc)
    assert again == d
    i = dg.info(d)
    assert i["num_commands"] == len(cmds) and i["inplace"] == inplace


def test_place_unplace_roundtrip_oracle(dg, orc):
    rng = random.Random(11)
    for k in range(40):
        R = rng.randbytes(rng.randrange(0, 3000))
        V = bytearray(R[rng.randrange(0, len(R) + 1):] + rng.randbytes(rng.randrange(0, 200)) + R)
        for _ in range(rng.randrange(0, 30)):
            if V:
                V[rng.randrange(len(V))] = rng.randrange(256)
        V = bytes(V)
        d = orc.encode(1 + (k & 1), R, V, p=2 + k % 15, q=1 if k % 5 == 0 else 4099)
        placed, inplace, vsize, sc, dc = dg.decode_delta(d)
        cmds = dg.unplace_commands(placed)
        assert dg.output_size(cmds) == vsize == len(V)
        assert dg.place_commands(cmds) == placed      # standard deltas are already in place order
        assert dg.encode_delta(dg.place_commands(cmds), version_size=vsize, src_crc=sc, dst_crc=dc) == d
        # apply (delta.py:1046-1052 semantics) gives V back
        out = bytearray(vsize)
        for c in placed:
            if isinstance(c, dg.PlacedCopy):
                out[c.dst:c.dst + c.length] = R[c.src:c.src + c.length]
            else:
                out[c.dst:c.dst + len(c.data)] = c.data
        assert bytes(out) == V


def test_unplace_sorts_inplace_delta(dg):
    case = next(c for c in GOLD_IP if json.dumps(c).count("delta_hex") and c["policy"] == 0
                and len(c["delta_hex"]) > 200)
    placed = dg.decode_delta(bytes.fromhex(case["delta_hex"]))[0]
    cmds = dg.unplace_commands(placed)
    dsts = [p.dst for p in sorted(placed, key=lambda p: p.dst)]
    assert [p.dst for p in dg.place_commands(cmds)] == dsts


def test_decode_errors(dg):
    d = bytes.fromhex(next(c for c in GOLD if c["name"] == "paper_p2_q1")["delta_hex"])
    for bad in (b"", d[:24], b"XLT\x03" + d[4:], d[:25] + b"\x07", d[:25] + b"\x01" + b"\0" * 11,
                d[:25] + b"\x02" + b"\0" * 7, d[:25] + b"\x02\0\0\0\0\0\0\0\x05ab"):
        with pytest.raises(dg.DeltaError) as e:
            dg.decode_delta(bad)
        assert e.value.code == 8
    # no END byte: accepted at the buffer end, as encoding.c:134 does
    assert dg.decode_delta(d[:-1])[0] == dg.decode_delta(d)[0]
    # bytes after END are ignored
    assert dg.decode_delta(d + b"junk")[0] == dg.decode_delta(d)[0]


def test_encode_rejects_u32_overflow(dg):
    z = b"\0" * 8
    with pytest.raises(dg.DeltaError) as e:
        dg.encode_delta([dg.PlacedCopy(0, 0, 1 << 32)], version_size=1, src_crc=z, dst_crc=z)
    assert e.value.code == 1
    with pytest.raises(dg.DeltaError):
        dg.encode_delta([], version_size=1 << 32, src_crc=z, dst_crc=z)
    empty = dg.encode_delta([], version_size=0, src_crc=z, dst_crc=z)
    assert empty == b"DLT\x03\0" + b"\0" * 4 + z + z + b"\0"
    assert dg.decode_delta(empty)[0] == []
