"""Integer models of two device arithmetic shortcuts (CPU only).

* `roll61w` (dg_correcting.hip): the correcting build's rolling step on a
  weakly reduced fingerprint (residue + 0..2 M, high dword <= 2^29) in dword
  arithmetic with explicit carries, and `fp61_canon`'s single-dword fix-up.
  Modelled bit for bit with Python integers and checked against
  (fp * 263 + nb + in) mod M over random, boundary and chained inputs.
* `mod_q_small` (dg_devutil.h): x mod q in FP64 with 1/q rounded DOWN, so the
  quotient estimate is exact or one short and a single fix-up suffices.
  Python floats are IEEE doubles; y = xh (2^32 mod q) + xl and the final
  fma are exact here (< 2^53), so only the product y * inv rounds, as on the
  device.
"""
import math
import random
import struct
from fractions import Fraction

M = (1 << 61) - 1
BASE = 263
MASK29 = (1 << 29) - 1
U32 = 0xFFFFFFFF


def roll61w(fp, nb, inb):
    lo, hi = fp & U32, fp >> 32
    assert hi <= (1 << 29)
    P = lo * BASE + nb                       # one 32x32+64 multiply-add
    Q = hi * BASE
    s = ((Q >> 29) & U32) + inb
    tl = ((P & U32) + s) & U32
    carry = 1 if tl < s else 0
    th = ((P >> 32) + (Q & MASK29) + carry) & U32
    f = th >> 29
    rl = (tl + f) & U32
    rh = (th & MASK29) + (1 if rl < f else 0)
    return (rh << 32) | rl


def fp61_canon(r):
    ge = r >= M
    lo = ((r & U32) + (1 if ge else 0)) & U32
    hi = 0 if ge else r >> 32
    return (hi << 32) | lo


def test_roll61w_matches_the_residue():
    rng = random.Random(61)
    edge_fp = [0, 1, M - 1, M, M + 1, M + 2, (1 << 61) - (1 << 40), (MASK29 << 32) | U32]
    edge_nb = [0, 1, M - 1, M - 263, 1 << 60]
    for _ in range(40000):
        fp = rng.choice(edge_fp) if rng.random() < 0.2 else rng.randrange(M + 3)
        nb = rng.choice(edge_nb) if rng.random() < 0.2 else rng.randrange(M)
        inb = rng.randrange(256)
        r = roll61w(fp, nb, inb)
        assert r <= M + 2 and (r >> 32) <= (1 << 29)
        assert fp61_canon(r) == (fp * BASE + nb + inb) % M
    for _ in range(300):   # chains never leave the weak range
        fp = rng.randrange(M)
        ref = fp
        for _ in range(64):
            nb, inb = rng.randrange(M), rng.randrange(256)
            fp = roll61w(fp, nb, inb)
            ref = (ref * BASE + nb + inb) % M
            assert fp61_canon(fp) == ref


def _inv_down(q):
    inv = 1.0 / q
    if Fraction(inv) * q > 1:
        inv = struct.unpack("<d", struct.pack("<q", struct.unpack("<q", struct.pack("<d", inv))[0] - 1))[0]
    return inv


def _mod_q_small(x, q, inv):
    k1 = (1 << 32) % q
    y = float(x >> 32) * float(k1) + float(x & U32)
    assert y == (x >> 32) * k1 + (x & U32)   # exact
    u = int(y - math.floor(y * inv) * q)
    assert 0 <= u < 2 * q                    # one fix-up is enough
    return min(u, (u - q) & U32)


def test_mod_q_small_one_fixup():
    rng = random.Random(23)
    for q in (3, 4099, 16411, 33457, 65537, 524309, 1048573, 8388593):
        inv = _inv_down(q)
        k1 = (1 << 32) % q
        ymax = MASK29 * k1 + U32
        for _ in range(4000):
            x = rng.randrange(M)
            assert _mod_q_small(x, q, inv) == x % q
        for _ in range(2000):   # y just below, at and above a multiple of q
            k = rng.randrange(1, ymax // q)
            for y in (k * q - 1, k * q, k * q + 1):
                if 0 <= y <= ymax:
                    u = int(y - math.floor(float(y) * inv) * q)
                    assert 0 <= u < 2 * q
