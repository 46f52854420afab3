"""The wave-per-pair serialiser's tiles (dg_serialize_wave.h serialize_run).

A pair's COPY records are written 64 per tile.  A tile whose bytes fit the
4 KiB LDS stage is flushed with a fixed number of buffer stores, and the next
tile's records are loaded before those stores and waited for by hand
(vmcnt(kTileStores)); a tile over the stage is written straight to HBM and
drains its stores (vmcnt(0)).  These pairs put record counts on and around
tile boundaries, mix staged and direct tiles in one pair, and use every ADD
payload path (the 4-byte head in the record, dword loads up to 32 bytes, the
wave-wide copy), in both the plain-chain and the member serialiser.  Every
delta is compared with the oracle and decoded back.
"""
import random

import pytest

pytestmark = pytest.mark.gpu

ONEPASS = 1


def _pair(rng, n_copies, ins_lens):
    """V = n_copies pieces of R (40 bytes each, from scattered offsets), each
    followed by an insertion whose length cycles through ins_lens."""
    R = rng.randbytes(1 << 16)
    V = bytearray()
    for k in range(n_copies):
        at = rng.randrange(0, len(R) - 64)
        V += R[at:at + 40]
        V += rng.randbytes(ins_lens[k % len(ins_lens)])
    return R, bytes(V)


def _cases(seed):
    rng = random.Random(seed)
    out = []
    for n in (1, 63, 64, 65, 127, 128, 129, 200):
        out.append((f"records_{n}", *_pair(rng, n, [1, 3, 4])))                 # inline heads only
        out.append((f"records_{n}_mixed", *_pair(rng, n, [2, 7, 17, 32, 33, 90])))
    # tiles over the stage between staged ones: a 5000-byte insertion every
    # 70 pieces pushes that tile past 4 KiB
    lens = [5] * 69 + [5000]
    out.append(("direct_tiles", *_pair(rng, 300, lens)))
    out.append(("all_direct", *_pair(rng, 130, [3000])))
    R = rng.randbytes(5000)
    out.append(("no_records", R, rng.randbytes(7000)))
    return out


@pytest.mark.parametrize("seed", [1, 2])
def test_serializer_tiles(dg, ctx_mode, orc, seed):
    cases = _cases(seed)
    got = dg.encode_batch([(R, V) for _, R, V in cases], "onepass", p=16, q=1, ctx=ctx_mode)
    for (name, R, V), d in zip(cases, got):
        assert d == orc.encode(ONEPASS, R, V, p=16, q=1), name
        assert dg.decode(R, d, ctx=ctx_mode) == V, name
