"""The automatic chain mode on large pairs whose matches leave diagonal 0.

A member plan (mean pair >= 128 KiB) routes a pair whose chunks verify fewer
than 2 diagonal members each to the plain chain (dg_onepass.hip,
onepass16_kernel<false, true>), inside the same plan as the member pairs.
Every delta is compared with the oracle: dense and sparse insertions and
deletions, unrelated streams, a random stretch inside a shifted pair, moved
blocks, a large insertion, V much shorter or longer than R, lengths around
the member chunk size, an unrelated first chunk before a diagonal rest.
"""
import random

import pytest

pytestmark = pytest.mark.gpu

ONEPASS = 1


def _shifted(rng, R, n_edits, indel_max):
    V = bytearray()
    pos = 0
    cuts = sorted(rng.sample(range(1, len(R) - 1), n_edits))
    for c in cuts:
        V += R[pos:c]
        u = rng.random()
        k = rng.randint(1, indel_max)
        if u < 0.33:
            V += rng.randbytes(k)          # insertion
            pos = c
        elif u < 0.66:
            pos = min(len(R), c + k)       # deletion
        else:
            V += bytes([rng.randrange(256)])
            pos = c + 1
    V += R[pos:]
    return bytes(V)


def _pairs(seed):
    rng = random.Random(seed)
    out = []
    for L in (65536, 98304, 131071, 262144):
        R = rng.randbytes(L)
        out.append((f"shift_dense_{L}", R, _shifted(rng, R, L // 12, 8)))
        R = rng.randbytes(L)
        out.append((f"shift_sparse_{L}", R, _shifted(rng, R, L // 900, 40)))
    R = rng.randbytes(200000)
    out.append(("unrelated", R, rng.randbytes(190000)))
    R = rng.randbytes(200000)
    V = bytearray(_shifted(rng, R, 2000, 8))
    V[70000:110000] = rng.randbytes(40000)                # a random stretch across pieces
    out.append(("random_stretch", R, bytes(V)))
    R = rng.randbytes(180000)
    blocks = [R[i:i + 9000] for i in range(0, len(R), 9000)]
    rng.shuffle(blocks)
    out.append(("moved_blocks", R, b"".join(blocks)))
    R = rng.randbytes(150000)
    out.append(("big_insert", R, R[:30000] + rng.randbytes(20000) + R[30000:]))
    # chunk 0 unrelated, the rest diagonal (1 % substitutions): the member
    # kernel skips the pair's later chunks once chunk 0 verified too few
    R = rng.randbytes(200000)
    V = bytearray(R)
    for k in rng.sample(range(3000, len(V)), len(V) // 100):
        V[k] = rng.randrange(256)
    V[:3000] = rng.randbytes(3000)
    out.append(("bad_head", R, bytes(V)))
    R = rng.randbytes(160000)
    out.append(("v_shorter", R, _shifted(rng, R[:70000], 500, 8)))
    R = rng.randbytes(70000)
    out.append(("r_shorter", R, _shifted(rng, R + R[:90000], 700, 8)))
    return out


@pytest.mark.parametrize("q", [1, 97])
def test_auto_mode_offdiagonal_vs_oracle(dg, orc, q):
    ctx = dg.Context(0)   # automatic mode
    try:
        pairs = _pairs(1234 + q)
        got = dg.encode_batch([(R, V) for _, R, V in pairs], "onepass", p=16, q=q, ctx=ctx)
        for (name, R, V), d in zip(pairs, got):
            assert d == orc.encode(ONEPASS, R, V, p=16, q=q), name
            assert dg.decode(R, d, ctx=ctx) == V, name
    finally:
        ctx.close()
