"""Member-mode onepass on data built to break the member checks.

The verified-members path (dg_members.hip) accepts a member only when
(A) no V window of a step equals an R window of another step of the member
and (B) the T step is the first writer of its slot in one of the tables
(onepass.c:141-219).  On random data both always hold, so the full-size C2/C3
batches cannot tell a weakened check from a correct one.  These pairs make
(A) and (B) fail often: periodic data (windows repeat at the period, inside
one member), low-entropy alphabets, and tiny table sizes (slot collisions).
Every delta is compared with the oracle; the chain mode runs the same pairs.
"""
import random

import pytest

pytestmark = pytest.mark.gpu

ONEPASS = 1


def _periodic(rng, n, period):
    unit = rng.randbytes(period)
    return (unit * (n // period + 1))[:n]


def _edit(rng, R, rate):
    """Substitutions by bytes drawn from R itself, so an edited V window can
    equal an R window elsewhere (a window holding a mismatch can only verify
    a lookup if it is byte-equal to one, onepass.c:186,212)."""
    V = bytearray(R)
    for _ in range(int(len(V) * rate)):
        V[rng.randrange(len(V))] = R[rng.randrange(len(R))]
    return bytes(V)


def _pairs(seed):
    rng = random.Random(seed)
    out = []
    for period in (17, 33, 64, 100, 250, 500, 1000):
        R = _periodic(rng, 65536 + rng.randrange(4096), period)
        out.append((f"periodic{period}", R, _edit(rng, R, rng.choice([0.002, 0.02, 0.1]))))
    for k in (2, 3, 4):
        R = bytes(rng.randrange(k) + 65 for _ in range(40000))
        for rate in (0.01, 0.05, 0.2):
            out.append((f"alphabet{k}_{rate}", R, _edit(rng, R, rate)))
    R = rng.randbytes(50000)
    # a block of V repeated from elsewhere in R at a short distance
    V = bytearray(_edit(rng, R, 0.05))
    for _ in range(20):
        a = rng.randrange(len(V) - 600)
        d = rng.randrange(1, 300)
        V[a:a + 200] = R[a + d:a + d + 200]
    out.append(("shifted_blocks", R, bytes(V)))
    return out


@pytest.mark.parametrize("q", [1, 7, 97])
def test_members_adversarial(dg, ctx_mode, orc, q):
    pairs = _pairs(100 + q)
    got = dg.encode_batch([(R, V) for _, R, V in pairs], "onepass", p=16, q=q, ctx=ctx_mode)
    for (name, R, V), d in zip(pairs, got):
        assert d == orc.encode(ONEPASS, R, V, p=16, q=q), name


def _sparse_pairs(seed):
    """Sparse edits placed around the end of a chunk's staged region
    (dg_members.hip: chunk c stages positions [2048 c - 16, 2048 c + 2288)):
    the chunk's last run then has no later run start staged, and its COPY
    runs to a mismatch found past the region -- just past it, several chunks
    later, at a stream end, or to an identical tail.  The search stops 16 KiB
    past the region (the member then stays unverified): k = 16383 / 16384 /
    16400 sit at that cap."""
    rng = random.Random(seed)
    out = []
    for k in (0, 1, 2, 15, 16, 17, 100, 700, 3000, 9000, 16383, 16384, 16400):
        L = 65536 + rng.randrange(2) * rng.randrange(1, 4096)
        R = rng.randbytes(L)
        V = bytearray(R)
        c = rng.randrange(4, 20)
        last = 2048 * c + rng.randrange(1900, 2048)        # the chunk's last mismatch
        V[last] ^= 0x5A
        if rng.random() < 0.5:
            V[last - rng.randrange(2, 15)] ^= 0x33       # a run of two
        nxt = 2048 * c + 2288 + k                         # first mismatch past the staged region
        if nxt < L:
            V[nxt] ^= 0xA5
        out.append((f"sparse_{k}", R, bytes(V)))
    R = rng.randbytes(70000)
    V = bytearray(R)
    V[2048 * 9 + 2000] ^= 1                                # then identical to the end
    out.append(("identical_tail", R, bytes(V)))
    V2 = bytearray(R[:2048 * 9 + 2040]) + bytes([R[2048 * 9 + 2040] ^ 1])   # V ends inside the look-ahead
    out.append(("short_v", R, bytes(V2)))
    # 1 MiB, 0.1 % edits: most chunks end on such a member
    R = rng.randbytes(1 << 20)
    V = bytearray(R)
    for _ in range(1000):
        V[rng.randrange(len(V))] ^= 1 + rng.randrange(255)
    out.append(("mib_sparse", R, bytes(V)))
    return out


@pytest.mark.parametrize("q", [1, 97])
def test_members_sparse_chunk_ends(dg, ctx_mode, orc, q):
    pairs = _sparse_pairs(7 + q)
    got = dg.encode_batch([(R, V) for _, R, V in pairs], "onepass", p=16, q=q, ctx=ctx_mode)
    for (name, R, V), d in zip(pairs, got):
        assert d == orc.encode(ONEPASS, R, V, p=16, q=q), name
        assert dg.decode(R, d, ctx=ctx_mode) == V, name


def _sparse_runs(seed):
    """Pairs whose deltas are a few percent of V (a sparse batch for the
    member serialiser).  Edits are runs of 1..300 bytes, so the payloads take
    every copy path (the 4-byte head, 4-byte words, 16-byte pieces, the
    wave-wide copy), some ending right before a chunk or stream boundary."""
    rng = random.Random(seed)
    out = []
    for i in range(12):
        L = 262144 + rng.randrange(3) * rng.randrange(1, 9000)
        R = rng.randbytes(L)
        V = bytearray(R)
        for _ in range(24):
            n = rng.choice((1, 3, 5, 9, 15, 17, 31, 64, 65, 120, 300))
            at = rng.randrange(0, L - n - 40)
            if rng.random() < 0.2:
                at = 2048 * rng.randrange(1, L // 2048 - 1) - n   # ending at a chunk boundary
            for k in range(n):
                V[at + k] ^= 1 + rng.randrange(255)
        out.append((f"runs_{i}", R, bytes(V)))
    return out


@pytest.mark.parametrize("q", [1, 97])
def test_members_sparse_payload_runs(dg, ctx_mode, orc, q):
    pairs = _sparse_runs(11 + q)
    got = dg.encode_batch([(R, V) for _, R, V in pairs], "onepass", p=16, q=q, ctx=ctx_mode)
    total = sum(len(d) for d in got)
    assert total * 8 < sum(len(V) for _, _, V in pairs)   # a sparse batch
    for (name, R, V), d in zip(pairs, got):
        assert d == orc.encode(ONEPASS, R, V, p=16, q=q), name
        assert dg.decode(R, d, ctx=ctx_mode) == V, name
