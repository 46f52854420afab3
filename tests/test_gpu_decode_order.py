"""In-place decode ordering on the device (apply.c:253-284).

decode_kernel applies a 4 KiB window of commands with all four waves at once
when the window is order-free: the commands that write (every ADD, every COPY
except an in-place one with src == dst, which memmoves a range onto itself)
have increasing, disjoint destinations, and no in-place COPY moves.  The
in-place format lists the COPYs first and the ADDs after them
(inplace.c:711-725), so C5's windows interleave no-op COPYs with ADDs whose
destinations restart below the COPYs' ends.  These cases build in-place
command lists that are and are not order-free (ADDs out of order, ADDs that
overwrite each other inside one batch of 64 and across batches, moving
COPYs, zero-length commands, ADDs inside no-op COPY ranges, many windows) and
check the device against the oracle's sequential replay.
"""
import random

import pytest

pytestmark = pytest.mark.gpu


def _delta(dg, orc, R, cmds, vsize):
    """In-place delta of `cmds` with the CRCs the oracle's replay implies."""
    z = b"\0" * 8
    d0 = dg.encode_delta(cmds, inplace=True, version_size=vsize, src_crc=z, dst_crc=z)
    rc, V = orc.decode(R, d0, ignore_hash=True)
    assert rc == 0
    d = dg.encode_delta(cmds, inplace=True, version_size=vsize, src_crc=orc.crc64_xz(R),
                        dst_crc=orc.crc64_xz(V))
    return d, V


def _case(dg, rng, kind, n_r=20000, n_cmds=1500):
    R = rng.randbytes(n_r)
    vsize = n_r if kind != "grow" else n_r + 3000
    cap = max(n_r, vsize)
    cmds = []
    # COPYs first (no-ops on the diagonal, some moving), then ADDs
    pos = 0
    while pos < n_r and len(cmds) < n_cmds // 2:
        ln = rng.randint(1, 40)
        if pos + ln > n_r:
            break
        if kind == "moving" and rng.random() < 0.02:
            src = rng.randrange(0, n_r - ln)
            cmds.append(dg.PlacedCopy(src=src, dst=pos, length=ln))
        elif kind == "zero" and rng.random() < 0.05:
            cmds.append(dg.PlacedCopy(src=pos, dst=pos, length=0))
        else:
            cmds.append(dg.PlacedCopy(src=pos, dst=pos, length=ln))
        pos += ln + rng.randint(0, 12)
    adds = []
    p = 0
    while p < cap - 64 and len(adds) < n_cmds // 2:
        ln = rng.randint(1, 24)
        adds.append((p, ln))
        p += ln + rng.randint(0, 30)
    if kind == "reversed":
        adds.reverse()
    elif kind == "overlap_batch":   # an ADD overwriting the one 5 commands before
        for k in range(10, len(adds), 97):
            d0, _ = adds[k - 5]
            adds[k] = (d0 + 1, 8)
    elif kind == "overlap_cross":   # an ADD overwriting one ~200 commands earlier
        for k in range(300, len(adds), 211):
            d0, _ = adds[k - 200]
            adds[k] = (d0, 4)
    elif kind == "shuffled_tail":   # victim-style ADDs appended out of order
        tail = [(rng.randrange(0, cap - 64), rng.randint(1, 40)) for _ in range(40)]
        adds += tail
    for d0, ln in adds:
        if kind == "zero" and rng.random() < 0.05:
            ln = 0
        cmds.append(dg.PlacedAdd(dst=d0, data=rng.randbytes(ln)))
    return R, cmds, vsize


KINDS = ["c5_shape", "reversed", "overlap_batch", "overlap_cross", "shuffled_tail", "moving", "zero", "grow"]


@pytest.mark.parametrize("kind", KINDS)
def test_inplace_order_cases(dg, ctx, orc, kind):
    rng = random.Random(1000 + KINDS.index(kind))
    for _ in range(3):
        R, cmds, vsize = _case(dg, rng, kind)
        d, V = _delta(dg, orc, R, cmds, vsize)
        assert len(d) > 3 * 4096   # several windows of the command stream
        assert dg.decode(R, d, ctx=ctx) == V, kind


def test_inplace_order_small_windows(dg, ctx, orc):
    """Short streams (one partial window) of each kind, many seeds."""
    rng = random.Random(7)
    for it in range(60):
        kind = KINDS[it % len(KINDS)]
        R, cmds, vsize = _case(dg, rng, kind, n_r=3000, n_cmds=rng.randint(2, 200))
        d, V = _delta(dg, orc, R, cmds, vsize)
        assert dg.decode(R, d, ctx=ctx) == V, (kind, it)


def _moves_case(dg, rng, kind, n=24000):
    """In-place command lists whose COPYs move: block rotations (a chain in
    which every COPY overwrites the bytes the previous one read), whole-buffer
    shifts (one COPY onto an overlapping range: a real memmove, forward and
    backward), and blocks swapped through an ADD (a broken cycle)."""
    R = rng.randbytes(n)
    cmds = []
    if kind == "rotate":
        bs = rng.choice([16, 100, 1000, 4096])
        nb = n // bs
        for b in range(nb - 1):   # V[b] = R[b + 1]: read before it is overwritten
            cmds.append(dg.PlacedCopy(src=(b + 1) * bs, dst=b * bs, length=bs))
        cmds.append(dg.PlacedAdd(dst=(nb - 1) * bs, data=R[:bs]))
        return R, cmds, nb * bs
    if kind in ("shift_fwd", "shift_back"):
        k = rng.choice([1, 7, 15, 16, 17, 300, 5000])
        if kind == "shift_fwd":   # V = R[k:] + tail: dst < src, overlapping
            cmds.append(dg.PlacedCopy(src=k, dst=0, length=n - k))
            cmds.append(dg.PlacedAdd(dst=n - k, data=rng.randbytes(k)))
        else:                     # V = head + R[:-k]: dst > src, overlapping
            cmds.append(dg.PlacedCopy(src=0, dst=k, length=n - k))
            cmds.append(dg.PlacedAdd(dst=0, data=rng.randbytes(k)))
        return R, cmds, n
    # "mixed": short moving COPYs in a valid order (each reads bytes no earlier
    # command wrote), some self-overlapping, no-op COPYs and ADDs between them
    written = bytearray(n)
    pos = 0
    while pos < n - 64:
        ln = rng.randint(1, 600)
        if pos + ln > n:
            break
        r = rng.random()
        if r < 0.3:
            cmds.append(dg.PlacedCopy(src=pos, dst=pos, length=ln))
        elif r < 0.8:
            for _ in range(20):
                src = rng.randrange(0, n - ln)
                if not any(written[src:src + ln]):
                    cmds.append(dg.PlacedCopy(src=src, dst=pos, length=ln))
                    break
        else:
            cmds.append(dg.PlacedAdd(dst=pos, data=rng.randbytes(ln)))
        written[pos:pos + ln] = b"\1" * ln
        pos += ln
    return R, cmds, n


MOVE_KINDS = ["rotate", "shift_fwd", "shift_back", "mixed"]


@pytest.mark.parametrize("kind", MOVE_KINDS)
def test_inplace_moving_copies(dg, ctx, orc, kind):
    """Windows that are not order-free go through the conflict-free groups
    (a chain of dependent COPYs, single COPYs onto overlapping ranges, mixed
    short moves): the device equals the oracle's sequential memmove replay."""
    rng = random.Random(2000 + MOVE_KINDS.index(kind))
    for _ in range(6):
        R, cmds, vsize = _moves_case(dg, rng, kind)
        d, V = _delta(dg, orc, R, cmds, vsize)
        assert dg.decode(R, d, ctx=ctx) == V, kind


@pytest.mark.parametrize("policy", ["localmin", "constant"])
def test_inplace_transposition_deltas(dg, ctx, orc, policy):
    """Real in-place deltas with moving COPYs: correcting deltas of block
    transpositions (gen_transpositions.py recipe) converted by dg_make_inplace,
    decoded on the device against V and against the oracle's replay."""
    for i in range(24):
        nb = 8 + (i * 7) % 57
        R, V = orc.synth_transpose(0xC5000000 + i, nb, 65536 // nb, 50)
        std = orc.encode(2, R, V, p=16, q=1)
        d = dg.make_inplace(R, std, policy=policy)
        assert d[4] == 1
        rc, Vo = orc.decode(R, d)
        assert rc == 0 and Vo == V
        assert dg.decode(R, d, ctx=ctx) == V, (i, policy)
