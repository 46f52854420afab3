#!/usr/bin/env python3
"""Regenerate tests/golden/golden.json from the REFERENCE itself.

The reference's tests hold no golden delta bytes (encoder
output is pinned only by cross-implementation byte identity), so the fixtures
are minted here by running the reference's own src/c, compiled from
/root/reference/src/c by oracle/Makefile (oracle/_ref/libdelta_ref.so,
`ref_encode_pair` = the main.c:257-292 chain).  Run in the dev container:

    make -C oracle ref && python tests/golden/make_golden.py

Stored per case: inputs as sha256 (+ the generator spec, see tests/cases.py
and DESIGN.md "Synthetic inputs"), the delta bytes (hex) when short, else
sha256 + length, and the two CRCs.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(HERE))

import oracle as O  # noqa: E402
from cases import small_cases  # noqa: E402

INLINE_MAX = 2048


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def entry(ref, algo, R, V, p, q, **extra):
    d = ref.encode(algo, R, V, p=p, q=q)
    e = {"algo": algo, "p": p, "q": q, "r_sha256": sha(R), "v_sha256": sha(V),
         "r_len": len(R), "v_len": len(V), "delta_len": len(d), "delta_sha256": sha(d),
         "src_crc": d[9:17].hex(), "dst_crc": d[17:25].hex()}
    if len(d) <= INLINE_MAX:
        e["delta_hex"] = d.hex()
    e.update(extra)
    return e


def main():
    ref = O.Reference()
    orc = O.Oracle()
    out = {"generator": "reference src/c via oracle/_ref (ref_encode_pair)",
           "crc_kat": {"123456789": "995dc9bbdf1939fa", "": "0000000000000000"},
           "cases": []}
    for name, R, V, p, q in small_cases():
        for algo in (O.ONEPASS, O.CORRECTING):
            if algo == O.CORRECTING and len(V) >= p and len(V) // 2 + p > len(V):
                continue  # reference reads past |V| here (correcting.c:133-136): undefined
            out["cases"].append(dict(name=name, kind="small", **entry(ref, algo, R, V, p, q)))
    # synthetic workloads: first pairs of each config (DESIGN.md "Synthetic inputs")
    synth = [
        ("c2", 0xC2000000, 65536, 655, 1, 8),
        ("c2_default_q", 0xC2000000, 65536, 655, 1048573, 2),
        ("c3", 0xC3000000, 262144, 26214, 1, 4),
        # the north star's upper pair size: 1 MiB, 1 %, q = next_prime(65536) = 65537
        ("c6", 0xC6000000, 1048576, 10486, 1, 4),
        ("c6_default_q", 0xC6000000, 1048576, 10486, 1048573, 1),
    ]
    for tag, seed, L, ne, q, count in synth:
        for i in range(count):
            R, V = orc.synth_pair(seed + i, L, ne)
            out["cases"].append(dict(name=f"{tag}_{i}", kind="synth_edits", seed=seed + i,
                                     pair_len=L, n_edits=ne, **entry(ref, O.ONEPASS, R, V, 16, q)))
    for i in range(4):
        nb = 8 + (i % 57)
        R, V = orc.synth_transpose(0xC4000000 + i, nb, 262144 // nb, 50)
        out["cases"].append(dict(name=f"c4_{i}", kind="synth_transpose", seed=0xC4000000 + i,
                                 num_blocks=nb, mean=262144 // nb, pct=50,
                                 **entry(ref, O.CORRECTING, R, V, 16, 1)))
        out["cases"].append(dict(name=f"c4_onepass_{i}", kind="synth_transpose", seed=0xC4000000 + i,
                                 num_blocks=nb, mean=262144 // nb, pct=50,
                                 **entry(ref, O.ONEPASS, R, V, 16, 1)))
    for i in range(3):   # shift pairs (C3s): edits that move the diagonal
        R, V = orc.synth_shift(0xC3500000 + i, 262144, 26214, 67)
        out["cases"].append(dict(name=f"c3s_{i}", kind="synth_shift", seed=0xC3500000 + i, pair_len=262144,
                                 n_edits=26214, indel_pct=67, **entry(ref, O.ONEPASS, R, V, 16, 1)))
    for i, pct in enumerate((5, 100)):   # sparse and indel-only mixes, smaller pairs
        R, V = orc.synth_shift(0xC3510000 + i, 65536, 300, pct)
        for algo in (O.ONEPASS, O.CORRECTING):
            out["cases"].append(dict(name=f"shift_{pct}_{algo}", kind="synth_shift", seed=0xC3510000 + i,
                                     pair_len=65536, n_edits=300, indel_pct=pct, **entry(ref, algo, R, V, 16, 1)))
    R = orc.synth_random(1, 1 << 20)
    V = orc.synth_random(2, 1 << 20)
    out["cases"].append(dict(name="c1_random_1MiB", kind="synth_random", r_seed=1, v_seed=2,
                             **entry(ref, O.ONEPASS, R, V, 16, 1048573)))
    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(out['cases'])} cases to {path}")
    make_inplace(ref, orc)


def make_inplace(ref, orc):
    """In-place deltas (main.c encode --inplace: delta_make_inplace +
    delta_encode(inplace=true)) with their bytes inline, so the decode tests
    can replay them on the GPU box where the reference is absent."""
    out = {"generator": "reference src/c via oracle/_ref (ref_encode_pair_inplace)", "cases": []}

    def add(name, algo, R, V, q, policy, **extra):
        d = ref.encode_inplace(algo, R, V, p=16, q=q, policy=policy)
        out["cases"].append(dict(name=name, algo=algo, q=q, policy=policy, r_sha256=sha(R),
                                 v_sha256=sha(V), r_len=len(R), v_len=len(V),
                                 delta_len=len(d), delta_hex=d.hex(), **extra))

    for name, R, V, p, q in small_cases():
        if p != 16:
            continue
        for policy in (0, 1):
            add(f"{name}_pol{policy}", O.ONEPASS, R, V, q, policy, kind="small")
    for i in range(4):
        R, V = orc.synth_pair(0xC2000000 + i, 65536, 655)
        add(f"c2_{i}", O.ONEPASS, R, V, 1, i & 1, kind="synth_edits", seed=0xC2000000 + i,
            pair_len=65536, n_edits=655)
    # shifted content: blocks move both ways, so the CRWI graph has cycles
    for i in range(2):
        nb = 8 + i
        R, V = orc.synth_transpose(0xC4000000 + i, nb, 65536 // nb, 50)
        for policy in (0, 1):
            add(f"transpose_{i}_pol{policy}", O.CORRECTING, R, V, 1, policy,
                kind="synth_transpose", seed=0xC4000000 + i, num_blocks=nb, mean=65536 // nb, pct=50)
    path = os.path.join(HERE, "golden_inplace.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print(f"wrote {len(out['cases'])} in-place cases to {path}")


if __name__ == "__main__":
    main()
