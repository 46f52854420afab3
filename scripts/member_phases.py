#!/usr/bin/env python3
"""Per-phase breakdown of member_chunk_kernel (profiling build, DG_LIB_VARIANT=prof).

usage: DG_LIB_VARIANT=prof python scripts/member_phases.py [--config c3] [--pairs N]
Prints per-chunk averages of the kernel's phase cycles (shader clock,
s_memtime, issue-to-issue: a phase absorbs the waits of loads issued before
it) and counts, with each phase's share of the total.
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["stage", "mask", "runs", "sn_last", "setup", "short", "long", "prefix", "total", "chunks",
         "members", "short_n", "long_n", "rounds", "unverified", "flagged", "d1_rounds"]
PHASES = NAMES[:8]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--pairs", type=int, default=0)
    args = ap.parse_args()
    os.environ.setdefault("DG_LIB_VARIANT", "prof")
    import torch
    from bench import CONFIGS, OPTS, load_product, make_inputs
    dg = load_product()
    L_ = dg.lib
    L_.dg_member_prof_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    L_.dg_member_prof_reset.argtypes = []
    ctx = dg.Context(0)
    npg, L, rate, q, seed = CONFIGS[args.config][:5]
    n = args.pairs or npg
    stream = torch.cuda.current_stream()
    ref, ver, layout = make_inputs(dg, ctx, torch, args.config, 0, n, stream)
    members = OPTS.get(args.config, {}).get("members")
    if members is not None:
        ctx.set_limit(dg.LIMIT_ONEPASS_MEMBERS, members)
    plan = dg.EncodePlan(ctx, "onepass", layout, q=q)
    out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
    offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), offs.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    L_.dg_member_prof_reset()
    plan.set_timing(1)
    plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), offs.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * len(NAMES))()
    k = L_.dg_member_prof_read(buf, len(NAMES))
    raw = {NAMES[i]: buf[i] for i in range(k)}
    ch = max(raw.get("chunks", 1), 1)
    per = {k2: round(v / ch, 2) for k2, v in raw.items()}
    tot = max(raw.get("total", 1), 1)
    share = {p: round(raw[p] / tot, 4) for p in PHASES if p in raw}
    print(json.dumps({"config": args.config, "pairs": n, "per_chunk": per, "share_of_total": share,
                      "stage_ms": plan.stage_times()}))


if __name__ == "__main__":
    main()
