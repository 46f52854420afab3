#!/usr/bin/env python3
"""Per-phase breakdown of onepass16_kernel (profiling build, DG_LIB_VARIANT=prof).

usage: DG_LIB_VARIANT=prof python scripts/onepass_phases.py [--config c2] [--pairs N]
Prints per-pair averages of the kernel's phase counters and cycle totals.
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["epochs", "diag_calls", "diag_epochs", "diag_zero", "a_entries", "a_match", "b_entries",
         "b_chunks", "c_chunks", "extends", "refills", "t_diag", "t_a", "t_bc", "t_ext", "t_refill",
         "t_total", "b_walked", "t_d1_list", "t_d2_chain", "t_d3_fp_lookup", "t_d4_resolve", "d_members",
         "d_steps", "t_d3a_map", "t_d3ab_map_fp", "t_take", "t_resync", "takes", "resyncs", "t_final", "t_c", "t_b1_fp", "t_b2_upto_walk", "t_b3_walk"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--pairs", type=int, default=0)
    ap.add_argument("--offset", type=int, default=0, help="first pair's index in the config's batch")
    args = ap.parse_args()
    os.environ.setdefault("DG_LIB_VARIANT", "prof")
    import torch
    from bench import CONFIGS, load_product
    dg = load_product()
    L_ = dg.lib
    L_.dg_onepass_prof_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    L_.dg_onepass_prof_reset.argtypes = []
    ctx = dg.Context(0)
    from bench import OPTS, make_inputs
    npg, L, rate, q, seed = CONFIGS[args.config][:5]
    n = args.pairs or npg
    stream = torch.cuda.current_stream()
    ref, ver, layout = make_inputs(dg, ctx, torch, args.config, args.offset, n, stream)
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
    L_.dg_onepass_prof_reset()
    plan.set_timing(1)
    plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), offs.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * len(NAMES))()
    k = L_.dg_onepass_prof_read(buf, len(NAMES))
    vals = {NAMES[i]: buf[i] / n for i in range(k)}
    vals["stage_ms"] = plan.stage_times()
    if hasattr(L_, "dg_onepass_pair_prof_read"):
        import numpy as np
        m = min(n, 16384)
        pb = (C.c_ulonglong * (4 * m))()
        L_.dg_onepass_pair_prof_read(pb, m)
        a = np.frombuffer(pb, dtype=np.uint64).reshape(m, 4).astype(np.int64)
        t0 = a[:, 0].min()
        st_us, en_us = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0   # 100 MHz realtime
        dur = en_us - st_us
        order = np.argsort(-dur)[:8]
        vals["pair_us"] = {"span": float(en_us.max()), "dur_p50": float(np.median(dur)),
                           "dur_p99": float(np.percentile(dur, 99)), "dur_max": float(dur.max()),
                           "start_p50": float(np.median(st_us)), "start_max": float(st_us.max()),
                           "top": [[int(i), round(float(dur[i]), 1), round(float(st_us[i]), 1), int(a[i, 2]),
                                    int(a[i, 3])] for i in order]}
    vals["pairs"] = n
    print(json.dumps({k2: (round(v, 2) if isinstance(v, float) else v) for k2, v in vals.items()}))


if __name__ == "__main__":
    main()
