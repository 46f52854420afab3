#!/usr/bin/env python3
"""Per-pair duration and placement of onepass16_kernel (variant build DG_LIB_VARIANT=pairtime,
-DDG_PAIR_TIME): start/end by s_memrealtime (100 MHz) and HW_ID / XCC_ID of each pair's wave.
usage: DG_LIB_VARIANT=pairtime python scripts/pair_time.py [--config c2]
(any encode config of bench.py: its generator and chain mode)"""
import argparse, ctypes as C, json, os, sys
import collections
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
args = ap.parse_args()
os.environ.setdefault("DG_LIB_VARIANT", "pairtime")
import numpy as np
import torch
from bench import CONFIGS, load_product
dg = load_product()
L_ = dg.lib
L_.dg_pair_time_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
ctx = dg.Context(0)
from bench import OPTS, make_inputs
npg, L, rate, q, seed = CONFIGS[args.config][:5]
n = npg
stream = torch.cuda.current_stream()
ref, ver, layout = make_inputs(dg, ctx, torch, args.config, 0, n, stream)
torch.cuda.synchronize()
members = OPTS.get(args.config, {}).get("members")
if members is not None:
    ctx.set_limit(dg.LIMIT_ONEPASS_MEMBERS, members)
plan = dg.EncodePlan(ctx, "onepass", layout, q=q)
out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
st = torch.empty(n, dtype=torch.int32, device="cuda")
res = []
for rep in range(6):
    plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), offs.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    if rep < 3:
        continue
    m = min(n, 16384)
    buf = (C.c_ulonglong * (3 * m))()
    L_.dg_pair_time_read(buf, m)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(m, 3).astype(np.int64)
    t0 = a[:, 0].min()
    start = (a[:, 0] - t0) / 100.0
    end = (a[:, 1] - t0) / 100.0
    dur = end - start
    hw = a[:, 2] & 0xFFFFFFFF
    xcc = a[:, 2] >> 32
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    key = xcc * 1000 + se * 100 + cu * 10 + simd   # one SIMD
    per_simd = collections.Counter(key.tolist())
    occ = np.array([per_simd[k] for k in key.tolist()])
    r = {"span_us": float(end.max()), "dur_p10": float(np.percentile(dur, 10)), "dur_p50": float(np.median(dur)),
         "dur_p90": float(np.percentile(dur, 90)), "dur_max": float(dur.max()), "start_max": float(start.max()),
         "simds": len(per_simd), "waves_per_simd_hist": dict(collections.Counter(per_simd.values())),
         "dur_by_waves_on_simd": {int(w): round(float(dur[occ == w].mean()), 1) for w in sorted(set(occ.tolist()))},
         "start_hist_ms": np.histogram(start / 1000.0, bins=12)[0].tolist(),
         "start_edges_ms": [round(float(x), 2) for x in np.histogram(start / 1000.0, bins=12)[1]],
         "end_p50_ms": float(np.median(end)) / 1000.0, "dur_by_start_bin_us": [round(float(dur[(start >= lo_) & (start < lo_ + (start.max() + 1) / 6)].mean()), 1) for lo_ in np.linspace(0, start.max() + 1, 7)[:6]],
         "dur_by_pair_quartile": [round(float(dur[i * n // 4:(i + 1) * n // 4].mean()), 1) for i in range(4)],
         "slowest": [[int(i), round(float(dur[i]), 1), int(xcc[i]), int(se[i]), int(cu[i]), int(simd[i])] for i in np.argsort(-dur)[:6]]}
    res.append(r)
print(json.dumps(res))
