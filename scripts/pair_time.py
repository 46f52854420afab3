#!/usr/bin/env python3
"""Per-pair duration and placement of onepass16_kernel (variant build DG_LIB_VARIANT=pairtime,
-DDG_PAIR_TIME): start/end by s_memrealtime (100 MHz) and HW_ID / XCC_ID of each pair's wave.
usage: DG_LIB_VARIANT=pairtime python scripts/pair_time.py [--config c2]"""
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
npg, L, rate, q, seed = CONFIGS[args.config][:5]
n = npg
ref = torch.empty(n * L, dtype=torch.uint8, device="cuda")
ver = torch.empty(n * L, dtype=torch.uint8, device="cuda")
ctx.check(L_.dg_synth_edit_pairs_device(ctx.handle, ref.data_ptr(), ver.data_ptr(), n, L, seed, int(rate * L + 0.5), None), "synth")
plan = dg.EncodePlan(ctx, "onepass", [(i * L, L, i * L, L) for i in range(n)], q=q)
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
         "dur_by_pair_quartile": [round(float(dur[i * n // 4:(i + 1) * n // 4].mean()), 1) for i in range(4)],
         "slowest": [[int(i), round(float(dur[i]), 1), int(xcc[i]), int(se[i]), int(cu[i]), int(simd[i])] for i in np.argsort(-dur)[:6]]}
    res.append(r)
print(json.dumps(res))
