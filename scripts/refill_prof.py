#!/usr/bin/env python3
"""Refill-wait share of onepass16 (variant build DG_LIB_VARIANT=refill, -DDG_REFILL_PROF).
usage: DG_LIB_VARIANT=refill python scripts/refill_prof.py [--config c2] [--serial]"""
import argparse, ctypes as C, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2")
args = ap.parse_args()
os.environ.setdefault("DG_LIB_VARIANT", "refill")
import torch
from bench import CONFIGS, load_product
dg = load_product()
L_ = dg.lib
L_.dg_refill_prof_read.argtypes = [C.POINTER(C.c_ulonglong)]
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
for _ in range(2):
    plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), offs.data_ptr(), st.data_ptr())
torch.cuda.synchronize()
L_.dg_refill_prof_reset()
plan.set_timing(1)
plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), offs.data_ptr(), st.data_ptr())
torch.cuda.synchronize()
b = (C.c_ulonglong * 3)()
L_.dg_refill_prof_read(b)
print(json.dumps({"config": args.config, "serial_crc": os.environ.get("DG_SERIAL_CRC", "0"),
                  "refill_wait_cycles_per_pair": b[0] / n, "refills_per_pair": b[1] / n,
                  "pair_cycles": b[2] / n, "refill_share": b[0] / max(b[2], 1), "stage_ms": plan.stage_times()}))
