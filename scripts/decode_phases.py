#!/usr/bin/env python3
"""Per-phase cycles of decode_kernel (profiling build, DG_LIB_VARIANT=prof).

usage: DG_LIB_VARIANT=prof python scripts/decode_phases.py [--pairs N]
Encodes C2 pairs on the device, then decodes them once with the phase
counters on; prints per-stream averages (shader cycles, s_memtime).
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["fill", "win_load", "n1", "doubling", "walk", "expand", "hdr+checks", "copy", "final_wait",
         "windows", "batches", "total", "ordered_windows", "c_cmd", "c_flat", "c_barrier", "crc_sync", "crc_seg",
         "crc_tail"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--inplace", action="store_true", help="C5: convert with make_inplace(localmin)")
    args = ap.parse_args()
    os.environ.setdefault("DG_LIB_VARIANT", "prof")
    import torch
    from bench import load_product
    dg = load_product()
    L_ = dg.lib
    L_.dg_decode_prof_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    L_.dg_decode_prof_reset.argtypes = []
    ctx = dg.Context(0)
    n, L = args.pairs, 65536
    ref = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    ver = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    ctx.check(L_.dg_synth_edit_pairs_device(ctx.handle, ref.data_ptr(), ver.data_ptr(), n, L, 0xC2000000,
                                            655, None), "synth")
    layout = [(i * L, L, i * L, L) for i in range(n)]
    enc = dg.EncodePlan(ctx, "onepass", layout, q=1)
    d_arena = torch.empty(enc.output_bound, dtype=torch.uint8, device="cuda")
    offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    est = torch.empty(n, dtype=torch.int32, device="cuda")
    enc.run(ref.data_ptr(), ver.data_ptr(), d_arena.data_ptr(), d_arena.numel(), offs.data_ptr(),
            est.data_ptr(), None)
    torch.cuda.synchronize()
    o = offs.cpu().tolist()
    if args.inplace:   # the C5 workload (bench.py bench_decode)
        std = d_arena[:o[-1]].cpu().numpy().tobytes()
        ref_h = ref.cpu().numpy().tobytes()
        ds = [dg.make_inplace(ref_h[i * L:(i + 1) * L], std[o[i]:o[i + 1]], policy="localmin") for i in range(n)]
        o = [0]
        for d in ds:
            o.append(o[-1] + len(d))
        d_arena = torch.frombuffer(bytearray(b"".join(ds)), dtype=torch.uint8).to("cuda")
    plan = dg.DecodePlan(ctx, [(r, rl, o[i], o[i + 1] - o[i], v, vl) for i, (r, rl, v, vl) in enumerate(layout)])
    out = torch.empty_like(ver)
    olen = torch.empty(n, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    plan.run(ref.data_ptr(), d_arena.data_ptr(), out.data_ptr(), olen.data_ptr(), st.data_ptr(), None)
    torch.cuda.synchronize()
    L_.dg_decode_prof_reset()
    plan.set_timing(1)
    plan.run(ref.data_ptr(), d_arena.data_ptr(), out.data_ptr(), olen.data_ptr(), st.data_ptr(), None)
    torch.cuda.synchronize()
    assert int(st.abs().sum()) == 0 and torch.equal(out, ver)
    buf = (C.c_ulonglong * len(NAMES))()
    k = L_.dg_decode_prof_read(buf, len(NAMES))
    vals = {NAMES[i]: round(buf[i] / n, 1) for i in range(k)}
    vals["stage_ms"] = plan.stage_times()
    print(json.dumps(vals))


if __name__ == "__main__":
    main()
