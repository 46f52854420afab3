#!/usr/bin/env python3
"""Host-to-host (PCIe-inclusive) onepass encode rate, for DESIGN.md.

The C2 workload, but the pairs start in pinned host memory and the packed
deltas end in pinned host memory: chunks of pairs are double-buffered over two
HIP streams (H2D of R and V -> dg_encode_plan_run -> D2H of the offsets, then
D2H of exactly the delta bytes once the offsets are known).  Reports
sum(|R|+|V|) / wall time of the whole pipeline.  This is NOT bench.py's
`value` (which is device-resident by the metric's definition).

usage: python scripts/bench_e2e.py [--pairs 16384] [--chunk 2048] [--reps 3]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=16384)
    ap.add_argument("--chunk", type=int, default=2048)
    ap.add_argument("--len", type=int, default=65536)
    ap.add_argument("--edit-rate", type=float, default=0.01)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()

    import torch
    from bench import load_product

    dg = load_product()
    ctx = dg.Context(0)
    L, n, ch = args.len, args.pairs, args.chunk
    assert n % ch == 0
    n_chunks = n // ch
    n_edits = int(args.edit_rate * L + 0.5)

    # host-resident inputs (generated on the device once, untimed)
    h_ref = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    h_ver = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    tmp_r = torch.empty(ch * L, dtype=torch.uint8, device="cuda")
    tmp_v = torch.empty(ch * L, dtype=torch.uint8, device="cuda")
    for c in range(n_chunks):
        ctx.check(dg.lib.dg_synth_edit_pairs_device(ctx.handle, tmp_r.data_ptr(), tmp_v.data_ptr(), ch, L,
                                                    0xC2000000 + c * ch, n_edits, None), "synth")
        torch.cuda.synchronize()
        h_ref[c * ch * L:(c + 1) * ch * L].copy_(tmp_r)
        h_ver[c * ch * L:(c + 1) * ch * L].copy_(tmp_v)
    del tmp_r, tmp_v

    layout = [(i * L, L, i * L, L) for i in range(ch)]
    slots = []
    for _ in range(2):
        plan = dg.EncodePlan(ctx, "onepass", layout, q=1)
        slots.append({
            "plan": plan,
            "stream": torch.cuda.Stream(),
            "ref": torch.empty(ch * L, dtype=torch.uint8, device="cuda"),
            "ver": torch.empty(ch * L, dtype=torch.uint8, device="cuda"),
            "out": torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda"),
            "offs": torch.empty(ch + 1, dtype=torch.int64, device="cuda"),
            "status": torch.empty(ch, dtype=torch.int32, device="cuda"),
            "h_offs": torch.empty(ch + 1, dtype=torch.int64, pin_memory=True),
            "h_status": torch.empty(ch, dtype=torch.int32, pin_memory=True),
            "ev": torch.cuda.Event(),
            "pending": None,
        })
    h_out = torch.empty(n * L + 64 * n, dtype=torch.uint8, pin_memory=True)

    def run_once():
        out_pos = 0
        sizes = []

        def drain(s):
            nonlocal out_pos
            if s["pending"] is None:
                return
            s["ev"].synchronize()
            if int(s["h_status"].abs().sum()) != 0:
                raise SystemExit("encode failed")
            total = int(s["h_offs"][-1])
            with torch.cuda.stream(s["stream"]):
                h_out[out_pos:out_pos + total].copy_(s["out"][:total], non_blocking=True)
            out_pos += total
            sizes.append(total)
            s["pending"] = None

        for c in range(n_chunks):
            s = slots[c % 2]
            drain(s)   # slot reuse: its previous chunk's deltas are on their way out
            with torch.cuda.stream(s["stream"]):
                s["ref"].copy_(h_ref[c * ch * L:(c + 1) * ch * L], non_blocking=True)
                s["ver"].copy_(h_ver[c * ch * L:(c + 1) * ch * L], non_blocking=True)
            s["plan"].run(s["ref"].data_ptr(), s["ver"].data_ptr(), s["out"].data_ptr(), s["out"].numel(),
                          s["offs"].data_ptr(), s["status"].data_ptr(), s["stream"].cuda_stream)
            with torch.cuda.stream(s["stream"]):
                s["h_offs"].copy_(s["offs"], non_blocking=True)
                s["h_status"].copy_(s["status"], non_blocking=True)
                s["ev"].record()
            s["pending"] = c
            drain(slots[(c + 1) % 2])
        for s in slots:
            drain(s)
        torch.cuda.synchronize()
        return out_pos

    run_once()   # warm-up
    best = None
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        total = run_once()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    # PCIe H2D reference rate on the same pinned buffers
    d = torch.empty(ch * L, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for c in range(n_chunks):
        d.copy_(h_ref[c * ch * L:(c + 1) * ch * L], non_blocking=True)
    torch.cuda.synchronize()
    h2d = n * L / (time.perf_counter() - t0) / 2**30
    print(json.dumps({
        "metric": "host-to-host onepass encode GiB/s (pinned, PCIe-inclusive)",
        "value": round(2 * n * L / best / 2**30, 3), "unit": "GiB/s",
        "pairs": n, "pair_bytes": L, "chunk_pairs": ch, "delta_bytes": total,
        "wall_s": round(best, 4), "h2d_only_GiBps": round(h2d, 2),
    }), flush=True)


if __name__ == "__main__":
    main()
