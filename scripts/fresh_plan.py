#!/usr/bin/env python3
"""Diagnostic (not a bench line): is the slow start of a bench line a property
of a fresh plan, of fresh buffers, or of the GPU coming out of idle?

Run under `rocprofv3 --kernel-trace` and read the dominant kernel's duration
per dispatch (scripts/fresh_plan_read.py).  Phases, back to back in one
process on one stream, each tagged by a marker kernel (a tiny synth launch):
  A  plan A, 120 steps                (fresh plan, GPU coming out of idle)
  B  plan B (new plan, same inputs), 120 steps, no idle before it
  C  plan A again, 120 steps, right after B
  D  idle 300 ms, then plan A, 120 steps
usage: python3 scripts/fresh_plan.py [config]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import torch
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    torch.cuda.set_device(0)
    dg = bench.load_product()
    ctx = dg.Context(0)
    stream = torch.cuda.Stream()
    npg, L, rate, q, seed, desc, algo = bench.CONFIGS[name]
    ref, ver, layout = bench.make_inputs(dg, ctx, torch, name, 0, npg, stream)
    torch.cuda.synchronize()
    plans = [dg.EncodePlan(ctx, algo, layout, q=q) for _ in range(2)]
    out = torch.empty(plans[0].output_bound, dtype=torch.uint8, device="cuda")
    offs = torch.empty(npg + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(npg, dtype=torch.int32, device="cuda")
    marker = torch.empty(64, dtype=torch.uint8, device="cuda")

    def mark():   # a tiny, recognisable launch between phases
        ctx.check(dg.lib.dg_synth_edit_pairs_device(ctx.handle, marker.data_ptr(), marker.data_ptr(), 1, 64, 7, 0,
                                                    stream.cuda_stream), "marker")

    def steps(plan, k):
        for _ in range(k):
            plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), offs.data_ptr(), st.data_ptr(),
                     stream.cuda_stream)

    time.sleep(0.3)   # idle before A
    t = {}
    for ph, plan, idle in (("A", 0, 0.0), ("B", 1, 0.0), ("C", 0, 0.0), ("D", 0, 0.3)):
        if idle:
            torch.cuda.synchronize()
            time.sleep(idle)
        mark()
        t0 = time.perf_counter()
        steps(plans[plan], 120)
        torch.cuda.synchronize()
        t[ph] = (time.perf_counter() - t0) / 120 * 1e3
    print({k: round(v, 4) for k, v in t.items()}, "ms per step (wall, 120 steps each)", flush=True)
    for p in plans:
        p.close()


if __name__ == "__main__":
    main()
