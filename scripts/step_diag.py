#!/usr/bin/env python3
"""Diagnostic (not a bench line): per-step wall and kernel time of C2 for
timed regions of different lengths in one process, and the host's enqueue
time per step (is a 20-step region host-bound?)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    import torch
    torch.cuda.set_device(0)
    dg = bench.load_product()
    ctx = dg.Context(0)
    stream = torch.cuda.Stream()
    npg, L, rate, q, seed, desc, algo = bench.CONFIGS["c2"]
    ref, ver, layout = bench.make_inputs(dg, ctx, torch, "c2", 0, npg, stream)
    plan = dg.EncodePlan(ctx, algo, layout, q=q)
    out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
    offs = torch.empty(npg + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(npg, dtype=torch.int32, device="cuda")

    batches = [(ref, ver)]
    if len(sys.argv) > 1 and sys.argv[1] == "rotate":   # 4 input batches in turn: 2.1 GB >> the 256 MB MALL
        for b in range(3):
            r2, v2, _ = bench.make_inputs(dg, ctx, torch, "c2", 4096 * (b + 1), npg, stream)
            batches.append((r2, v2))
    cur = [0]

    def step():
        r, v = batches[cur[0] % len(batches)]
        cur[0] += 1
        plan.run(r.data_ptr(), v.data_ptr(), out.data_ptr(), out.numel(), offs.data_ptr(), st.data_ptr(),
                 stream.cuda_stream)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    mode = sys.argv[1] if len(sys.argv) > 1 else "c2"
    if mode == "matmul":   # ~150 ms of unrelated GPU load first: a clock ramp, or C2-specific?
        a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
        t = time.perf_counter()
        while time.perf_counter() - t < 0.15:
            a @ a
        torch.cuda.synchronize()
    if mode == "idle":     # 50 ms idle after warmup
        time.sleep(0.05)
    for K in [20, 20, 200, 20, 20, 200, 50, 20]:
        plan.set_timing(K, dominant_only=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        s = plan.stage_times()
        print(f"K={K:4d} wall/step {1e3 * (t2 - t0) / K:.4f} ms  host enqueue/step {1e3 * (t1 - t0) / K:.4f} ms  "
              f"diff {s.get('diff', 0):.4f} ms", flush=True)
    plan.close()


if __name__ == "__main__":
    main()
