#!/usr/bin/env python3
"""A/B measurement over a variant library (DG_LIB_VARIANT=ab|prof|<name>) with
the DG_* measurement switches of that build.  Not the benchmark of record:
bench.py refuses to run with any DG_* variable set; this wrapper prints the
same fields, tagged "ab": true with the switches used, for profiles/
experiment tables only.

usage: DG_LIB_VARIANT=ab DG_SERIAL_CRC=1 python scripts/ab_bench.py --config c2 --steps 20
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(bench.CONFIGS))
    ap.add_argument("--pairs", type=int, default=0)
    args = ap.parse_args()
    args.no_cpu_baseline = True
    # "dominant" (bench.py's default), "all" stage events or "none" in the timed steps
    args.stage_timing = os.environ.get("AB_TIMING", "dominant")
    args.timing_every = int(os.environ.get("AB_EVERY", bench.TIMING_EVERY))   # timed steps with events
    import torch
    torch.cuda.set_device(0)
    R = bench.Rank(1, 0, 0, None, torch)
    dg = bench.load_product()
    shard = bench.load_shard()
    ctx = dg.Context(0)
    line = bench.run_config(args.config, args, R, dg, ctx, shard, torch.cuda.Stream())
    line["ab"] = True
    line["ab_switches"] = {k: v for k, v in os.environ.items() if k.startswith("DG_")}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
