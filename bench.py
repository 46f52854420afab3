#!/usr/bin/env python3
"""bench.py — batched delta-encode throughput on MI355X.

Metric (BASELINE.json): "delta-encode GiB/s (device-resident batched pairs)".
One *step* = one pass of the hot path over one batch already resident in HBM:
CRC-64/XZ of every R and V, onepass differencing, placement and DLT\\x03
serialisation into one packed output arena (dg_encode_plan_run), plus — at
N > 1 — the RCCL all-gather of per-pair delta sizes that builds the global
output index.  value = sum(|R|+|V|) over all ranks and steps / max-over-ranks
wall time of the timed region, in GiB/s.

Workload (default, N=1 line): BASELINE configs[1] = C2, 4096 independent
64 KiB pairs per GPU, 1% random byte substitutions, --table-size 1 (q=4099),
synthetic inputs generated on the device (DESIGN.md "Synthetic inputs").
Pairs shard across ranks by contiguous index ranges (weak scaling).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU, RCCL over xGMI).
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "delta-compression_amd")

CONFIGS = {
    # name: (pairs per GPU, pair bytes, edit rate (< 0: transpositions, -pct), --table-size,
    #        seed base, description, algorithm)
    "c2": (4096, 65536, 0.01, 1, 0xC2000000,
           "4096 x 64 KiB pairs per GPU, 1% edits, onepass, --table-size 1", "onepass"),
    "c3": (8192, 262144, 0.10, 1, 0xC3000000,
           "8192 x 256 KiB pairs per GPU (65536 on 8 GPUs), 10% edits, onepass, --table-size 1",
           "onepass"),
    "c4": (4096, 262144, -50, 1, 0xC4000000,
           "4096 pairs of ~256 KiB per GPU, 8-64 block transpositions (50% moved), correcting, "
           "--table-size 1", "correcting"),
    # C5: decode + CRC-64/XZ verify of C2-style deltas (1024 streams, ~1.1M commands)
    "c5": (1024, 65536, 0.01, 1, 0xC2000000,
           "1024 onepass deltas of C2 pairs (~1.1M COPY/ADD commands), decode + src/dst CRC "
           "verify on device", "decode"),
}
ALGO_ID = {"onepass": 1, "correcting": 2, "decode": 11}

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md


def load_product():
    spec = importlib.util.spec_from_file_location(
        "delta_compression_amd", os.path.join(PKG_DIR, "__init__.py"),
        submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["delta_compression_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def pmc_traffic(config, kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (scripts/pmc_traffic.sh -> profiles/<round>_pmc_traffic_<config>.json:
    FETCH_SIZE/WRITE_SIZE passes, gfx950 corrections applied), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_traffic_{config}.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:  # noqa: BLE001
            continue
        if d.get("kernel") == kernel and d.get("hbm_bytes_per_launch"):
            return int(d["hbm_bytes_per_launch"]), os.path.relpath(f, ROOT)
    return None, None


def cpu_baseline(cfg, n_pairs_sample, threads):
    """The reference's src/c (oracle/_ref/ref_bench, compiled from
    /root/reference by oracle/Makefile) on the host cores, bounded sample of
    the same workload.  Falls back to nothing if the build is absent."""
    npg, L, rate, q, seed, _, algo = cfg
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_bench")
    if not os.path.exists(exe):
        return None
    cmd = [exe, str(ALGO_ID[algo]), str(n_pairs_sample), str(L), str(rate), str(seed), str(threads),
           str(q), "3"]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, check=True)
        res = json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f"cpu_baseline failed: {e}", file=sys.stderr)
        return None
    return {
        "value": round(res["gib_per_s"], 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "reference",
        "sample": (f"{n_pairs_sample} pairs x ~{L} B of the same workload, src/c "
                   + ("delta_decode + apply + src/dst CRC checks" if algo == "decode" else
                      f"{algo} (crc x2 + diff + place + encode)")
                   + f", {threads} threads, best of 3"),
    }


def decode_bench(args, dg, ctx, torch, dist, world, rank, n, L, q, layout, ref, ver, stream, cfg):
    """C5: the deltas of this rank's pairs are produced on the device first
    (untimed); one step = dg_decode_plan_run over all of them (reference CRC
    on a side stream, decode, output CRC, verify)."""
    shard = importlib.import_module("delta_compression_amd.shard")
    enc = dg.EncodePlan(ctx, "onepass", layout, q=q)
    d_arena = torch.empty(enc.output_bound, dtype=torch.uint8, device="cuda")
    offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    est = torch.empty(n, dtype=torch.int32, device="cuda")
    enc.run(ref.data_ptr(), ver.data_ptr(), d_arena.data_ptr(), d_arena.numel(), offs.data_ptr(),
            est.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    assert int(est.abs().sum()) == 0
    o = offs.cpu().tolist()
    descs = [(r_off, r_len, o[i], o[i + 1] - o[i], v_off, v_len)
             for i, (r_off, r_len, v_off, v_len) in enumerate(layout)]
    plan = dg.DecodePlan(ctx, descs)
    out = torch.empty_like(ver)
    out_len = torch.empty(n, dtype=torch.int64, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")

    def step():
        plan.run(ref.data_ptr(), d_arena.data_ptr(), out.data_ptr(), out_len.data_ptr(),
                 status.data_ptr(), stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    out.zero_()
    step()
    torch.cuda.synchronize()
    if (int(status.abs().sum()) != 0 or not torch.equal(out, ver)) and not os.environ.get("DG_DEBUG_BITS"):
        raise SystemExit(f"decode failed: status {status.unique().tolist()}")   # (DG_DEBUG_BITS: A/B runs only)
    plan.set_timing(args.steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stages = plan.stage_times()
    elapsed = shard.max_over_ranks(dist, elapsed, world, "cuda")
    v_bytes = sum(vl for _, _, _, vl in layout)
    d_bytes = o[-1]
    dec_ms = stages.get("decode", 0.0)
    # decode_kernel algorithmic bytes: the deltas read, COPY sources read and
    # the outputs written (<= |delta| + 2 sum|V|)
    alg = d_bytes + 2 * v_bytes
    achieved = alg / (dec_ms / 1e3) / 1e9 if dec_ms > 0 else 0.0
    if rank == 0:
        line = {
            "metric": "delta-decode GiB/s (device-resident, sum |V| reconstructed, CRC-verified)",
            "value": round(v_bytes * world * args.steps / elapsed / 2**30, 3),
            "unit": "GiB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (C2 pairs generated on device, deltas from the device encoder)",
            "config": {"workload": cfg[5], "streams_per_gpu": n, "delta_bytes_per_gpu": d_bytes,
                       "parallelism": f"dp{world} (stream shards)"},
            "roofline": {"bound": "hbm", "kernel": "decode_kernel", "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                         "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(dec_ms, 4),
                         "stage_ms": {k: round(v, 4) for k, v in stages.items()}},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = min(16, os.cpu_count() or 1)
            line["cpu_baseline"] = cpu_baseline(cfg, args.cpu_pairs or 4096, threads)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--pairs", type=int, default=0, help="override pairs per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-pairs", type=int, default=0,
                    help="CPU baseline sample size (default: ~10-30 s of src/c work)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    dg = load_product()
    shard = importlib.import_module("delta_compression_amd.shard")   # the orchestration the gloo tests run
    ctx = dg.Context(local)
    npg, L, rate, q, seed_base, desc, algo = CONFIGS[args.config]
    if args.pairs:
        npg = args.pairs
    cfg = (npg, L, rate, q, seed_base, desc, algo)

    # rank 0 decides the pair-index ranges and scatters them (RCCL broadcast);
    # equal-size pairs make the byte-balanced ranges equal index ranges
    ranges = shard.balanced_ranges([1] * (npg * world), world) if rank == 0 else None
    lo, hi = shard.scatter_ranges(dist, ranges, world, rank, "cuda")
    n = hi - lo

    stream = torch.cuda.Stream()
    if rate >= 0:   # substitution pairs (C2/C3)
        n_edits = int(rate * L + 0.5)
        ref = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        ver = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        ctx.check(dg.lib.dg_synth_edit_pairs_device(ctx.handle, ref.data_ptr(), ver.data_ptr(), n, L,
                                                    seed_base + lo, n_edits, stream.cuda_stream),
                  "synth")
        layout = [(i * L, L, i * L, L) for i in range(n)]
    else:           # transposition pairs (C4)
        import ctypes as C
        pairs = (dg._lib.Pair * n)()
        rb, vb = C.c_uint64(), C.c_uint64()
        ctx.check(dg.lib.dg_synth_transpose_pairs_device(ctx.handle, seed_base + lo, n, L, int(-rate),
                                                         pairs, C.byref(rb), C.byref(vb), None, None,
                                                         None), "layout")
        ref = torch.empty(rb.value, dtype=torch.uint8, device="cuda")
        ver = torch.empty(vb.value, dtype=torch.uint8, device="cuda")
        ctx.check(dg.lib.dg_synth_transpose_pairs_device(ctx.handle, seed_base + lo, n, L, int(-rate),
                                                         pairs, C.byref(rb), C.byref(vb), ref.data_ptr(),
                                                         ver.data_ptr(), stream.cuda_stream), "synth")
        layout = [(x.r_off, x.r_len, x.v_off, x.v_len) for x in pairs]
    if algo == "decode":
        return decode_bench(args, dg, ctx, torch, dist, world, rank, n, L, q, layout, ref, ver, stream,
                            cfg)
    plan = dg.EncodePlan(ctx, algo, layout, q=q)
    plan_aligned16 = all((r_off | v_off) % 16 == 0 for r_off, _, v_off, _ in layout)
    out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
    offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()

    def step():
        plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), offs.data_ptr(),
                 status.data_ptr(), stream.cuda_stream)
        if world > 1:
            with torch.cuda.stream(stream):
                shard.gather_sizes(dist, offs[1:] - offs[:-1], world)   # the global output index

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if int(status.abs().sum().item()) != 0:
        raise SystemExit(f"encode failed: status {status.unique().tolist()}")

    # one HIP-event set per timed step, recorded on the streams the kernels
    # run on; read back only after the timed region
    plan.set_timing(args.steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    stages = plan.stage_times()   # per-stage means over the K timed steps
    plan.set_timing(0)
    diff_ms = stages.get("diff", 0.0) * args.steps
    crc_ms = stages.get("crc64", 0.0) * args.steps

    elapsed = shard.max_over_ranks(dist, elapsed, world, "cuda")

    in_bytes_rank = sum(rl + vl for _, rl, _, vl in layout)
    total_bytes = in_bytes_rank * world * args.steps
    value = total_bytes / elapsed / 2**30
    avg_diff_s = diff_ms / args.steps / 1e3
    achieved = in_bytes_rank / avg_diff_s / 1e9 if avg_diff_s > 0 else 0.0
    delta_bytes = int(offs[-1].item())
    kname = ("correcting_build_kernel + correcting_scan_kernel" if algo == "correcting"
             else "onepass16_kernel" if plan_aligned16 else "onepass_kernel")
    traffic, traffic_src = pmc_traffic(args.config, kname) if npg == CONFIGS[args.config][0] \
        else (None, None)

    if rank == 0:
        line = {
            "metric": "delta-encode GiB/s (device-resident batched pairs) at 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": ("synthetic (splitmix64 pairs + seeded byte substitutions, generated on device)"
                     if rate >= 0 else
                     "synthetic (splitmix64 R, gen_transpositions.py-style block permutation, "
                     "generated on device)"),
            "config": {
                "workload": desc,
                "algorithm": algo,
                "pairs_per_gpu": n,
                "pair_bytes": L,
                "edit_rate": rate if rate >= 0 else None,
                "moved_block_pct": -rate if rate < 0 else None,
                "table_size_floor": q,
                "q": plan.table_size(0),
                "seed_len": 16,
                "delta_bytes_per_gpu": delta_bytes,
                "parallelism": f"dp{world} (pair shards, RCCL index scatter + size all-gather)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kname,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": in_bytes_rank,
                "avg_launch_ms": round(avg_diff_s * 1e3, 4),
                "crc_ms_per_step": round(crc_ms / args.steps, 4),
                "stage_ms": {k: round(v, 4) for k, v in stages.items()},
            },
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline:
            threads = min(16, os.cpu_count() or 1)
            # bounded sample: about 10-30 s of src/c work on `threads` cores
            sample = args.cpu_pairs or {"c2": 2048, "c3": 256, "c4": 1024}[args.config]
            line["cpu_baseline"] = cpu_baseline(cfg, sample, threads)
        print(json.dumps(line), flush=True)

    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
