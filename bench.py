#!/usr/bin/env python3
"""bench.py — batched delta-encode throughput on MI355X.

Metric (BASELINE.json): "delta-encode GiB/s (device-resident batched pairs)
at 1/2/4/8 MI355X".  One *step* = one pass of the hot path over one batch
already resident in HBM: CRC-64/XZ of every R and V, onepass differencing,
placement and DLT\\x03 serialisation into one packed output arena
(dg_encode_plan_run), plus — at N > 1 — the RCCL all-gather of per-pair delta
sizes and the prefix sum that builds the global output index.  value =
sum(|R|+|V|) over all ranks and steps / max-over-ranks wall time of the timed
region, in GiB/s.

The printed line is the C2 workload (BASELINE configs[1]: 4096 independent
64 KiB pairs per GPU, 1% byte substitutions, --table-size 1 -> q = 4099).
Beside it, under "also", the same run measures the other BASELINE configs on
the same ranks, each with its own roofline and CPU baseline:
  c3  8192 x 256 KiB pairs per GPU, 10% edits, onepass, q = 16411 (the config
      BASELINE shards over 8 GPUs: 65536 pairs on 8);
  c4  4096 transposition pairs of ~256 KiB per GPU, correcting;
  c5  1024 in-place deltas per GPU (device-encoded C2 deltas converted by
      dg_make_inplace(localmin), ~1.1 M commands), decode + src/dst CRC verify.
Inputs are synthetic and generated on the device (DESIGN.md "Synthetic
inputs").  Pairs shard across ranks by contiguous index ranges (weak scaling).

Launch: python bench.py [--gpus N --steps K --warmup W].  With N > 1 and no
WORLD_SIZE in the environment, bench.py starts torch.distributed.run with N
ranks itself (before any GPU call); under torch.distributed.run it runs as
one rank per GPU (RCCL over xGMI).  --dry-run brings the ranks up over gloo on
the CPU and runs only the orchestration (no GPU, no encode, value null): the
launcher test of tests/test_bench_cpu.py.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import platform
import socket
import statistics
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
    # C5: decode + CRC-64/XZ verify of in-place deltas of C2 pairs (1024 streams, ~1.1M commands)
    "c5": (1024, 65536, 0.01, 1, 0xC2000000,
           "1024 in-place deltas of C2 pairs per GPU (device onepass encode + dg_make_inplace "
           "localmin, ~1.1M COPY/ADD commands), decode + src/dst CRC verify on device", "decode"),
    # stated extra line (not a BASELINE config): in-place
    # deltas whose COPYs move, so the replay order matters (apply.c:253-267)
    "c5o": (1024, 262144, -50, 1, 0xC4000000,
            "1024 in-place deltas of C4 transposition pairs per GPU (device correcting encode + "
            "dg_make_inplace localmin: moving COPYs, order-dependent replay), decode + src/dst CRC "
            "verify on device", "decode"),
    # stated extra lines: edits that move the diagonal, and
    # onepass on the C4 transposition pairs, each in the automatic chain mode
    # and with the plain per-pair chain forced
    "c3s": (8192, 262144, 0.10, 1, 0xC3500000,
            "8192 x 256 KiB shift pairs per GPU: 10% edits, 2/3 of them insertions or deletions of "
            "1-8 bytes (half each), 1/3 byte substitutions; onepass, --table-size 1, automatic chain mode",
            "onepass"),
    "c3s_chain": (8192, 262144, 0.10, 1, 0xC3500000,
                  "c3s with the plain per-pair chain forced (DG_LIMIT_ONEPASS_MEMBERS = 2)", "onepass"),
    "c4o": (4096, 262144, -50, 1, 0xC4000000,
            "C4's 4096 transposition pairs of ~256 KiB per GPU, onepass, --table-size 1, automatic chain mode",
            "onepass"),
    "c4o_chain": (4096, 262144, -50, 1, 0xC4000000,
                  "c4o with the plain per-pair chain forced (DG_LIMIT_ONEPASS_MEMBERS = 2)", "onepass"),
    # the north star's upper pair size: 1 MiB pairs,
    # --table-size 1 -> q = next_prime(65536) = 65537 (onepass.c:61-62)
    "c6": (1024, 1048576, 0.01, 1, 0xC6000000,
           "1024 x 1 MiB pairs per GPU, 1% edits, onepass, --table-size 1", "onepass"),
    # C2 at the CLI's default --table-size (q = 1048573, delta.h:21)
    "c2_defq": (4096, 65536, 0.01, 1048573, 0xC2000000,
                "C2 (4096 x 64 KiB pairs per GPU, 1% edits) onepass at the default --table-size "
                "(q = 1048573)", "onepass"),
}
# per-config options: shift pairs (percent of edits that are insertions or
# deletions), the chain mode forced through the context limit, the config
# whose CPU baseline a forced-mode line shares
OPTS = {
    "c3s": {"indel_pct": 67},
    "c3s_chain": {"indel_pct": 67, "members": 2, "cpu_as": "c3s"},
    "c4o_chain": {"members": 2, "cpu_as": "c4o"},
}
# oracle/_ref/ref_bench modes: encode onepass / correcting; decode standard / in-place deltas
REF_MODE = {"onepass": 1, "correcting": 2, "decode": 12, "decode_correcting": 13}
# CPU baseline samples (pairs): ~1-3 s per timed repetition of the reference's src/c
CPU_SAMPLE = {"c2": (1024, 4096), "c3": (64, 512), "c4": (64, 512), "c5": (1024, 4096), "c5o": (128, 1024),
              "c3s": (32, 256), "c4o": (64, 512), "c6": (64, 256), "c2_defq": (1024, 4096)}

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak, /opt/skills/guides/MI355X_MICROARCH.md
# In the timed steps the kernel events are recorded on every TIMING_EVERY-th
# step only: each event costs its stream ~3.5 us (C2's two per step cost the
# line ~1.5 %); the average launch time comes from those sampled launches.
TIMING_EVERY = 4


def timing_ring(steps, every=TIMING_EVERY):
    """(every, slots): the ring holds exactly the sampled timed steps."""
    every = max(1, min(every, steps))
    return every, max(1, steps // every)


def load_product():
    spec = importlib.util.spec_from_file_location(
        "delta_compression_amd", os.path.join(PKG_DIR, "__init__.py"),
        submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["delta_compression_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_shard():
    spec = importlib.util.spec_from_file_location("dg_shard", os.path.join(PKG_DIR, "shard.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def lib_sha16():
    """The product library's identity (sha256 of the .so, 16 hex digits): a
    PMC traffic summary is only reported for the library it was measured on."""
    import hashlib
    path = os.path.join(PKG_DIR, "lib", "libdeltagpu.so")
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def pmc_traffic(config, kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (scripts/profile_round.sh + profile_collect.py -> profiles/<round>_pmc_traffic_
    <config>.json: FETCH_SIZE/WRITE_SIZE passes, gfx950 corrections applied),
    or None.  A summary measured on another build of the library is stale (a
    kernel change moves the traffic) and is not reported: the source says so."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_traffic_{config}.json")))
    cur = lib_sha16()
    stale = None
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:  # noqa: BLE001
            continue
        if d.get("kernel") == kernel and d.get("hbm_bytes_per_launch"):
            if d.get("lib_sha16") and d["lib_sha16"] == cur:
                return int(d["hbm_bytes_per_launch"]), os.path.relpath(f, ROOT)
            stale = stale or os.path.relpath(f, ROOT)
    return None, (f"stale: {stale} was measured on another build of the library" if stale else None)


def pmc_path(config):
    """HBM bytes per step of every kernel of the step (profiles/<round>_pmc_path_
    <config>.json, scripts/profile_round.sh path + profile_collect.py), lower and
    upper readings, or None when the newest summary is of another library build."""
    import glob
    cur = lib_sha16()
    stale = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_path_{config}.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:  # noqa: BLE001
            continue
        if d.get("path_traffic_per_step"):
            if d.get("lib_sha16") and d["lib_sha16"] == cur:
                return d, os.path.relpath(f, ROOT)
            stale = stale or os.path.relpath(f, ROOT)
    return None, (f"stale: {stale} was measured on another build of the library" if stale else None)


# ───────────────────────────── CPU baseline ─────────────────────────────────

def cpu_share() -> int:
    """Host threads this process may use: the affinity set, capped by
    OMP_NUM_THREADS where the pool sets it (16 per GPU on the GPU boxes)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _ref_bench(name, pairs, threads, reps=5):
    npg, L, rate, q, seed, _, algo = CONFIGS[name]
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_bench")
    mode = REF_MODE["decode_correcting" if algo == "decode" and rate < 0 else algo]
    cmd = [exe, str(mode), str(pairs), str(L), str(rate), str(seed), str(threads), str(q), str(reps)]
    if OPTS.get(name, {}).get("indel_pct") is not None:
        cmd.append(str(OPTS[name]["indel_pct"]))
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, check=True)
    return json.loads(r.stdout.strip().splitlines()[-1])


def cpu_baseline(name):
    """The reference's own src/c (oracle/_ref/ref_bench, compiled from
    /root/reference by oracle/Makefile) on the host, a bounded sample of the
    same workload: 1 thread and every thread of this process's CPU share,
    median of 5 timed repetitions each."""
    name = OPTS.get(name, {}).get("cpu_as", name)
    cfg = CONFIGS[name]
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_bench")
    if not os.path.exists(exe):
        return None
    n1, nall = CPU_SAMPLE[name]
    threads = cpu_share()
    try:
        one = _ref_bench(name, n1, 1)
        many = _ref_bench(name, nall, threads)
    except Exception as e:  # noqa: BLE001
        print(f"cpu_baseline failed: {e}", file=sys.stderr)
        return None
    algo = cfg[6]
    enc = "correcting" if cfg[2] < 0 else "onepass"
    work = ("delta_decode + delta_apply_delta_inplace + src/dst CRC checks of in-place "
            f"(localmin) {enc} deltas; rate = sum |V| / time" if algo == "decode" else
            f"{algo} chain crc x2 + delta_diff + delta_place_commands + delta_encode; "
            "rate = sum(|R|+|V|) / time")
    work = f"[{name}] " + work
    return {
        "value": round(many["gib_per_s"], 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "reference",
        "sample": (f"src/c {work}; {nall} pairs x ~{cfg[1]} B of the same workload on {threads} "
                   f"threads, median of {many['reps']} (times {many.get('times_s')})"),
        "single_thread": {"value": round(one["gib_per_s"], 4), "pairs": n1,
                          "median_s": one.get("median_s"), "times_s": one.get("times_s")},
        "nproc": os.cpu_count(),
        "affinity_cpus": _affinity(),
        "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
        # the GPU pool grants each one-GPU lease a share of the host (16 CPUs,
        # OMP_NUM_THREADS=16) while nproc shows the whole machine: the timed
        # baseline stays inside the share; beside it, the single-thread rate
        # scaled linearly to every host CPU (an upper bound: the reference's
        # malloc-bound chain scales sub-linearly)
        "full_host_upper_bound": {"value": round(one["gib_per_s"] * (os.cpu_count() or 1), 4),
                                  "cores": os.cpu_count(),
                                  "basis": "single_thread x nproc (not run: outside the lease's CPU share)"},
        "cpu_model": cpu_model(),
    }


def _affinity():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return None


# ───────────────────────────── device workloads ─────────────────────────────

class Rank:
    def __init__(self, world, rank, local, dist, torch):
        self.world, self.rank, self.local, self.dist, self.torch = world, rank, local, dist, torch

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()


def job_pair_bytes(dg, ctx, name, total):
    """|R|+|V| of every pair of the whole job, from the generators' host-side
    layout (no device bytes): the byte weights rank 0 balances the ranges by
    (SURVEY 8(e)).  Substitution pairs are all 2L; shift and transposition
    pairs vary."""
    npg, L, rate, q, seed_base, desc, algo = CONFIGS[name]
    indel = OPTS.get(name, {}).get("indel_pct")
    if indel is None and rate >= 0:
        return [2 * L] * total
    import ctypes as C
    pairs = (dg._lib.Pair * max(total, 1))()
    rb, vb = C.c_uint64(), C.c_uint64()
    if indel is not None:
        ctx.check(dg.lib.dg_synth_shift_pairs_device(ctx.handle, seed_base, total, L, int(rate * L + 0.5), indel,
                                                     pairs, C.byref(rb), C.byref(vb), None, None, None), "layout")
    else:
        ctx.check(dg.lib.dg_synth_transpose_pairs_device(ctx.handle, seed_base, total, L, int(-rate), pairs,
                                                         C.byref(rb), C.byref(vb), None, None, None), "layout")
    return [x.r_len + x.v_len for x in pairs[:total]]


def make_inputs(dg, ctx, torch, name, lo, n, stream):
    npg, L, rate, q, seed_base, desc, algo = CONFIGS[name]
    indel = OPTS.get(name, {}).get("indel_pct")
    if indel is not None:   # shift pairs (C3s): substitutions, insertions, deletions
        import ctypes as C
        n_edits = int(rate * L + 0.5)
        pairs = (dg._lib.Pair * max(n, 1))()
        rb, vb = C.c_uint64(), C.c_uint64()
        ctx.check(dg.lib.dg_synth_shift_pairs_device(ctx.handle, seed_base + lo, n, L, n_edits, indel, pairs,
                                                     C.byref(rb), C.byref(vb), None, None, None), "layout")
        ref = torch.empty(max(rb.value, 1), dtype=torch.uint8, device="cuda")
        ver = torch.empty(max(vb.value, 1), dtype=torch.uint8, device="cuda")
        ctx.check(dg.lib.dg_synth_shift_pairs_device(ctx.handle, seed_base + lo, n, L, n_edits, indel, pairs,
                                                     C.byref(rb), C.byref(vb), ref.data_ptr(), ver.data_ptr(),
                                                     stream.cuda_stream), "synth")
        return ref, ver, [(x.r_off, x.r_len, x.v_off, x.v_len) for x in pairs[:n]]
    if rate >= 0:   # substitution pairs (C2/C3/C5)
        n_edits = int(rate * L + 0.5)
        ref = torch.empty(max(n, 1) * L, dtype=torch.uint8, device="cuda")
        ver = torch.empty(max(n, 1) * L, dtype=torch.uint8, device="cuda")
        ctx.check(dg.lib.dg_synth_edit_pairs_device(ctx.handle, ref.data_ptr(), ver.data_ptr(), n, L,
                                                    seed_base + lo, n_edits, stream.cuda_stream),
                  "synth")
        return ref, ver, [(i * L, L, i * L, L) for i in range(n)]
    import ctypes as C   # transposition pairs (C4)
    pairs = (dg._lib.Pair * max(n, 1))()
    rb, vb = C.c_uint64(), C.c_uint64()
    ctx.check(dg.lib.dg_synth_transpose_pairs_device(ctx.handle, seed_base + lo, n, L, int(-rate), pairs,
                                                     C.byref(rb), C.byref(vb), None, None, None), "layout")
    ref = torch.empty(max(rb.value, 1), dtype=torch.uint8, device="cuda")
    ver = torch.empty(max(vb.value, 1), dtype=torch.uint8, device="cuda")
    ctx.check(dg.lib.dg_synth_transpose_pairs_device(ctx.handle, seed_base + lo, n, L, int(-rate), pairs,
                                                     C.byref(rb), C.byref(vb), ref.data_ptr(),
                                                     ver.data_ptr(), stream.cuda_stream), "synth")
    return ref, ver, [(x.r_off, x.r_len, x.v_off, x.v_len) for x in pairs[:n]]


def timed(R, args, step):
    """W untimed steps, then exactly K steps bracketed by barrier + synchronize;
    returns the max-over-ranks wall time of the K steps."""
    torch = R.torch
    R.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    R.barrier()
    return time.perf_counter() - t0


def bench_encode(name, args, R, dg, ctx, shard, stream):
    torch = R.torch
    cfg = CONFIGS[name]
    npg, L, rate, q, seed_base, desc, algo = cfg
    if args.pairs:
        npg = args.pairs
    total = npg * R.world
    ranges = (shard.balanced_ranges(job_pair_bytes(dg, ctx, name, total), R.world) if R.world > 1
              else [(0, total)]) if R.rank == 0 else None
    allr = shard.all_ranges(R.dist, ranges, R.world, R.rank, "cuda")
    lo, hi = allr[R.rank]
    n = hi - lo
    ref, ver, layout = make_inputs(dg, ctx, torch, name, lo, n, stream)
    members = OPTS.get(name, {}).get("members")
    if members is not None:
        ctx.set_limit(dg.LIMIT_ONEPASS_MEMBERS, members)
    try:
        plan = dg.EncodePlan(ctx, algo, layout, q=q)
    finally:
        if members is not None:
            ctx.set_limit(dg.LIMIT_ONEPASS_MEMBERS, dg.MEMBERS_AUTO)
    aligned16 = all((r_off | v_off) % 16 == 0 for r_off, _, v_off, _ in layout)
    out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
    offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")
    sizes = torch.empty(n, dtype=torch.int64, device="cuda")
    gather = shard.SizeGather([b - a for a, b in allr], "cuda")
    torch.cuda.synchronize()

    def step():
        plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), offs.data_ptr(),
                 status.data_ptr(), stream.cuda_stream)
        if R.world > 1:   # the global output index: all-gather of sizes + prefix sum
            with torch.cuda.stream(stream):
                torch.sub(offs[1:], offs[:-1], out=sizes)
                gather.global_offsets(gather(R.dist, sizes))

    # a checked step first (status, global index), then the W warmup steps
    # straight into the K timed ones: no host round trip between them, so
    # the GPU does not idle (and drop its clocks) just before the timer starts
    torch.cuda.synchronize()
    t_chk = time.perf_counter()
    step()
    torch.cuda.synchronize()
    t_chk = time.perf_counter() - t_chk
    bad = int((status != 0).sum().item())
    if bad:
        raise SystemExit(f"{name}: encode failed on {bad} pairs: status {status.unique().tolist()}")
    if R.world > 1:   # the global index covers every rank's packed deltas
        tot = offs[-1:].clone()
        R.dist.all_reduce(tot)
        if int(gather.offsets[-1].item()) != int(tot.item()):
            raise SystemExit(f"{name}: global output index inconsistent")
    yield None   # prepared: the caller decides when the measurement runs

    # The stage breakdown first: an untimed pass with every stage event, over
    # at least K steps and ~50 ms of GPU time.  It also brings the plan to its
    # steady state: a fresh C2 plan runs its first ~40 steps ~12 % slower
    # (scripts/step_diag.py: the same with 4 input batches in turn, so not the
    # Infinity Cache, and after unrelated GPU load, so not the clocks).
    n_prof = max(args.steps, min(200, int(0.05 / max(t_chk, 1e-6))))
    plan.set_timing(n_prof)
    for _ in range(n_prof):
        step()
    profile = plan.stage_times()

    # In the timed steps only the events around the dominant kernel(s) are
    # recorded; the full stage breakdown comes from an untimed pass of the
    # same steps afterwards.  (The ring keeps the last K runs: the timed ones.)
    timing = getattr(args, "stage_timing", "dominant")
    every, slots = timing_ring(args.steps, getattr(args, "timing_every", TIMING_EVERY))
    if timing != "none":
        plan.set_timing(slots, dominant_only=timing == "dominant", every=every)
    else:
        plan.set_timing(0)
    for _ in range(args.warmup):
        step()
    modes0 = plan.run_modes
    elapsed = timed(R, args, step)
    modes1 = plan.run_modes
    stages = plan.stage_times() if timing != "none" else {}
    plan.set_timing(0)
    elapsed = shard.max_over_ranks(R.dist, elapsed, R.world, "cuda")

    in_bytes_rank = sum(rl + vl for _, rl, _, vl in layout)
    in_bytes_job = shard.sum_over_ranks(R.dist, in_bytes_rank, R.world, "cuda")
    value = in_bytes_job * args.steps / elapsed / 2**30
    members = plan.members
    # automatic member mode over a batch it routes entirely to the plain chain:
    # the timed runs go as a plain plan between member-mode probes
    member_runs, plain_runs = modes1[0] - modes0[0], modes1[1] - modes0[1]
    plain_runs_dominate = members and plain_runs > member_runs
    # the dominant kernel: the member kernel alone in member mode (its own
    # event pair), else the differencing kernel(s) of the "diff" stage
    diff_ms = stages.get("members", 0.0) if members else stages.get("diff", 0.0)
    chains_dominate = False
    if plain_runs_dominate:
        diff_ms = stages.get("diff", 0.0) - stages.get("members", 0.0)
    elif members and stages.get("diff", 0.0) - stages.get("members", 0.0) > stages.get("members", 0.0):
        # most pairs were routed to the plain chain (matches off diagonal 0):
        # the chain kernels after the member kernel dominate
        diff_ms = stages["diff"] - stages["members"]
        chains_dominate = True
    if algo == "correcting":   # the build and the scan, back to back
        diff_ms = stages.get("corr_build", 0.0) + stages.get("corr_scan", 0.0)
    achieved = in_bytes_rank / (diff_ms / 1e3) / 1e9 if diff_ms > 0 else 0.0
    delta_bytes = int(offs[-1].item())
    kname = ("correcting_build_kernel + correcting_scan_kernel" if algo == "correcting"
             else "onepass16_kernel (member chain + routed plain chain)" if chains_dominate
             else "member_chunk_kernel" if members and not plain_runs_dominate
             else "onepass16_kernel" if aligned16 else "onepass_kernel")
    traffic, traffic_src = pmc_traffic(name, kname) if npg == CONFIGS[name][0] else (None, None)
    # the path-level roofline of SURVEY §8(d) / BASELINE.md §3: every input
    # byte read once plus every delta byte written, over the whole step
    path_bytes = in_bytes_rank + delta_bytes
    step_s = elapsed / args.steps
    line = {
        "metric": "delta-encode GiB/s (device-resident batched pairs) at 1/2/4/8 MI355X",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": R.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "untimed_steps": 1 + n_prof + args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": ("synthetic (splitmix64 R, seeded substitutions / insertions / deletions, generated on "
                 "device)" if OPTS.get(name, {}).get("indel_pct") is not None else
                 "synthetic (splitmix64 pairs + seeded byte substitutions, generated on device)"
                 if rate >= 0 else
                 "synthetic (splitmix64 R, gen_transpositions.py-style block permutation, "
                 "generated on device)"),
        "config": {
            "workload": desc,
            "name": name,
            "algorithm": algo,
            "pairs_per_gpu": n,
            "pairs_total": total,
            "pair_bytes": L,
            "edit_rate": rate if rate >= 0 else None,
            "moved_block_pct": -rate if rate < 0 else None,
            "indel_pct": OPTS.get(name, {}).get("indel_pct"),
            "table_size_floor": q,
            "q": plan.table_size(0),
            "seed_len": 16,
            "onepass_chain": ((f"automatic: {plain_runs} of the {member_runs + plain_runs} timed runs as a plain "
                               f"plan (the last member-mode run routed every pair to the per-pair chain), "
                               f"{member_runs} member-mode probes" if plain_runs_dominate else
                               "verified diagonal members") if members else "per-pair chain")
                             if algo == "onepass" else None,
            "delta_bytes_per_gpu": delta_bytes,
            "parallelism": f"dp{R.world} (pair shards, RCCL index scatter + size all-gather)",
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
            "algorithmic_bytes_per_pair": "|R| + |V| (both streams read once)",
            "avg_launch_ms": round(diff_ms, 4),
            "timed_launches_sampled": f"events on every {every}th timed step ({slots} launches)",
            "timing": ("HIP events on the run stream after the member kernel and after the chain "
                       "kernels (member chain, routed plain chain), mean over the timed steps"
                       if chains_dominate else
                       "HIP events on the run stream around the chain kernels (plain runs: the plain "
                       "chain; member-mode probes: the member and routed chains after the member "
                       "kernel), mean over the timed steps"
                       if plain_runs_dominate else
                       "HIP events on the run stream around the member kernel, mean over the timed "
                       "steps (the only events recorded in them)"
                       if members else
                       "HIP events on the run stream around the correcting R-index build and the V "
                       "scan, mean over the timed steps (the only events recorded in them)"
                       if algo == "correcting" else
                       "HIP events on the run stream around the onepass kernel, mean over the timed "
                       "steps (the only events recorded in them)"),
            "stage_ms": {k: round(v, 4) for k, v in stages.items()},
            "stage_ms_profile": {k: round(v, 4) for k, v in profile.items()},
            "stage_ms_profile_note": (f"every stage event, an untimed pass of {n_prof} steps before the W warmup "
                                      "and K timed steps"),
            "path_bytes_per_step": path_bytes,
            "path_bytes": "sum(|R|+|V|) + sum|delta| per rank (SURVEY 8(d))",
            "path_achieved": round(path_bytes / step_s / 1e9, 2),
            "path_frac": round(path_bytes / step_s / 1e9 / HBM_PEAK_GBS, 5),
        },
        "cpu_baseline": None,
        "lib_sha16": lib_sha16(),
    }
    if npg == CONFIGS[name][0]:
        pt, pt_src = pmc_path(name)
        rl = line["roofline"]
        rl["path_traffic"] = pt["path_traffic_per_step"] if pt else None
        rl["path_traffic_upper"] = pt["path_traffic_upper_per_step"] if pt else None
        rl["path_traffic_ratio"] = round(pt["path_traffic_per_step"] / path_bytes, 3) if pt else None
        rl["path_traffic_source"] = pt_src
    if algo == "correcting" and stages.get("corr_build") is not None:
        # the build and the scan apart (HIP events on the run stream; the
        # CRC shares the CUs with them)
        line["roofline"]["kernels_ms"] = {"build": round(stages["corr_build"], 4),
                                          "scan": round(stages["corr_scan"], 4)}
    yield line
    plan.close()
    del ref, ver, out, offs, status, sizes, gather
    torch.cuda.empty_cache()


def bench_decode(name, args, R, dg, ctx, shard, stream):
    """C5 / C5o: in-place deltas of this rank's pairs are produced first
    (untimed: device onepass (C2 pairs) or correcting (C4 transposition
    pairs) encode, then dg_make_inplace(localmin) on the host, as `delta
    encode --inplace` does); one step = dg_decode_plan_run over all of them
    (one kernel: parse, apply, source and output CRC-64/XZ checks)."""
    torch = R.torch
    cfg = CONFIGS[name]
    npg, L, rate, q, seed_base, desc, algo = cfg
    if args.pairs:
        npg = args.pairs
    total = npg * R.world
    ranges = (shard.balanced_ranges(job_pair_bytes(dg, ctx, name, total), R.world) if R.world > 1
              else [(0, total)]) if R.rank == 0 else None
    lo, hi = shard.all_ranges(R.dist, ranges, R.world, R.rank, "cuda")[R.rank]
    n = hi - lo
    ref, ver, layout = make_inputs(dg, ctx, torch, name, lo, n, stream)
    enc_algo = "onepass" if rate >= 0 else "correcting"
    enc = dg.EncodePlan(ctx, enc_algo, layout, q=q)
    d_arena = torch.empty(enc.output_bound, dtype=torch.uint8, device="cuda")
    offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    est = torch.empty(n, dtype=torch.int32, device="cuda")
    enc.run(ref.data_ptr(), ver.data_ptr(), d_arena.data_ptr(), d_arena.numel(), offs.data_ptr(),
            est.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    assert int(est.abs().sum()) == 0
    o = offs.cpu().tolist()
    std = d_arena[:o[-1]].cpu().numpy().tobytes()
    ref_h = ref.cpu().numpy().tobytes()
    enc.close()
    del d_arena, est
    deltas, commands = [], 0
    moving = 0
    for i, (r_off, r_len, v_off, v_len) in enumerate(layout):
        d = dg.make_inplace(ref_h[r_off:r_off + r_len], std[o[i]:o[i + 1]], policy="localmin")
        deltas.append(d)
        commands += dg.info(d)["num_commands"]
        if rate < 0:   # COPYs that move (src != dst): the replay order matters
            moving += sum(1 for c in dg.decode_delta(d)[0] if isinstance(c, dg.PlacedCopy) and c.src != c.dst)
    del std, ref_h
    d_offs = [0]
    for d in deltas:
        d_offs.append(d_offs[-1] + len(d))
    d_dev = torch.frombuffer(bytearray(b"".join(deltas)), dtype=torch.uint8).to("cuda")
    # output i at V's own arena offset (16-byte aligned), room for max(|R|, |V|)
    descs = [(r_off, r_len, d_offs[i], len(deltas[i]), v_off, max(r_len, v_len))
             for i, (r_off, r_len, v_off, v_len) in enumerate(layout)]
    plan = dg.DecodePlan(ctx, descs)
    out_bytes = max(max(d[4] + d[5] for d in descs), ver.numel())
    out = torch.empty(out_bytes, dtype=torch.uint8, device="cuda")
    pads = [(v_off + v_len, (v_off + v_len + 15) // 16 * 16) for _, _, v_off, v_len in layout]
    if any(b > a for a, b in pads):   # the arena's padding between streams is not part of V
        for a, b in pads:
            ver[a:b] = 0
    out_len = torch.empty(n, dtype=torch.int64, device="cuda")
    status = torch.empty(n, dtype=torch.int32, device="cuda")

    def step():
        plan.run(ref.data_ptr(), d_dev.data_ptr(), out.data_ptr(), out_len.data_ptr(),
                 status.data_ptr(), stream.cuda_stream)

    out.zero_()                 # (torch's stream: finished before the decode's stream starts)
    torch.cuda.synchronize()
    step()                      # a checked step, then warmup straight into the timed steps
    torch.cuda.synchronize()
    if int(status.abs().sum()) != 0 or not torch.equal(out[:ver.numel()], ver):
        raise SystemExit(f"{name}: decode failed: status {status.unique().tolist()}")
    yield None   # prepared
    every, slots = timing_ring(args.steps, getattr(args, "timing_every", TIMING_EVERY))
    plan.set_timing(slots, every=every)
    for _ in range(args.warmup):
        step()
    elapsed = timed(R, args, step)
    stages = plan.stage_times()
    elapsed = shard.max_over_ranks(R.dist, elapsed, R.world, "cuda")
    v_bytes = sum(vl for _, _, _, vl in layout)
    v_bytes_job = shard.sum_over_ranks(R.dist, v_bytes, R.world, "cuda")
    d_bytes = d_offs[-1]
    dec_ms = stages.get("decode", 0.0)
    # decode algorithmic bytes: every delta byte read, R read
    # once, the output written once -> |delta| + |R| + |V|.  The kernel as
    # designed moves more (design_bytes: the in-place image is R copied into
    # the output first, R's CRC taken from the same read, the COPY sources are
    # read from the image, and the output is read again by the output CRC
    # check: |delta| + |R| + 3|V|)
    r_bytes = sum(rl for _, rl, _, _ in layout)
    alg = d_bytes + r_bytes + v_bytes
    design = d_bytes + r_bytes + 3 * v_bytes
    achieved = alg / (dec_ms / 1e3) / 1e9 if dec_ms > 0 else 0.0
    step_s = elapsed / args.steps
    traffic, traffic_src = pmc_traffic(name, "decode_kernel") if npg == CONFIGS[name][0] else (None, None)
    line = {
        "metric": "delta-decode GiB/s (device-resident, sum |V| reconstructed, CRC-verified)",
        "value": round(v_bytes_job * args.steps / elapsed / 2**30, 3),
        "unit": "GiB/s", "n_gpus": R.world, "steps": args.steps, "warmup": args.warmup,
        "untimed_steps": 1 + args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": (f"synthetic ({'C2' if rate >= 0 else 'C4 transposition'} pairs generated on device; "
                 f"deltas from the device {enc_algo} encoder, converted to in-place by "
                 "dg_make_inplace localmin)"),
        "config": {"workload": desc, "name": name, "inplace": True, "policy": "localmin",
                   "encoder": enc_algo, "pair_bytes": L,
                   "streams_per_gpu": n, "commands_per_gpu": commands, "delta_bytes_per_gpu": d_bytes,
                   "moving_copies_per_gpu": moving if rate < 0 else None,
                   "parallelism": f"dp{R.world} (stream shards)"},
        "roofline": {"bound": "hbm", "kernel": "decode_kernel", "achieved": round(achieved, 2),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": alg,
                     "algorithmic_bytes_per_stream": "|delta| + |R| + |V| (SURVEY 8(d))",
                     "design_bytes_per_launch": design,
                     "design_bytes_per_stream": "|delta| + |R| + 3 |V| (R image with R's CRC, COPY "
                                                "sources, output, the output CRC re-read)",
                     "avg_launch_ms": round(dec_ms, 4),
                     "timed_launches_sampled": f"events on every {every}th timed step ({slots} launches)",
                     "stage_ms": {k: round(v, 4) for k, v in stages.items()},
                     "path_bytes_per_step": alg,
                     "path_achieved": round(alg / step_s / 1e9, 2),
                     "path_frac": round(alg / step_s / 1e9 / HBM_PEAK_GBS, 5)},
        "cpu_baseline": None,
        "lib_sha16": lib_sha16(),
    }
    yield line
    plan.close()
    del ref, ver, out, d_dev, out_len, status
    torch.cuda.empty_cache()


E2E_PAIRS, E2E_CHUNK_PAIRS = 16384, 1024


def bench_e2e(args, R, dg, ctx, stream):
    """The PCIe-inclusive rate (north_star): 16384 C2
    pairs (4 x the C2 batch, 2 GiB of R + V) in pinned host memory, encoded
    host to host by dg_encode_pipelined (1024-pair chunks, two in flight: H2D
    of chunk i+1 and D2H of chunk i-1's delta bytes overlap the encode of
    chunk i; main.c:249-292 per pair in the reference).  value = sum(|R|+|V|)
    / wall time of one call (median of K calls after a warm-up call); beside
    it the H2D-only rate of the same pinned arenas."""
    import ctypes as C
    torch = R.torch
    npg, L, rate, q, seed_base = CONFIGS["c2"][:5]
    n = E2E_PAIRS
    ref_d = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    ver_d = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    ctx.check(dg.lib.dg_synth_edit_pairs_device(ctx.handle, ref_d.data_ptr(), ver_d.data_ptr(), n, L, seed_base,
                                                int(rate * L + 0.5), stream.cuda_stream), "synth")
    torch.cuda.synchronize()
    ref_h = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    ver_h = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    ref_h.copy_(ref_d)
    ver_h.copy_(ver_d)
    p = 16
    cap = n * (35 + L + (L // p) * (22 - p))   # the plan's output bound per pair (onepass)
    out_h = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
    L_ = dg._lib
    pa = (L_.Pair * n)(*[L_.Pair(i * L, L, i * L, L) for i in range(n)])
    offs = (C.c_uint64 * (n + 1))()
    st = (C.c_int32 * n)()
    o = L_.DiffOptions.make(q=q)
    chunk = 2 * L * E2E_CHUNK_PAIRS

    def call():
        ctx.check(dg.lib.dg_encode_pipelined(ctx.handle, 1, ref_h.data_ptr(), ver_h.data_ptr(), pa, n, C.byref(o),
                                             chunk, out_h.data_ptr(), cap, offs, st), "dg_encode_pipelined")

    call()   # plans, device buffers, pinned staging
    bad = sum(1 for i in range(n) if st[i])
    if bad:
        raise SystemExit(f"e2e_c2: {bad} pairs failed")
    # spot check: the same bytes as the device-resident C2 plan's (checked by
    # the parity suite) through the one-pair entry point
    ob = out_h.numpy()
    rh, vh = ref_h.numpy(), ver_h.numpy()
    for i in range(0, n, n // 4 + 1):
        want = dg.encode(rh[i * L:(i + 1) * L].tobytes(), vh[i * L:(i + 1) * L].tobytes(), "onepass", q=q)
        if ob[offs[i]:offs[i + 1]].tobytes() != want:
            raise SystemExit(f"e2e_c2: pair {i} differs from dg_encode")
    reps = max(3, min(args.steps, 7))
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        call()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    med = ts[len(ts) // 2]
    h2d = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            ref_d.copy_(ref_h, non_blocking=True)
            ver_d.copy_(ver_h, non_blocking=True)
        torch.cuda.synchronize()
        h2d.append(time.perf_counter() - t0)
    h2d.sort()
    in_bytes = 2 * n * L
    line = {
        "metric": "host-to-host delta-encode GiB/s (dg_encode_pipelined, pinned host arenas)",
        "value": round(in_bytes / med / 2**30, 3), "unit": "GiB/s", "n_gpus": 1, "calls": reps,
        "ms_per_call": round(med * 1e3, 3), "min_ms": round(ts[0] * 1e3, 3),
        "h2d_gibs": round(in_bytes / h2d[len(h2d) // 2] / 2**30, 3),
        "h2d_note": "R and V arenas pinned host -> device alone (torch copy_, one stream), median of 3",
        "config": {"workload": f"{n} C2 pairs (64 KiB, 1% edits, --table-size 1) host to host",
                   "pairs": n, "pair_bytes": L, "chunk_pairs": E2E_CHUNK_PAIRS,
                   "delta_bytes": int(offs[n])},
    }
    del ref_d, ver_d, ref_h, ver_h, out_h
    torch.cuda.empty_cache()
    return line


def prepare_config(name, args, R, dg, ctx, shard, stream):
    """The config's inputs, plan and a checked step; returns (measure,
    release): measure() runs the W warmup and K timed steps and returns the
    line, release() frees the config's device memory."""
    fn = bench_decode if CONFIGS[name][6] == "decode" else bench_encode
    g = fn(name, args, R, dg, ctx, shard, stream)
    next(g)
    return (lambda: next(g)), (lambda: next(g, None))


def run_config(name, args, R, dg, ctx, shard, stream, cpu=True):
    measure, release = prepare_config(name, args, R, dg, ctx, shard, stream)
    line = measure()
    release()
    if cpu:
        add_cpu_baseline(name, line, args, R)
    return line


def add_cpu_baseline(name, line, args, R):
    if R.world == 1 and R.rank == 0 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(name)


# ───────────────────────────── the printed line ─────────────────────────────

LINE_MAX = 4000   # bytes: the driver keeps only the tail of stdout


def _cpu_short(cb):
    if not cb:
        return None
    out = {k: cb[k] for k in ("value", "unit", "cores", "kind") if k in cb}
    smp = cb.get("sample", "")
    out["sample"] = smp.split(" (times")[0][:220]
    if cb.get("single_thread"):
        out["single_thread"] = cb["single_thread"]["value"]
    for k in ("nproc", "affinity_cpus"):
        if cb.get(k) is not None:
            out[k] = cb[k]
    if cb.get("full_host_upper_bound"):
        out["full_host_upper_bound"] = cb["full_host_upper_bound"]["value"]
    return out


def _roof_short(r):
    keys = ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic", "avg_launch_ms",
            "algorithmic_bytes_per_launch", "path_achieved", "path_frac", "path_traffic", "path_traffic_ratio")
    out = {k: r[k] for k in keys if k in r}
    if r.get("traffic") and r.get("algorithmic_bytes_per_launch"):
        out["traffic_ratio"] = round(r["traffic"] / r["algorithmic_bytes_per_launch"], 3)
    if r.get("traffic") is None and str(r.get("traffic_source") or "").startswith("stale"):
        out["traffic_stale"] = True   # the committed PMC summary is of another library build
    return out


def also_entry(line):
    """One config of the run in a few numbers (the full line is in the file)."""
    if "roofline" not in line:   # the host-to-host line (bench_e2e)
        if line.get("error"):
            return {"value": None, "error": line["error"], "metric": "e2e"}
        return {"value": line["value"], "ms_per_call": line["ms_per_call"], "h2d_gibs": line["h2d_gibs"],
                "metric": "e2e"}
    r = line["roofline"]
    e = {"value": line["value"], "ms_per_step": line["ms_per_step"], "kernel_ms": r.get("avg_launch_ms"),
         "frac": r.get("frac"), "path_frac": r.get("path_frac")}
    if r.get("path_traffic_ratio"):
        e["path_traffic_ratio"] = r["path_traffic_ratio"]
    if r.get("traffic") and r.get("algorithmic_bytes_per_launch"):
        e["traffic_ratio"] = round(r["traffic"] / r["algorithmic_bytes_per_launch"], 3)
    cb = line.get("cpu_baseline")
    if cb:
        e["cpu"] = cb["value"]
    if line["metric"] != LINE_METRIC:
        e["metric"] = "decode" if "decode" in line["metric"] else line["metric"]
    return e


LINE_METRIC = "delta-encode GiB/s (device-resident batched pairs) at 1/2/4/8 MI355X"


def compact_line(line, also, full_path):
    """The headline as the driver parses it: the BASELINE metric on its config
    with roofline and cpu_baseline, `also` one short object per config,
    at most LINE_MAX bytes; every other field is in `full_path`."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "untimed_steps", "ms_per_step",
            "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "lib_sha16")
    out = {k: line[k] for k in keep if k in line}
    cfg = line["config"]
    out["config"] = {k: cfg[k] for k in ("workload", "name", "algorithm", "pairs_per_gpu", "pairs_total",
                                         "pair_bytes", "q", "parallelism") if k in cfg}
    out["roofline"] = _roof_short(line["roofline"])
    out["cpu_baseline"] = _cpu_short(line.get("cpu_baseline"))
    if also:
        out["also"] = {k: also_entry(v) for k, v in also.items()}
    out["full"] = full_path
    txt = json.dumps(out, separators=(",", ":"))
    for drop in ("path_frac", "kernel_ms", "metric"):   # stay inside the driver's tail
        if len(txt) <= LINE_MAX:
            break
        for e in out.get("also", {}).values():
            e.pop(drop, None)
        txt = json.dumps(out, separators=(",", ":"))
    return txt


# ───────────────────────────── launch ───────────────────────────────────────

def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args) -> int:
    """N > 1 without WORLD_SIZE: run this script under torch.distributed.run
    (one rank per GPU) as a child process; nothing here touches the GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def refuse_ab_switches():
    """The product library reads no environment; the A/B builds do
    (make -C delta-compression_amd ab).  A measurement line is never printed
    with any of those switches, or a variant library, selected."""
    bad = sorted(k for k in os.environ if k.startswith("DG_"))
    if bad:
        raise SystemExit(f"bench.py: refusing to measure with A/B switches set: {bad} "
                         "(scripts/ab_bench.py runs A/B comparisons)")


def dry_run(args, world, rank):
    """Launcher check on the CPU (gloo): ranks come up, the orchestration of
    the timed step runs on synthetic sizes; no GPU is touched, value is null."""
    import torch
    import torch.distributed as dist
    shard = load_shard()
    if world > 1:
        dist.init_process_group("gloo")
    npg = CONFIGS[args.config][0]
    total = npg * world + (world - 1)   # deliberately unequal ranges
    ranges = shard.balanced_ranges([1] * total, world) if rank == 0 else None
    allr = shard.all_ranges(dist, ranges, world, rank, "cpu")
    lo, hi = allr[rank]
    gather = shard.SizeGather([b - a for a, b in allr], "cpu")
    sizes = torch.arange(lo, hi, dtype=torch.int64) + 26
    t0 = time.perf_counter()
    off = gather.global_offsets(gather(dist, sizes))
    elapsed = shard.max_over_ranks(dist, time.perf_counter() - t0, world, "cpu")
    ok = int(off[-1]) == sum(range(total)) + 26 * total
    # the job's bytes as the timed lines count them: every rank's own sum,
    # all-reduced (the ranges are unequal, so rank 0's bytes x world is not it)
    pair_bytes = [1000 * (1 + i % 7) for i in range(total)]
    bytes_rank = sum(pair_bytes[lo:hi])
    bytes_job = shard.sum_over_ranks(dist, bytes_rank, world, "cpu")
    ok = ok and bytes_job == sum(pair_bytes)
    if rank == 0:
        print(json.dumps({"metric": "launcher dry run (no GPU, no encode)", "value": None,
                          "n_gpus": world, "steps": 0, "warmup": 0, "ranges": allr,
                          "index_ok": ok, "elapsed_s": elapsed, "bytes_job": bytes_job,
                          "bytes_expected": sum(pair_bytes), "bytes_rank0_x_world": bytes_rank * world}),
              flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0 if ok else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--also", default="c3,c4,c5,c5o,c6,c2_defq,c3s,c3s_chain,c4o,c4o_chain",
                    help="extra configs measured in the same run, reported under 'also' "
                         "('none' to skip)")
    ap.add_argument("--pairs", type=int, default=0, help="override pairs per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", dest="e2e", action="store_false",
                    help="skip the host-to-host line (also.e2e_c2: dg_encode_pipelined, 16384 pinned C2 pairs)")
    ap.add_argument("--full-out", default=os.path.join(ROOT, "gpurun_out", "bench_full.json"),
                    help="where the full detail of every line goes (the printed line is compact)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher/orchestration check on the CPU over gloo (no GPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        sys.exit(dry_run(args, world, rank))
    refuse_ab_switches()

    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    R = Rank(world, rank, local, dist, torch)
    dg = load_product()
    shard = load_shard()
    ctx = dg.Context(local)
    stream = torch.cuda.Stream()

    # The headline config first, then the other lines, then the CPU baselines
    # (host only).  A GPU leaving ~300 ms of idle runs ~40 C2 steps ~15 %
    # slow (profiles/r04_fresh_plan_c2.json); each line's own untimed steps
    # (the checked step, the stage-profile pass, W warmup: `untimed_steps`)
    # cover that, and the headline measured first reads the same as measured
    # last (C2 1734 / 1720 alone vs 1721 last, one box, round 4).
    extras = [c for c in args.also.split(",") if c and c != "none" and c != args.config]
    head_measure, head_release = prepare_config(args.config, args, R, dg, ctx, shard, stream)
    line = head_measure()
    head_release()
    also, release = {}, None
    for name in extras:
        if release:
            release()
        measure, release = prepare_config(name, args, R, dg, ctx, shard, stream)
        also[name] = measure()
    if release:
        release()
    if args.e2e and world == 1 and args.config == "c2":
        # (only beside the C2 headline, and a box without the
        # pinned memory reports the failure in the line instead of aborting)
        try:
            also["e2e_c2"] = bench_e2e(args, R, dg, ctx, stream)
        except Exception as e:  # noqa: BLE001
            torch.cuda.synchronize()
            also["e2e_c2"] = {"value": None, "error": f"{type(e).__name__}: {e}"[:200]}
    add_cpu_baseline(args.config, line, args, R)
    for name in extras:
        add_cpu_baseline(name, also[name], args, R)
    if rank == 0:
        full = dict(line, also=also) if also else line
        path = args.full_out
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(full, f, indent=1)
        print(f"bench.py: every field of every line in {path}", file=sys.stderr, flush=True)
        print(compact_line(line, also or None, os.path.relpath(path, ROOT)), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
