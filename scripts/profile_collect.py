#!/usr/bin/env python3
"""Collect one profile session (scripts/profile_round.sh TAG, merged back
under gpurun_out/TAG) into profiles/:

  profiles/TAG_kernel_stats_<cfg>.csv   rocprofv3 --stats of the config run alone
  profiles/TAG_bench_<cfg>.json         the bench line of that same run
  profiles/TAG_pmc_calib.json           FETCH_SIZE / WRITE_SIZE per access class
  profiles/TAG_pmc_traffic_<cfg>.json   HBM bytes per launch of the dominant kernel(s)
  profiles/TAG_rooflines.md             HIP-event vs rocprof average per config

usage: scripts/profile_collect.py TAG
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KNOWN = {   # pmc_calib.cpp: bytes each kernel moves per launch (2 GiB buffers, 16 Mi lines)
    "stream16": 2 << 30, "dma16": 2 << 30, "stream8": 2 << 30, "dma4": 2 << 30, "rand16": (16 << 20) * 16, "rand4": (16 << 20) * 4,
    "store16": 2 << 30, "store16r": (16 << 20) * 16,
}
# the dominant kernel(s) of each line, as bench.py names them, and the
# rocprof names that make them up (one launch of each per step)
DOMINANT = {
    "onepass16_kernel": [r"onepass16_kernel<false, false>"],
    "member_chunk_kernel": [r"member_chunk_kernel"],
    "onepass16_kernel (member chain + routed plain chain)": [r"onepass16_kernel<true, false>",
                                                             r"onepass16_kernel<false, true>"],
    "correcting_build_kernel + correcting_scan_kernel": [r"correcting_build_lds_kernel", r"correcting_build_kernel",
                                                         r"correcting_scan_kernel"],
    "decode_kernel": [r"decode_kernel"],
}
# FETCH class of each dominant kernel's reads (pmc_calib factors apply per class)
FETCH_CLASS = {"onepass16_kernel": "dma16", "member_chunk_kernel": "dma16", "decode_kernel": "stream16",
               "correcting_build_kernel + correcting_scan_kernel": "stream16"}


# the access class of each kernel of a step (path-level traffic): the first
# pattern that matches names the pmc_calib class whose factor applies
PATH_CLASS = [(r"onepass16_kernel|member_chunk_kernel|onepass_kernel", "dma16"),
              (r"crc_rows_wide", "stream16"), (r"crc_rows_kernel", "stream8"),
              (r"correcting_build", "stream16"), (r"decode_kernel", "stream16")]
# (the serialisers mix 4-byte record loads, short unaligned payload reads and
# staged V rows: no one class; they take the x1 lower and x2 upper readings)
CALIB_DEFAULT = {"dma16": 2.0, "stream16": 2.0}


def stats_rows(path):
    rows = {}
    for r in csv.DictReader(open(path)):
        rows[r["Name"]] = r
    return rows


def counter(dirpath, name):
    """Per kernel name: mean per dispatch of counter `name` (KiB)."""
    per = {}
    for f in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == name:
                per.setdefault(row.get("Kernel_Name", ""), []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", tag)
    prof = os.path.join(ROOT, "profiles")
    table = ["| config | dominant kernel | HIP-event avg, timed steps (ms) | rocprof avg, all calls (ms) | rocprof calls | "
             "rocprof trace, last K dispatches (ms) | diff (trace vs events) |",
             "|---|---|---|---|---|---|---|"]
    # ── per-config kernel stats + bench line ──
    for d in sorted(glob.glob(os.path.join(src, "ks_*"))):
        if not os.path.isdir(d):
            continue
        cfg = os.path.basename(d)[3:]
        st = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
        full = os.path.join(d, "bench_full.json")
        if not st or not os.path.exists(full):
            print(f"{cfg}: incomplete", file=sys.stderr)
            continue
        shutil.copy(st[0], os.path.join(prof, f"{tag}_kernel_stats_{cfg}.csv"))
        shutil.copy(full, os.path.join(prof, f"{tag}_bench_{cfg}.json"))
        line = json.load(open(full))
        r = line["roofline"]
        kname = r["kernel"]
        rows = stats_rows(st[0])
        pats = DOMINANT.get(kname, [re.escape(kname)])
        tot_ns, calls = 0.0, []
        for p in pats:
            hit = [(n, x) for n, x in rows.items() if re.search(p, n)]
            for n, x in hit:
                tot_ns += float(x["AverageNs"])
                calls.append(int(x["Calls"]))
        rp = tot_ns / 1e6
        ev = r.get("avg_launch_ms") or 0.0
        # the timed steps are the last K dispatches of each dominant kernel
        k_steps = int(line.get("steps") or 0)
        tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        last = float("nan")
        if tr and k_steps:
            per = {}
            for row in csv.DictReader(open(tr[0])):
                for p in pats:
                    if re.search(p, row["Kernel_Name"]):
                        per.setdefault(p, []).append((int(row["Start_Timestamp"]),
                                                      (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6))
            last = sum(sum(x for _, x in sorted(v)[-k_steps:]) / k_steps for v in per.values()) if per else float("nan")
        diff = (last - ev) / ev if ev else float("nan")
        table.append(f"| {cfg} | {kname} | {ev:.4f} | {rp:.4f} | {'/'.join(map(str, calls))} | {last:.4f} | "
                     f"{100 * diff:+.1f} % |")
    # ── PMC calibration per access class ──
    calib = {}
    for k, nbytes in KNOWN.items():
        f, _ = counter(os.path.join(src, f"calib_{k}_FETCH_SIZE"), "FETCH_SIZE")
        w, _ = counter(os.path.join(src, f"calib_{k}_WRITE_SIZE"), "WRITE_SIZE")
        fk = sum(v for n, v in f.items() if k in n)
        wk = sum(v for n, v in w.items() if k in n)
        if fk or wk:
            calib[k] = {"known_bytes": nbytes, "fetch_kib": fk, "write_kib": wk,
                        "bytes_per_fetch_kib": nbytes / (fk * 1024) if fk else None,
                        "bytes_per_write_kib": nbytes / (wk * 1024) if wk else None}
    if calib:
        json.dump({"source": "scripts/micro/pmc_calib.cpp under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                             "(one counter per pass, kernel-include-regex per class)",
                   "classes": calib}, open(os.path.join(prof, f"{tag}_pmc_calib.json"), "w"), indent=1)
    # ── PMC traffic per config ──
    for d in sorted(glob.glob(os.path.join(src, "pmc_*_FETCH_SIZE"))):
        cfg = os.path.basename(d)[4:-len("_FETCH_SIZE")]
        f, nf = counter(d, "FETCH_SIZE")
        w, nw = counter(os.path.join(src, f"pmc_{cfg}_WRITE_SIZE"), "WRITE_SIZE")
        bj = os.path.join(src, f"pmc_{cfg}_FETCH_SIZE.json")
        bline = json.load(open(bj)) if os.path.exists(bj) else {}
        kname = bline.get("roofline", {}).get("kernel")
        # the line's dominant kernel(s) only: a pass may also hold other
        # kernels the include regex admits (c3s / c4o plain runs: the member
        # kernel and chains of the member-mode probes)
        pats = DOMINANT.get(kname)
        dom = (lambda k: any(re.search(p, k) for p in pats)) if pats else (lambda k: True)
        raw_f = sum(v for k, v in f.items() if dom(k)) * 1024
        raw_w = sum(v for k, v in w.items() if dom(k)) * 1024
        cls = FETCH_CLASS.get(kname, "dma16")
        fac = (calib.get(cls) or {}).get("bytes_per_fetch_kib") or 2.0
        # the table tier's random 16-byte loads: pmc_calib shows FETCH_SIZE
        # tallies 64 B per such load (4x its useful bytes); whether the line
        # moved is 64 or 128 B the counter cannot tell, so these configs carry
        # both readings: x1 (64-B requests) and x2 (as the streaming reads)
        table_tier = cfg in ("c3s", "c3s_chain", "c4o", "c4o_chain")
        if table_tier:
            cls, fac = "mixed: LDS-DMA windows + random 16-byte table loads", 1.0
        res = {"kernel": kname, "config": cfg, "lib_sha16": bline.get("lib_sha16"),
               "kernels": {k: {"fetch_kib": f.get(k), "write_kib": w.get(k),
                                                                 "dispatches": [nf.get(k), nw.get(k)]}
                                                             for k in sorted(set(f) | set(w))},
               "fetch_bytes_raw": raw_f, "write_bytes": raw_w,
               "fetch_class": cls, "fetch_factor": fac,
               "fetch_bytes_per_launch": raw_f * fac,
               "write_bytes_per_launch": raw_w,
               "hbm_bytes_per_launch": raw_f * fac + raw_w,
               "correction": f"FETCH_SIZE KiB x 1024 x {fac:.3f} ({cls}, profiles/{tag}_pmc_calib.json); "
                             "WRITE_SIZE KiB x 1024"}
        if cfg == "c4":
            # the LDS build streams R (x fac, as calibrated); the scan mixes
            # coalesced windows / extension steps with random index (4 B) and
            # seed-verify (16 B) loads, each tallied at 64 B: x1 and x2 readings
            scan = sum(v for k, v in f.items() if "correcting_scan" in k) * 1024
            rest = raw_f - scan
            res["kernels_fetch_class"] = {"build": cls, "scan": "mixed: coalesced windows + random index loads"}
            res["fetch_bytes_per_launch"] = rest * fac + scan
            res["hbm_bytes_per_launch"] = rest * fac + scan + raw_w
            res["hbm_bytes_upper"] = rest * fac + scan * 2.0 + raw_w
            res["correction"] = (f"build FETCH_SIZE x {fac:.3f} ({cls}); scan FETCH_SIZE x 1 (lower reading: "
                                 "random requests tallied at 64 B) and x 2 in hbm_bytes_upper; WRITE_SIZE x 1")
        if table_tier:
            res["hbm_bytes_upper"] = raw_f * 2.0 + raw_w
            res["correction"] = ("FETCH_SIZE KiB x 1024 x 1 (lower reading: every request 64 B as tallied); "
                                 "hbm_bytes_upper: x 2 (every request 128 B tallied at 64 B, as streaming reads); "
                                 "WRITE_SIZE KiB x 1024")
        json.dump(res, open(os.path.join(prof, f"{tag}_pmc_traffic_{cfg}.json"), "w"), indent=1)
    # ── path-level traffic: every kernel of a step (scripts/profile_round.sh path) ──
    if not calib:   # this session ran no calibration: the newest committed one
        cf = sorted(glob.glob(os.path.join(prof, "r*_pmc_calib.json")))
        if cf:
            calib = json.load(open(cf[-1]))["classes"]
    for d in sorted(glob.glob(os.path.join(src, "path_*_FETCH_SIZE"))):
        if not os.path.isdir(d):
            continue
        cfg = os.path.basename(d)[5:-len("_FETCH_SIZE")]
        f, nf = counter(d, "FETCH_SIZE")
        w, nw = counter(os.path.join(src, f"path_{cfg}_WRITE_SIZE"), "WRITE_SIZE")
        bj = os.path.join(src, f"path_{cfg}_FETCH_SIZE.json")
        bline = json.load(open(bj)) if os.path.exists(bj) else {}
        path_bytes = (bline.get("roofline") or {}).get("path_bytes_per_step")
        kern, lo, hi = {}, 0.0, 0.0
        for k in sorted(set(f) | set(w)):
            cls = next((c for p, c in PATH_CLASS if re.search(p, k)), None)
            fac = (calib.get(cls) or {}).get("bytes_per_fetch_kib") or CALIB_DEFAULT.get(cls, 1.0) if cls else 1.0
            fk = (f.get(k) or 0.0) * 1024
            wk = (w.get(k) or 0.0) * 1024
            k_lo = fk * fac + wk
            k_hi = fk * max(fac, 2.0) + wk
            lo += k_lo
            hi += k_hi
            kern[k] = {"fetch_kib": f.get(k), "write_kib": w.get(k), "dispatches": [nf.get(k), nw.get(k)],
                       "fetch_class": cls or "small / random (x1 lower, x2 upper)", "fetch_factor": round(fac, 4),
                       "hbm_bytes": int(k_lo), "hbm_bytes_upper": int(k_hi)}
        res = {"config": cfg, "lib_sha16": bline.get("lib_sha16"), "kernels": kern,
               "path_traffic_per_step": int(lo), "path_traffic_upper_per_step": int(hi),
               "path_bytes_per_step": path_bytes,
               "ratio": round(lo / path_bytes, 3) if path_bytes else None,
               "ratio_upper": round(hi / path_bytes, 3) if path_bytes else None,
               "correction": "per kernel: FETCH_SIZE KiB x 1024 x its access class's factor "
                             f"(profiles/{tag}_pmc_calib.json; classes without one x1), + WRITE_SIZE KiB x 1024; "
                             "upper: every FETCH at least x2",
               "command": f"rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE --kernel-include-regex dg:: --kernel-exclude-regex "
                          f"synth -- python3 bench.py --config {cfg} --also none --steps 5 --warmup 1"}
        json.dump(res, open(os.path.join(prof, f"{tag}_pmc_path_{cfg}.json"), "w"), indent=1)
        print("path", cfg, res["path_traffic_per_step"], res["ratio"], res["ratio_upper"])
    # ── fresh-plan warm-up: per-dispatch durations of each config's dominant
    #    kernel in launch order (the checked step, the profile pass, warmup, timed) ──
    warm = {}
    for d in sorted(glob.glob(os.path.join(src, "ks_*"))):
        cfg = os.path.basename(d)[3:]
        tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        full = os.path.join(d, "bench_full.json")
        if not tr or not os.path.exists(full):
            continue
        kname = json.load(open(full))["roofline"]["kernel"]
        pats = DOMINANT.get(kname, [re.escape(kname)])
        durs = []
        for row in csv.DictReader(open(tr[0])):
            if any(re.search(p, row["Kernel_Name"]) for p in pats[:1]):
                durs.append((int(row["Start_Timestamp"]), (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6))
        durs.sort()
        ms = [x for _, x in durs]
        if len(ms) >= 20:
            k = len(ms)
            warm[cfg] = {"dispatches": k, "first_10_ms": round(sum(ms[:10]) / 10, 4),
                         "dispatch_10_to_40_ms": round(sum(ms[10:40]) / max(len(ms[10:40]), 1), 4),
                         "last_20_ms": round(sum(ms[-20:]) / 20, 4),
                         "per_dispatch_ms": [round(x, 4) for x in ms]}
    if warm:
        json.dump(warm, open(os.path.join(prof, f"{tag}_warmup.json"), "w"), indent=1)
        for c, w in warm.items():
            print(c, {k: v for k, v in w.items() if k != "per_dispatch_ms"})
    open(os.path.join(prof, f"{tag}_rooflines.md"), "w").write(
        f"# {tag}: dominant-kernel time, HIP events (bench.py) vs rocprofv3 --stats of the same run\n\n"
        + "\n".join(table) + "\n")
    print("\n".join(table))
    if calib:
        print(json.dumps(calib, indent=1))


if __name__ == "__main__":
    main()
