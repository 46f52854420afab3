#!/usr/bin/env python3
"""Per-phase duration profile of the dominant kernel from the rocprofv3 kernel
trace of scripts/fresh_plan.py (phases are separated by synth marker launches).
usage: scripts/fresh_plan_read.py TRACE_DIR [kernel_regex] > summary.json"""
import csv
import glob
import json
import os
import re
import sys

d = sys.argv[1]
kre = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"onepass16_kernel<false, false>|member_chunk_kernel")
tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
phases, cur = [], None
for r in rows:
    n = r["Kernel_Name"]
    if "synth_random_kernel" in n:   # inputs, then one marker before each phase
        cur = []
        phases.append(cur)
        continue
    if cur is not None and kre.search(n):
        cur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
out = {}
for name, ms in zip("ABCD", phases[-4:]):
    if not ms:
        continue
    out[name] = {"dispatches": len(ms), "first_10": round(sum(ms[:10]) / 10, 4),
                 "10_to_40": round(sum(ms[10:40]) / len(ms[10:40]), 4), "last_40": round(sum(ms[-40:]) / 40, 4),
                 "per_dispatch": [round(x, 4) for x in ms]}
json.dump(out, sys.stdout, indent=1)
print()
for k, v in out.items():
    print(k, {a: b for a, b in v.items() if a != "per_dispatch"}, file=sys.stderr)
