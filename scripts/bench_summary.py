"""Print one line per config of a bench.py JSON output (headline + "also")."""
import json
import sys

for line in open(sys.argv[1]):
    line = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    rows = [("headline", d)] + list(d.get("also", {}).items())
    for name, x in rows:
        r = x.get("roofline") or {}
        cpu = (x.get("cpu_baseline") or {}).get("value")
        print(f"{name:10s} {x['value']:9.2f} {x['unit']} {x['ms_per_step']:9.4f} ms "
              f"{r.get('kernel')} {r.get('avg_launch_ms')} frac={r.get('frac')} "
              f"path_frac={r.get('path_frac')} cpu={cpu}")
