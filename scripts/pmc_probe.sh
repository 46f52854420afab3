#!/bin/bash
# Counter passes for one kernel of one bench config (one pass per counter set,
# kernel trace only; MI355X_MICROARCH.md limits per block).
# usage: scripts/pmc_probe.sh OUTDIR CONFIG KERNEL_REGEX "set1" "set2" ...  (sets: space-free, comma-separated)
set -o pipefail
OUT=$1; CFG=$2; KRE=$3; shift 3
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for s in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc ${s//,/ } --kernel-include-regex "$KRE" --output-format csv \
      -d $OUT/p$i -o pmc -- python3 bench.py --config $CFG --also none --steps 3 --warmup 1 --no-cpu-baseline \
      > $OUT/p$i.log 2>&1 || { echo "pass $i ($s) failed rc=$?"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
out = sys.argv[1]
agg = {}
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        agg.setdefault((row["Kernel_Name"][:40], row["Counter_Name"]), []).append(float(row["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:40s} {c:32s} {sum(v)/len(v):16.1f} n={len(v)}")
PY
