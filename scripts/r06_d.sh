#!/bin/bash
# round 6 session d: rocprof kernel stats of C2 and C3 for the product and the round-5 library
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
for c in c2 c3; do
for v in prod r05; do
  vv=$v; [ $v = prod ] && vv=""
  timeout -k 10 300 env DG_LIB_VARIANT=$vv rocprofv3 --kernel-trace --stats -d $O/prof_${v}_$c -o run -- python3 scripts/ab_bench.py --config $c --steps 30 --warmup 5 > $O/prof_${v}_$c.log 2>&1 || { echo "prof $v $c fail"; tail -5 $O/prof_${v}_$c.log; exit 1; }
  f=$(find $O/prof_${v}_$c -name "*kernel_stats.csv" | head -1); echo "== $v $c"; cut -d, -f1-4 $f | head -7
done
done
