#!/bin/bash
# round 6 session c: refill cache-warming A/B (touch2048/touch4096 vs product), the refill share with
# warming, and rocprof kernel stats of C2 for the product and the round-5 library (the serialiser)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 env DG_LIB_VARIANT=touch2048 $T > $O/tests_touch.log 2>&1 || { echo tests fail; tail -30 $O/tests_touch.log; exit 1; }
tail -1 $O/tests_touch.log
bash scripts/r06_ab.sh r06c/ab "c2 c3s_chain" "prod touch2048 touch4096" 2 || exit 1
timeout -k 10 120 env DG_LIB_VARIANT=touchrefill python scripts/refill_prof.py --config c2 > $O/refill_touch_c2.json 2> $O/refill_touch_c2.err || { echo refill fail; tail $O/refill_touch_c2.err; exit 1; }
cat $O/refill_touch_c2.json
for v in prod r05; do
  vv=$v; [ $v = prod ] && vv=""
  timeout -k 10 200 env DG_LIB_VARIANT=$vv rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 scripts/ab_bench.py --config c2 --steps 40 --warmup 5 > $O/prof_$v.log 2>&1 || { echo "prof $v fail"; tail -5 $O/prof_$v.log; exit 1; }
  f=$(find $O/prof_$v -name "*kernel_stats.csv" | head -1); echo "== $v"; cut -d, -f1-4 $f | head -8
done
