#!/bin/bash
# round 6 session e: GPU suite, then the pipelined serialisers A/B (product vs both
# serialisers as in round 5 (ser5) vs the round-5 library), the four-chain correcting
# build (corr4), and the kernel times from rocprofv3 traces (csv)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 $T > $O/tests.log 2>&1 || { echo tests fail; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/r06_ab.sh r06e/ab "c2 c3 c4 c6" "prod ser5 corr4" 2 || exit 1
for v in prod ser5; do
  vv=$v; [ $v = prod ] && vv=""
  for c in c2 c3; do
  timeout -k 10 200 env DG_LIB_VARIANT=$vv rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${v}_$c -o run -- python3 scripts/ab_bench.py --config $c --steps 20 --warmup 5 > $O/prof_${v}_$c.log 2>&1 || { echo "prof $v fail"; tail -5 $O/prof_${v}_$c.log; exit 1; }
  f=$(find $O/prof_${v}_$c -name "*kernel_stats.csv" | head -1); echo "== $v $c"; cut -d, -f1-4 $f | head -6
  done
done
