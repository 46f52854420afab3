#!/bin/bash
# round 6 session ai: smoke and two more default bench runs on the final library
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ai
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo smoke fail; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 2 3; do
  timeout -k 10 600 python3 bench.py --full-out $O/bench_run$r.json > $O/bench_run${r}_line.json 2> $O/bench_run$r.err || { echo bench fail; tail -5 $O/bench_run$r.err; exit 1; }
  cut -c1-200 $O/bench_run${r}_line.json
done
