#!/bin/bash
# round 6 session v: the driver's default bench command twice more on the final
# library (run-to-run spread of the line) and the smoke entry point
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke fail; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for r in 1 2; do
  timeout -k 10 600 python3 bench.py --full-out $O/bench_full_$r.json > $O/bench_line_$r.json 2> $O/bench_$r.err || { echo bench fail; tail -5 $O/bench_$r.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_full_$r.json')); print('$r', d['value'], d['lib_sha16'], {k: v.get('value') for k, v in d['also'].items()})"
done
