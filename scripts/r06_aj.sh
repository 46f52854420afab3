#!/bin/bash
# round 6 session aj: c4o / c4o_chain order within one bench process
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06aj
mkdir -p $O
for order in "c4o_chain c4o" "c4o c4o_chain" "c3 c4o_chain"; do
  set -- $order
  timeout -k 10 400 python3 bench.py --config $1 --also $2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --full-out $O/$1_$2.json > $O/$1_$2.line 2> $O/$1_$2.err || { echo fail; tail -5 $O/$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$1_$2.json')); print('first $1', d['value'], 'then', {k: v['value'] for k, v in d['also'].items()})"
done
