#!/bin/bash
# round 6 session ak: c4o_chain first in a process, product vs the table pool
# allocated twice (trealloc)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ak
mkdir -p $O
for v in prod trealloc prod trealloc; do
  vv=$v; [ $v = prod ] && vv=""
  timeout -k 10 400 env DG_LIB_VARIANT=$vv python3 scripts/ab_bench.py --config c4o_chain --steps 10 --warmup 2 > $O/$v.json 2> $O/$v.err || { echo fail; tail -5 $O/$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
