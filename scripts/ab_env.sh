#!/bin/bash
# Same-box A/B over one measurement switch of the ab build:
# [AB_STEPS=K] scripts/ab_env.sh TAG VAR "v1 v2 ..." "c3s c4o" [rounds]
set -o pipefail
O=gpurun_out/$1
VAR=$2
VS=$3
CS=${4:-c2}
RS=${5:-2}
mkdir -p $O
export TMPDIR=/tmp
for r in $(seq $RS); do
 for v in $VS; do
  for c in $CS; do
   env DG_LIB_VARIANT=${AB_LIB:-ab} $VAR=$v timeout -k 10 200 python scripts/ab_bench.py --config $c --steps ${AB_STEPS:-10} --warmup ${AB_WARMUP:-2} > $O/$v.$c.$r.json 2> $O/$v.$c.$r.err || { echo "$v $c rc=$?"; tail -5 $O/$v.$c.$r.err; exit 1; }
   python3 -c "import json; d=json.loads(open('$O/$v.$c.$r.json').read().strip().splitlines()[-1]); print('$r $VAR=$v $c', d['value'], 'ms', d['ms_per_step'], 'dom', d['roofline']['stage_ms'])"
  done
 done
done
