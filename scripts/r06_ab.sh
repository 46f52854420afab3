#!/bin/bash
# round 6 A/B: product vs named variant libraries over configs, R reps
# usage: scripts/r06_ab.sh OUT "cfg1 cfg2" "var1 var2" [reps]
set -o pipefail
O=gpurun_out/$1; CFGS=$2; VARS=$3; REPS=${4:-2}
mkdir -p $O
for r in $(seq 1 $REPS); do
 for v in $VARS; do
  vv=$v; [ "$v" = prod ] && vv=""
  for c in $CFGS; do
   timeout -k 10 300 env DG_LIB_VARIANT=$vv python scripts/ab_bench.py --config $c --steps 20 --warmup 3 > $O/ab.$v.$c.$r.json 2> $O/ab.$v.$c.$r.err || { echo "ab $v $c rc=$?"; tail -3 $O/ab.$v.$c.$r.err; exit 1; }
   python3 -c "import json; d=json.loads(open('$O/ab.$v.$c.$r.json').read().strip().splitlines()[-1]); print('$r', '$v'.ljust(9), '$c'.ljust(10), d['value'], d['ms_per_step'], d['roofline']['stage_ms'])"
  done
 done
done
