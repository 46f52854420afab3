#!/bin/bash
# Same-box A/B over kernel switch bits of the ab build:
# [AB_STEPS=K] scripts/ab_bits.sh TAG "0x0 0x400 ..." "c5 c5o" [rounds]
set -o pipefail
O=gpurun_out/$1
BS=$2
CS=${3:-c5}
RS=${4:-2}
mkdir -p $O
export TMPDIR=/tmp
for r in $(seq $RS); do
 for b in $BS; do
  for c in $CS; do
   DG_LIB_VARIANT=ab DG_DEBUG_BITS=$b timeout -k 10 200 python scripts/ab_bench.py --config $c --steps ${AB_STEPS:-10} --warmup ${AB_WARMUP:-2} > $O/$b.$c.$r.json 2> $O/$b.$c.$r.err || { echo "$b $c rc=$?"; tail -5 $O/$b.$c.$r.err; exit 1; }
   python3 -c "import json; d=json.loads(open('$O/$b.$c.$r.json').read().strip().splitlines()[-1]); print('$r $b $c', d['value'], 'ms', d['ms_per_step'], 'dom', d['roofline']['stage_ms'])"
  done
 done
done
