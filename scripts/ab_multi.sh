#!/bin/bash
# Same-box A/B over several variant libraries: [AB_STEPS=K AB_WARMUP=W] scripts/ab_multi.sh TAG "v1 v2 ..." "c2 c3" [rounds]
# (variants: make -C delta-compression_amd variant V=.. VFLAGS=.., or scripts/build_variant_from.sh REV NAME)
set -o pipefail
O=gpurun_out/$1
VS=$2
CS=${3:-c2 c3}
RS=${4:-2}
mkdir -p $O
export TMPDIR=/tmp
for r in $(seq $RS); do
 for v in $VS; do
  for c in $CS; do
   DG_LIB_VARIANT=$v timeout -k 10 200 python scripts/ab_bench.py --config $c --steps ${AB_STEPS:-10} --warmup ${AB_WARMUP:-2} > $O/$v.$c.$r.json 2> $O/$v.$c.$r.err || { echo "$v $c rc=$?"; tail -5 $O/$v.$c.$r.err; exit 1; }
   python3 -c "import json; d=json.loads(open('$O/$v.$c.$r.json').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; p=d['roofline'].get('stage_ms_profile',{}); print('$r $v $c', d['value'], 'ms', d['ms_per_step'], 'dom', s, 'crc', p.get('crc64'))"
  done
 done
done
