#!/bin/bash
# What the CRC costs a step: the A/B build with the CRC beside the
# differencing (default), after it (DG_SERIAL_CRC=1) and not at all
# (DG_SKIP_CRC=1, header CRCs wrong: an upper bound on any CRC fusion).
set -o pipefail
O=gpurun_out/crcb
mkdir -p $O
for r in 1 2; do
 for c in c2 c3; do
  for m in default serial skip; do
   E=""; [ $m = serial ] && E="DG_SERIAL_CRC=1"; [ $m = skip ] && E="DG_SKIP_CRC=1"
   env DG_LIB_VARIANT=ab $E timeout -k 10 200 python scripts/ab_bench.py --config $c --steps 20 --warmup 3 > $O/$m.$c.$r.json 2> $O/$m.$c.$r.err || { echo "$m $c rc=$?"; tail -3 $O/$m.$c.$r.err; exit 1; }
   python3 -c "import json; d=json.loads(open('$O/$m.$c.$r.json').read().strip().splitlines()[-1]); print('$r $c $m', d['value'], d['ms_per_step'], d['roofline']['stage_ms'])"
  done
 done
done
