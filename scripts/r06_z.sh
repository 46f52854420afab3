#!/bin/bash
# round 6 session z: member plans' chains after the CRC pass has ended
# (DG_CRC_FIRST=1 DG_CHAIN_JOIN=1) vs beside it; c3s routes every pair to
# the plain chain, C3 / c6 none
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06z
mkdir -p $O
for r in 1 2; do
 for v in base first join; do
  case $v in base) E="";; first) E="DG_CRC_FIRST=1";; join) E="DG_CRC_FIRST=1 DG_CHAIN_JOIN=1";; esac
  for c in c3s c3 c6; do
   env DG_LIB_VARIANT=ab $E timeout -k 10 200 python scripts/ab_bench.py --config $c --steps 6 --warmup 2 > $O/$v.$c.$r.json 2> $O/$v.$c.$r.err || { echo "$v $c failed"; tail -5 $O/$v.$c.$r.err; exit 1; }
   python3 -c "import json; d=json.loads(open('$O/$v.$c.$r.json').read().strip().splitlines()[-1]); print('$r $v $c', d['value'], 'ms', d['ms_per_step'], 'dom', d['roofline']['stage_ms'])"
  done
 done
done
