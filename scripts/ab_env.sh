#!/bin/bash
# Same-box A/B of the A/B build's environment switches on one config:
#   ENVS="DG_CORR_CRC=wide DG_CORR_CRC=fused" CONFIG=c4 scripts/ab_env.sh TAG [rounds]
# (make -C delta-compression_amd ab first; "-" = no switch)
set -o pipefail
O=gpurun_out/$1
mkdir -p $O
export TMPDIR=/tmp
for r in $(seq ${2:-2}); do
for e in $ENVS; do
  tag=$(echo "$e" | tr '=/' '__')
  env DG_LIB_VARIANT=ab $( [ "$e" != "-" ] && echo "$e" ) timeout -k 10 200 python scripts/ab_bench.py --config ${CONFIG:-c2} --steps ${AB_STEPS:-20} --warmup ${AB_WARMUP:-5} > $O/$tag.$r.json 2> $O/$tag.$r.err || { echo "$e rc=$?"; tail -5 $O/$tag.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$tag.$r.json').read().strip().splitlines()[-1]); print('$r $e', d['value'], d['ms_per_step'], d['roofline']['stage_ms'], d['roofline'].get('stage_ms_profile',{}).get('crc64'))"
done
done
