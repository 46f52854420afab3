#!/bin/bash
# A/B bench lines over the A/B build (make -C delta-compression_amd ab, which
# reads the DG_* measurement switches; the product library reads none and
# bench.py refuses to print a line with any of them set).
# Each argument is "ENV=VAL ... -- bench args" (quoted).
# usage: scripts/ab.sh TAG "DG_FUSED=1 -- --config c2" "-- --config c2" ...
set -o pipefail
TAG=$1; shift
O=gpurun_out
mkdir -p $O
i=0
for spec in "$@"; do
  envs=${spec%%--*}
  args=${spec#*--}
  i=$((i+1))
  env DG_LIB_VARIANT=ab $envs timeout -k 10 300 python scripts/ab_bench.py $args > $O/$TAG.$i.json 2> $O/$TAG.$i.err \
    || { echo "run $i ($spec) rc=$?"; tail -5 $O/$TAG.$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/$TAG.$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$spec'.ljust(40), d['value'], d['ms_per_step'], r.get('stage_ms'))"
done
