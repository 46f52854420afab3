#!/bin/bash
# A/B bench lines: each argument is "ENV=VAL ... -- bench args" (quoted).
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
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline $args > $O/$TAG.$i.json 2> $O/$TAG.$i.err \
    || { echo "run $i ($spec) rc=$?"; tail -5 $O/$TAG.$i.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/$TAG.$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$spec'.ljust(40), d['value'], d['ms_per_step'], r.get('stage_ms'))"
done
