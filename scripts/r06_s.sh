#!/bin/bash
# round 6 session s: the five-bit CRC rows pass beside member plans: four
# pieces per batch (f5pf4, 67 VGPRs) and the grid (DG_CRC_BLOCKS)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
run() {   # name variant config env...
  local n=$1 v=$2 c=$3; shift 3
  timeout -k 10 300 env DG_LIB_VARIANT=$v "$@" python scripts/ab_bench.py --config $c --steps 20 --warmup 3 > $O/$n.$c.json 2> $O/$n.$c.err || { echo "$n $c fail"; tail -3 $O/$n.$c.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.$c.json').read().strip().splitlines()[-1]); print('$n'.ljust(12), '$c'.ljust(8), d['value'], d['ms_per_step'], d['roofline']['stage_ms'])"
}
for r in 1 2; do
  for c in c6 c3 c3s; do
    run vp.$r vp $c || exit 1
    run f5pf4.$r f5pf4 $c || exit 1
    run vp768.$r vp $c DG_CRC_BLOCKS=768 || exit 1
  done
done
