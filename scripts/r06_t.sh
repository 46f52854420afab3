#!/bin/bash
# round 6 session t: the cost of the CRC stream's fork / join events at C2
# (DG_NO_FORKJOIN=1: timing bound only, header CRCs unordered) and of the
# CRC itself (DG_SKIP_CRC=1), product flags as a variant (vp)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
run() {   # name config env...
  local n=$1 c=$2; shift 2
  timeout -k 10 300 env DG_LIB_VARIANT=vp "$@" python scripts/ab_bench.py --config $c --steps 40 --warmup 5 > $O/$n.$c.json 2> $O/$n.$c.err || { echo "$n $c fail"; tail -3 $O/$n.$c.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.$c.json').read().strip().splitlines()[-1]); print('$n'.ljust(12), '$c'.ljust(8), d['value'], d['ms_per_step'], d['roofline']['stage_ms'])"
}
for r in 1 2 3; do
  run vp.$r c2 || exit 1
  run nofj.$r c2 DG_NO_FORKJOIN=1 || exit 1
  run skip.$r c2 DG_SKIP_CRC=1 || exit 1
done
