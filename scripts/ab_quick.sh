#!/bin/bash
# Same-box A/B: the A/B build of the working tree (ab) against a baseline
# variant (default: base), configs c2 and c3, alternating, 2 rounds.
set -o pipefail
O=gpurun_out/${1:-ab}
B=${2:-base}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
 for v in $B ab; do
  for c in c2 c3; do
   DG_LIB_VARIANT=$v timeout -k 10 200 python scripts/ab_bench.py --config $c --steps 10 --warmup 2 > $O/$v.$c.$r.json 2> $O/$v.$c.$r.err || { echo "$v $c rc=$?"; tail -5 $O/$v.$c.$r.err; exit 1; }
   python3 -c "import json; d=json.loads(open('$O/$v.$c.$r.json').read().strip().splitlines()[-1]); print('$r $v $c', d['value'], d['roofline']['stage_ms'])"
  done
 done
done
