#!/bin/bash
# C5 same-box A/B: base (previous commit) vs the working tree's A/B build
set -o pipefail
O=gpurun_out/c5ab
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do for v in base ab; do
  DG_LIB_VARIANT=$v timeout -k 10 200 python scripts/ab_bench.py --config c5 --steps 50 --warmup 10 > $O/$v.$r.json 2> $O/$v.$r.err || { echo "$v rc=$?"; tail -5 $O/$v.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$v.$r.json').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$v', d['value'], d['ms_per_step'], 'decode', s.get('decode'))"
done; done
