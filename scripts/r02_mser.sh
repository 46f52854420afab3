#!/bin/bash
# member serialiser: persistent waves per CU (8 / 16 / 24), C3
set -o pipefail
O=gpurun_out/mser
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do for v in ab ms8 ms24; do
  DG_LIB_VARIANT=$v timeout -k 10 200 python scripts/ab_bench.py --config c3 --steps 10 --warmup 3 > $O/$v.$r.json 2> $O/$v.$r.err || { echo "$v rc=$?"; tail -5 $O/$v.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$v.$r.json').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$v', d['value'], d['ms_per_step'], 'ser', s.get('serialize+join'))"
done; done
