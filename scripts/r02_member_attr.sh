#!/bin/bash
# Member kernel (C3) time attribution: timing variants that skip parts of the
# verification (wrong verdicts: timing only), then the PMC instruction mix.
set -o pipefail
O=gpurun_out/mattr
mkdir -p $O
export TMPDIR=/tmp
for v in ab skipfp skipa skiplong skipshort; do
  DG_LIB_VARIANT=$v timeout -k 10 200 python scripts/ab_bench.py --config c3 --steps 10 --warmup 2 > $O/$v.json 2> $O/$v.err || { echo "$v rc=$?"; tail -5 $O/$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$v', d['value'], 'members', s.get('members'), 'diff', s.get('diff'), 'ser', s.get('serialize+join'))"
done
bash scripts/pmc_kernel.sh $O/pmc member_chunk_kernel "--config c3 --also none --steps 2 --warmup 1 --no-cpu-baseline" > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc.log; exit 1; }
cat $O/pmc.log | tail -40
