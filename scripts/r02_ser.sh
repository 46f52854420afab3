#!/bin/bash
# Serialiser iteration: encode parity tests, then same-box A/B tile-parallel vs wave-per-pair.
set -o pipefail
O=gpurun_out/ser
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do for c in c2 c4; do for sw in 0 1; do
  DG_SER_WAVE=$sw DG_LIB_VARIANT=ab timeout -k 10 200 python scripts/ab_bench.py --config $c --steps 50 --warmup 10 > $O/$c.$sw.$r.json 2> $O/$c.$sw.$r.err || { echo "$c $sw rc=$?"; tail -5 $O/$c.$sw.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$c.$sw.$r.json').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$c ser_wave=$sw', d['value'], d['ms_per_step'], 'diff', s.get('diff'), 'ser', s.get('serialize+join'))"
done; done; done
