#!/bin/bash
# C2 iteration: onepass parity, then same-box A/B (base = previous commit) at C2 and C3.
set -o pipefail
O=gpurun_out/c2ab
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do for c in c2 c3; do for v in base ab; do
  DG_LIB_VARIANT=$v timeout -k 10 200 python scripts/ab_bench.py --config $c --steps 30 --warmup 5 > $O/$v.$c.$r.json 2> $O/$v.$c.$r.err || { echo "$v rc=$?"; tail -5 $O/$v.$c.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$v.$c.$r.json').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$v $c', d['value'], d['ms_per_step'], 'diff', s.get('diff'), 'members', s.get('members'))"
done; done; done
