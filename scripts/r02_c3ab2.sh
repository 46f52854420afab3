#!/bin/bash
# C3 iteration with the adversarial member tests: parity, then same-box A/B (base = previous commit).
set -o pipefail
O=gpurun_out/c3ab2
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_members_adversarial.py tests/test_gpu_commands.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do for v in base ab; do
  DG_LIB_VARIANT=$v timeout -k 10 200 python scripts/ab_bench.py --config c3 --steps 10 --warmup 3 > $O/$v.$r.json 2> $O/$v.$r.err || { echo "$v rc=$?"; tail -5 $O/$v.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$v.$r.json').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$v', d['value'], d['ms_per_step'], 'members', s.get('members'), 'diff', s.get('diff'))"
done; done
