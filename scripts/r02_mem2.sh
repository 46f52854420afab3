#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-mem2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash scripts/r02_iso.sh ${1:-mem2}/iso
for c in c2 c3; do
  timeout -k 10 200 python bench.py --config $c --also none --steps 10 --warmup 2 --no-cpu-baseline > $O/$c.json 2> $O/$c.err || { echo "$c rc=$?"; tail -5 $O/$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$c.json').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$c', d['value'], s)"
done
DG_MEMBERS=1 DG_LIB_VARIANT=prof timeout -k 10 120 python scripts/onepass_phases.py --config c3 > $O/c3.phases.json 2>&1 && tail -1 $O/c3.phases.json
