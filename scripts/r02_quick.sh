#!/bin/bash
# Quick GPU iteration: onepass parity subset, C2 + C3 bench lines, C3 phase counters.
set -o pipefail
O=gpurun_out/${1:-q}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "onepass or golden or c3 or c2 or pool" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --also c3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
for x in [d]+list(d.get('also',{}).values()):
    print(x['config']['name'], x['value'], x['ms_per_step'], x['roofline']['stage_ms'])"
DG_LIB_VARIANT=prof timeout -k 10 300 python scripts/onepass_phases.py --config c3 > $O/c3.phases.json 2> $O/c3.phases.err || { echo "phases rc=$?"; tail $O/c3.phases.err; exit 1; }
cat $O/c3.phases.json
DG_LIB_VARIANT=prof timeout -k 10 300 python scripts/onepass_phases.py --config c2 > $O/c2.phases.json 2> $O/c2.phases.err || { echo "phases rc=$?"; tail $O/c2.phases.err; exit 1; }
cat $O/c2.phases.json
