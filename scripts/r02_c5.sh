#!/bin/bash
# C5 iteration: decode tests, C5 bench line, decode phase counters (in-place).
set -o pipefail
O=gpurun_out/c5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode_order.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "decode or inplace or c5 or order" > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --config c5 --also none --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['config']['name'], d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['stage_ms'])"
DG_LIB_VARIANT=prof timeout -k 10 200 python scripts/decode_phases.py --inplace > $O/phases.json 2> $O/phases.err || { echo "phases rc=$?"; tail -5 $O/phases.err; exit 1; }
cat $O/phases.json
