#!/bin/bash
# The driver's round-end sequence on one box: every GPU test, smoke(), the default bench.
set -o pipefail
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -10 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'])
for k,v in d.get('also',{}).items(): print(k, v['value'], v['ms_per_step'], v['roofline']['frac'])
print('cpu', d['cpu_baseline']['value'], d['cpu_baseline']['single_thread']['value'])"
