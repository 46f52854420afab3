#!/bin/bash
# CRC lane-size iteration: CRC + decode tests, C5 and C2 bench lines.
set -o pipefail
O=gpurun_out/crc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode_order.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_pipelined.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --config c5 --also c2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
for x in [d]+list(d.get('also',{}).values()):
    print(x['config']['name'], x['value'], x['ms_per_step'], x['roofline']['frac'], x['roofline']['stage_ms'])"
