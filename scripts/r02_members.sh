#!/bin/bash
# GPU iteration for the member path: full onepass parity + bench lines + same-box A/B vs the plain chain
set -o pipefail
O=gpurun_out/${1:-mem}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in ab; do for c in c2 c3; do
  DG_LIB_VARIANT=$v timeout -k 10 200 python scripts/ab_bench.py --config $c --steps 10 --warmup 2 > $O/$v.$c.json 2> $O/$v.$c.err || { echo "$v $c rc=$?"; tail -5 $O/$v.$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$v.$c.json').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$v $c', d['value'], s)"
  DG_NO_MEMBERS=1 DG_LIB_VARIANT=$v timeout -k 10 200 python scripts/ab_bench.py --config $c --steps 10 --warmup 2 > $O/$v.$c.nm.json 2> $O/$v.$c.nm.err || { echo "$v $c nm rc=$?"; tail -5 $O/$v.$c.nm.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$v.$c.nm.json').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$v $c nomembers', d['value'], s)"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --also c3 --steps 10 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof rc=$?"; tail -5 $O/prof.log; exit 1; }
find $O/prof -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-150 | head -14
