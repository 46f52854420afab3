#!/bin/bash
# nibble-table CRC: C5 (in-decode CRC, product build) and the encode CRC A/B (variant nib vs ab)
set -o pipefail
O=gpurun_out/nib
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode_order.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
DG_LIB_VARIANT=nib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "crc or golden" > $O/tests_nib.log 2>&1 || { echo "nib tests rc=$?"; tail -30 $O/tests_nib.log; exit 1; }
tail -1 $O/tests_nib.log
for r in 1 2; do for c in c5 c2 c4 c3; do for v in ab nib; do
  [ $c = c5 ] && [ $v = nib ] && continue
  DG_LIB_VARIANT=$v timeout -k 10 200 python scripts/ab_bench.py --config $c --steps 20 --warmup 5 > $O/$v.$c.$r.json 2> $O/$v.$c.$r.err || { echo "$v $c rc=$?"; tail -5 $O/$v.$c.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$v.$c.$r.json').read().strip().splitlines()[-1]); s=d['roofline']['stage_ms']; print('$v $c', d['value'], d['ms_per_step'], s)"
done; done; done
