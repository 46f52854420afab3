#!/bin/bash
# round 6 session g: onepass window 4 KiB (win4k), with the five-bit CRC row
# pass beside it (win4k5: both fit 16 waves + 2 CRC blocks per CU), the
# five-bit pass alone (crc5); GPU suite on win4k5 first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 env DG_LIB_VARIANT=win4k5 $T > $O/tests_win4k5.log 2>&1 || { echo tests fail; tail -40 $O/tests_win4k5.log; exit 1; }
tail -1 $O/tests_win4k5.log
bash scripts/r06_ab.sh r06g/ab "c2 c3s_chain c4o_chain" "prod crc5 win4k win4k5" 2 || exit 1
timeout -k 10 120 env DG_LIB_VARIANT=refill python scripts/refill_prof.py --config c2 > $O/refill_c2.json 2> $O/refill_c2.err && cat $O/refill_c2.json
