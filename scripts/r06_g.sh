#!/bin/bash
# round 6 session g: onepass window 4 KiB (win4k), with the five-bit CRC row
# pass beside it (win4k5: both fit 16 waves + 2 CRC blocks per CU), the
# five-bit pass alone (crc5), issue priority by progress (prio); vprod = the
# product's flags built as a variant (the A/B switches compiled in, as in the others)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 env DG_LIB_VARIANT=win4k5 $T > $O/tests_win4k5.log 2>&1 || { echo tests fail; tail -40 $O/tests_win4k5.log; exit 1; }
tail -1 $O/tests_win4k5.log
timeout -k 10 200 env DG_LIB_VARIANT=prio_pt python3 scripts/pair_time.py --config c2 > $O/pair_time_prio_c2.json 2> $O/pair_time.err || { echo pairtime fail; tail -20 $O/pair_time.err; exit 1; }
cut -c1-700 $O/pair_time_prio_c2.json
bash scripts/r06_ab.sh r06g/ab "c2 c3s_chain c4o_chain c3" "vprod prio crc5 win4k win4k5" 2 || exit 1
