#!/bin/bash
# round 6 session u: the CRC rows pass beside onepass with two interleaved
# byte-table copies (half the bank conflicts) in one block per CU, PF 4 (nc2)
# or PF 8 (nc2pf8), vs the product's flags (vp); CRC tests on nc2pf8 first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 env DG_LIB_VARIANT=nc2pf8 $T -k "crc or c2 or parity" > $O/tests.log 2>&1 || { echo tests fail; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/r06_ab.sh r06u/ab "c2 c2_defq" "vp nc2 nc2pf8" 3 || exit 1
