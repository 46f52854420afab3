#!/bin/bash
# round 6 session w: two commands per lane in the decode's flat batches
# (dec2: 128 commands per batch, one round of batches per 4 KiB window at C5)
# vs one (vp); decode tests on dec2 first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 env DG_LIB_VARIANT=dec2 $T -k "decode or apply or inplace or c5 or parity or many" > $O/tests_dec2.log 2>&1 || { echo tests fail; tail -40 $O/tests_dec2.log; exit 1; }
tail -1 $O/tests_dec2.log
bash scripts/r06_ab.sh r06w/ab "c5 c5o" "vp dec2" 3 || exit 1
