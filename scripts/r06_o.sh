#!/bin/bash
# round 6 session o: member serialiser with DMAs two jobs ahead (three ring
# slots; mser2a: 13 waves per CU as the LDS allows, mser2b: the default 16
# launched) vs the product's flags (vp); member parity tests on mser2a first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 env DG_LIB_VARIANT=mser2a $T -k "c3 or c6 or member or serial" > $O/tests_mser2a.log 2>&1 || { echo tests fail; tail -40 $O/tests_mser2a.log; exit 1; }
tail -1 $O/tests_mser2a.log
bash scripts/r06_ab.sh r06o/ab "c3 c6 c3s" "vp mser2a mser2b" 2 || exit 1
