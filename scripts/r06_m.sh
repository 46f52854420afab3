#!/bin/bash
# round 6 session m: CRC rows pass beside onepass as 16-byte pieces in one
# 4-wave block per CU (crcwide) vs 8-byte pieces in two blocks (vp)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 env DG_LIB_VARIANT=crcwide $T -k "crc or c2 or parity" > $O/tests_crcwide.log 2>&1 || { echo tests fail; tail -40 $O/tests_crcwide.log; exit 1; }
tail -1 $O/tests_crcwide.log
bash scripts/r06_ab.sh r06m/ab "c2 c2_defq" "vp crcwide" 3 || exit 1
