#!/bin/bash
# round 6 session q: four byte-table pieces per batch in the CRC rows pass
# (product) vs two (pf2); CRC / C2 parity tests on the product first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 $T -k "crc or c2 or parity or correcting or c4" > $O/tests.log 2>&1 || { echo tests fail; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/r06_ab.sh r06q/ab "c2 c2_defq c4 c3" "vp pf2" 3 || exit 1
