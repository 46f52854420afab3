#!/bin/bash
# round 6 session ag: plain serialiser placed by its own look-back (no scan
# kernel; product) vs HEAD (vp): GPU suite first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ag
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 400 $T tests > $O/tests.log 2>&1 || { echo tests fail; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/r06_ab.sh r06ag "c2 c2_defq c4 c3s" "prod vp" 3 || exit 1
