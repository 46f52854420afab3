#!/bin/bash
# round 6 session af: member serialiser staged at the output's alignment
# (product) vs HEAD (vp): member GPU tests first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06af
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 400 $T tests > $O/tests.log 2>&1 || { echo tests fail; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/r06_ab.sh r06af "c3 c6" "prod vp" 3 || exit 1
