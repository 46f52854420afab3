#!/bin/bash
# round 6 session b: GPU suite on the product, then A/B product vs round 5 (r05) and the
# correcting LDS-table variant (corrnb), and the correcting-build census at C4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 $T > $O/tests.log 2>&1 || { echo tests fail; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/r06_ab.sh r06b/ab "c2 c4 c3" "prod r05 corrnb" 2 || exit 1
bash scripts/pmc_census.sh $O/census c4 "correcting_build_lds|correcting_scan|crc_rows" || exit 1
cat $O/census/summary.txt
