#!/bin/bash
# round 6 final session: GPU suite, the driver's default bench command, kernel
# traces of every config, PMC traffic of the dominant kernels and of whole steps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 $T > $O/tests.log 2>&1 || { echo tests fail; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python3 bench.py --full-out $O/bench_default_full.json > $O/bench_default_line.json 2> $O/bench_default.err || { echo bench fail; tail -5 $O/bench_default.err; exit 1; }
cut -c1-400 $O/bench_default_line.json
bash scripts/profile_round.sh r06 ks || exit 1
bash scripts/profile_round.sh r06 pmc || exit 1
bash scripts/profile_round.sh r06 path c2 c3 c4 c6 c2_defq || exit 1
