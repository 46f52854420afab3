#!/bin/bash
# round 6: onepass16 at C2 — phase profile, refill share, four PMC census passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipelined.py tests/test_gpu_serialize_tiles.py > $O/tests.log 2>&1 || { echo tests fail; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 120 env DG_LIB_VARIANT=prof python scripts/onepass_phases.py --config c2 > $O/phases_c2.json 2> $O/phases_c2.err || { echo phases fail; tail $O/phases_c2.err; exit 1; }
timeout -k 10 120 env DG_LIB_VARIANT=refill python scripts/refill_prof.py --config c2 > $O/refill_c2.json 2> $O/refill_c2.err || { echo refill fail; tail $O/refill_c2.err; exit 1; }
bash scripts/pmc_census.sh $O/census c2 "onepass16|crc_rows|serialize_wave" || exit 1
cat $O/phases_c2.json $O/refill_c2.json $O/census/summary.txt
