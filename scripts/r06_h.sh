#!/bin/bash
# round 6 session h: GPU suite on the product (issue priority by progress,
# one-round-trip partial chunks in the decode); decode A/B (dtail0 = round 5's
# partial-chunk copy, dec5 = five-bit CRC tables in the decode); onepass A/B
# (noprio; win3584; CRC rows pass at issue priority 1 / 2); vp = the product's
# flags built as a variant (A/B switches compiled in, as in the others)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 $T > $O/tests.log 2>&1 || { echo tests fail; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 env DG_LIB_VARIANT=dec5 $T -k "decode or apply or inplace" > $O/tests_dec5.log 2>&1 || { echo tests dec5 fail; tail -40 $O/tests_dec5.log; exit 1; }
tail -1 $O/tests_dec5.log
timeout -k 10 200 env DG_LIB_VARIANT=prof python3 scripts/decode_phases.py --inplace > $O/decode_phases_c5.json 2> $O/decode_phases.err || { echo decphase fail; tail -20 $O/decode_phases.err; exit 1; }
cut -c1-900 $O/decode_phases_c5.json
bash scripts/r06_ab.sh r06h/ab "c5 c5o" "vp dtail0 dec5" 2 || exit 1
bash scripts/r06_ab.sh r06h/ab "c2 c3s_chain c4o_chain c3s" "vp noprio win3584 crcp1 crcp2" 2 || exit 1
