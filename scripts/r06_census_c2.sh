#!/bin/bash
# round 6: the GPU suite (product, then the winlim variant), A/B of the
# window-limited diagonal batch, and onepass16 at C2 — phase profile, refill
# share, four PMC census passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 $T > $O/tests.log 2>&1 || { echo tests fail; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 env DG_LIB_VARIANT=winlim $T > $O/tests_winlim.log 2>&1 || { echo winlim tests fail; tail -30 $O/tests_winlim.log; exit 1; }
tail -2 $O/tests_winlim.log
for r in 1 2; do
 for v in "" winlim winlim1k; do
  for c in c2 c3s_chain; do
   timeout -k 10 200 env DG_LIB_VARIANT=$v python scripts/ab_bench.py --config $c --steps 20 --warmup 3 > $O/ab.$v.$c.$r.json 2> $O/ab.$v.$c.$r.err || { echo "ab $v $c rc=$?"; tail -3 $O/ab.$v.$c.$r.err; exit 1; }
   python3 -c "import json; d=json.loads(open('$O/ab.$v.$c.$r.json').read().strip().splitlines()[-1]); print('$r', '$v'.ljust(9), '$c'.ljust(10), d['value'], d['ms_per_step'], d['roofline']['stage_ms'])"
  done
 done
done
timeout -k 10 120 env DG_LIB_VARIANT=prof python scripts/onepass_phases.py --config c2 > $O/phases_c2.json 2> $O/phases_c2.err || { echo phases fail; tail $O/phases_c2.err; exit 1; }
timeout -k 10 120 env DG_LIB_VARIANT=refill python scripts/refill_prof.py --config c2 > $O/refill_c2.json 2> $O/refill_c2.err || { echo refill fail; tail $O/refill_c2.err; exit 1; }
bash scripts/pmc_census.sh $O/census c2 "onepass16|crc_rows|serialize_wave" || exit 1
cat $O/phases_c2.json $O/refill_c2.json $O/census/summary.txt
