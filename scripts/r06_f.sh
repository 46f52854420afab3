#!/bin/bash
# round 6 session f: GPU suite on the product (hand-counted serialize_run restored,
# member pipeline kept), A/B product vs member serialiser of round 5 (mser0) vs
# round-5 library, kernel stats; per-pair placement of the onepass kernel at C2
# (pairtime build), decode phase counters at C5 (prof build), PMC calibration
# classes (stream8 / dma4 added)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 $T > $O/tests.log 2>&1 || { echo tests fail; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/r06_ab.sh r06f/ab "c2 c3 c6" "prod mser0 r05" 2 || exit 1
for v in prod r05; do
  vv=$v; [ $v = prod ] && vv=""
  for c in c2 c3; do
  timeout -k 10 200 env DG_LIB_VARIANT=$vv rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${v}_$c -o run -- python3 scripts/ab_bench.py --config $c --steps 20 --warmup 5 > $O/prof_${v}_$c.log 2>&1 || { echo "prof $v fail"; tail -5 $O/prof_${v}_$c.log; exit 1; }
  f=$(find $O/prof_${v}_$c -name "*kernel_stats.csv" | head -1); echo "== $v $c"; grep -E "serialize|onepass16_kernel<false, false>|member_chunk" $f | cut -d, -f1-4
  done
done
timeout -k 10 200 env DG_LIB_VARIANT=pairtime python3 scripts/pair_time.py --config c2 > $O/pair_time_c2.json 2> $O/pair_time.err || { echo pairtime fail; tail -20 $O/pair_time.err; exit 1; }
cut -c1-1500 $O/pair_time_c2.json
timeout -k 10 200 env DG_LIB_VARIANT=prof python3 scripts/decode_phases.py --inplace > $O/decode_phases_c5.json 2> $O/decode_phases.err || { echo decphase fail; tail -20 $O/decode_phases.err; exit 1; }
cut -c1-1500 $O/decode_phases_c5.json
bash scripts/profile_round.sh r06f calib || exit 1
python3 scripts/profile_collect.py r06f > $O/collect.log 2>&1; tail -3 $O/collect.log
cp profiles/r06f_pmc_calib.json $O/ 2>/dev/null
python3 -c "import json; d=json.load(open('$O/r06f_pmc_calib.json'))['classes']; [print(k, v['bytes_per_fetch_kib'], v['bytes_per_write_kib']) for k,v in d.items()]"
