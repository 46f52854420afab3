#!/bin/bash
# round 6 session i: GPU suite with both CRCs computed by the onepass waves
# for plain plans (onepass16_crc_kernel); A/B product vs noopcrc (the CRC
# rows pass beside onepass16_kernel, as before); CRC rows pass at issue
# priority 1 beside the member / correcting kernels (crcp1) vs vp
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 $T > $O/tests.log 2>&1 || { echo tests fail; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/r06_ab.sh r06i/ab "c2 c2_defq" "prod noopcrc" 3 || exit 1
bash scripts/r06_ab.sh r06i/ab "c3 c6 c3s c4o c4" "vp crcp1" 2 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 scripts/ab_bench.py --config c2 --steps 20 --warmup 5 > $O/prof_c2.log 2>&1 || { echo "prof fail"; tail -5 $O/prof_c2.log; exit 1; }
f=$(find $O/prof_c2 -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 $f | head -8
