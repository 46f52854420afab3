#!/bin/bash
# One GPU-box session: parity tests, bench lines (C2 default, C2 serial CRC,
# C3, C4, C5), rocprofv3 kernel-trace stats of the default bench command and
# the FETCH/WRITE_SIZE passes of the dominant kernel.
# usage: scripts/gpu_check.sh TAG   (outputs under gpurun_out/TAG*)
set -o pipefail
TAG=${1:-x}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread > $O/$TAG.tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/$TAG.tests.log; exit 1; }
tail -2 $O/$TAG.tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/$TAG.c2.json 2> $O/$TAG.c2.err || { echo "bench c2 rc=$?"; tail $O/$TAG.c2.err; exit 1; }
cat $O/$TAG.c2.json
DG_SERIAL_CRC=1 timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/$TAG.c2s.json 2>&1 || { echo "bench c2 serial rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 1 > $O/$TAG.c3.json 2>&1 || { echo "bench c3 rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 1 > $O/$TAG.c4.json 2>&1 || { echo "bench c4 rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 > $O/$TAG.c5.json 2>&1 || { echo "bench c5 rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$TAG.prof -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/$TAG.prof.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
find $O/$TAG.prof -name '*kernel_stats.csv' -exec cat {} \;
bash scripts/pmc_traffic.sh $TAG c2 onepass16_kernel > $O/$TAG.pmct.log 2>&1 || { echo "pmc traffic rc=$?"; tail -5 $O/$TAG.pmct.log; exit 1; }
echo done
