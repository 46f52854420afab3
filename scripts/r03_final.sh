#!/bin/bash
# Round-3 closing session on one box: parity tests, the driver's default
# bench command, rocprofv3 kernel-trace stats of the same command, and PMC
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of each line's dominant kernel.
# usage: scripts/r03_final.sh TAG
set -o pipefail
T=${1:-fin}
O=gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?"; tail -20 $O/bench.err; exit 1; }
python3 scripts/bench_summary.py $O/bench.json
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
bash scripts/pmc_traffic.sh r03 c2 onepass16_kernel > $O/p2.log 2>&1 || { echo "pmc c2 failed"; tail -5 $O/p2.log; exit 1; }
bash scripts/pmc_traffic.sh r03 c3s_chain onepass16_kernel > $O/p3s.log 2>&1 || { echo "pmc c3s failed"; tail -5 $O/p3s.log; exit 1; }
bash scripts/pmc_traffic.sh r03 c4o_chain onepass16_kernel > $O/p4o.log 2>&1 || { echo "pmc c4o failed"; tail -5 $O/p4o.log; exit 1; }
echo final done
