#!/bin/bash
# GPU-box session: parity tests then the driver's default bench command.
# usage: scripts/r03_check.sh TAG
set -o pipefail
TAG=${1:-x}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread > $O/$TAG.tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/$TAG.tests.log; exit 1; }
tail -2 $O/$TAG.tests.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/$TAG.bench.json 2> $O/$TAG.bench.err || { echo "bench rc=$?"; tail -20 $O/$TAG.bench.err; exit 1; }
python3 scripts/bench_summary.py $O/$TAG.bench.json
if [ -n "$PHASES" ]; then
  for c in $PHASES; do
    DG_LIB_VARIANT=prof timeout -k 10 300 python3 scripts/onepass_phases.py --config $c --pairs 2048 > $O/$TAG.phases_$c.json 2>&1 || { echo "phases $c rc=$?"; tail -5 $O/$TAG.phases_$c.json; exit 1; }
    echo "$c"; cat $O/$TAG.phases_$c.json
  done
fi
