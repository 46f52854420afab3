#!/bin/bash
# GPU-box A/B session: parity tests, then single-config bench lines and
# (PHASES) onepass phase profiles.  usage: CONFIGS="c2 c3s" PHASES="c3s_chain" scripts/r03_quick.sh TAG
set -o pipefail
TAG=${1:-x}
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread > $O/$TAG.tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/$TAG.tests.log; exit 1; }
tail -2 $O/$TAG.tests.log
fi
for c in $CONFIGS; do
  timeout -k 10 300 python3 bench.py --config $c --also none --steps ${STEPS:-10} --warmup ${WARMUP:-3} --no-cpu-baseline > $O/$TAG.$c.json 2> $O/$TAG.$c.err || { echo "bench $c rc=$?"; tail -20 $O/$TAG.$c.err; exit 1; }
  python3 scripts/bench_summary.py $O/$TAG.$c.json
done
for c in $PHASES; do
  DG_LIB_VARIANT=prof timeout -k 10 300 python3 scripts/onepass_phases.py --config $c --pairs 2048 > $O/$TAG.phases_$c.json 2>&1 || { echo "phases $c rc=$?"; tail -5 $O/$TAG.phases_$c.json; exit 1; }
  echo "$c"; grep -v amdgpu.ids $O/$TAG.phases_$c.json
done
