#!/bin/bash
# Parity tests on the product library, then a same-box A/B of variant
# libraries.  usage: VARIANTS="base x" CONFIGS="c2 c3s_chain" scripts/tests_then_ab.sh TAG [rounds]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$NOTESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/$1.tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/$1.tests.log; exit 1; }
tail -2 gpurun_out/$1.tests.log
fi
AB_STEPS=${AB_STEPS:-10} AB_WARMUP=${AB_WARMUP:-2} bash scripts/ab_multi.sh $1 "$VARIANTS" "$CONFIGS" ${2:-2}
