#!/bin/bash
# round 6 session ac: the serialiser split over 2 waves per pair (product) vs
# 1 (split1) vs 4 (split4): GPU suite on the product first
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ac
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests"
timeout -k 10 400 $T > $O/tests.log 2>&1 || { echo tests fail; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 env DG_LIB_VARIANT=split4 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests4.log 2>&1 || { echo tests4 fail; tail -40 $O/tests4.log; exit 1; }
tail -1 $O/tests4.log
bash scripts/r06_ab.sh r06ac "c2 c2_defq c4 c3s_chain" "prod split1 split4" 2 || exit 1
