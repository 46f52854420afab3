#!/bin/bash
# round 6 session aa: the routed chain after the CRC pass when the plan's last
# run routed more than a round of pairs (product) vs HEAD (vp): member-mode
# GPU tests first, then c3s / c3 / c6 / c4o / c3s_chain
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06aa
mkdir -p $O
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 500 $T tests/test_gpu_auto_offdiag.py tests/test_gpu_shift.py tests/test_gpu_members_adversarial.py > $O/tests.log 2>&1 || { echo tests fail; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/r06_ab.sh r06aa "c3s c3 c6 c4o" "prod vp" 2 || exit 1
