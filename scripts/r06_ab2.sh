#!/bin/bash
# round 6 session ab2: fully routed batches as plain runs between member
# probes, the routed chain after the CRC pass (product) vs HEAD (vp)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ab2
mkdir -p $O
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_route_hint.py tests/test_gpu_auto_offdiag.py tests/test_gpu_shift.py tests/test_gpu_members_adversarial.py > $O/tests.log 2>&1 || { echo tests fail; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash scripts/r06_ab.sh r06ab2 "c3s c3s_chain c4o c4o_chain c3 c6" "prod vp" 2 || exit 1
