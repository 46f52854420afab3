#!/bin/bash
# round 6 session y: c3s routed chain vs the forced plain chain with and
# without the CRC pass (DG_SKIP_CRC=1: header CRCs wrong, timing only)
set -o pipefail
export TMPDIR=/tmp
AB_STEPS=6 bash scripts/ab_env.sh r06y DG_SKIP_CRC "0 1" "c3s c3s_chain" 2
