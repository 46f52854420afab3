#!/bin/bash
# round 6 session x: c3s routed chain vs the forced plain chain under an
# occupancy cap (DG_OP_LDS_PAD: dynamic LDS per onepass16 block)
set -o pipefail
export TMPDIR=/tmp
AB_STEPS=6 bash scripts/ab_env.sh r06x DG_OP_LDS_PAD "0 2048 4096 8192" "c3s c3s_chain" 2
