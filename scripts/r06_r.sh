#!/bin/bash
# round 6 session r: eight byte-table pieces per batch (72 VGPRs) vs four (product flags, vp)
set -o pipefail
export TMPDIR=/tmp
bash scripts/r06_ab.sh r06r/ab "c2 c2_defq c4" "vp pf8" 3 || exit 1
