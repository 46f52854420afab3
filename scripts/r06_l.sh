#!/bin/bash
# round 6 session l: member plans raise the CRC rows pass to issue priority 1
# once the member kernel is done (crcflag) vs the product's flags (vp)
set -o pipefail
export TMPDIR=/tmp
bash scripts/r06_ab.sh r06l/ab "c3 c6 c3s c4o c2" "vp crcflag" 2 || exit 1
