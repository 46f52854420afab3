#!/bin/bash
# round 6 session ae: code placement: HEAD (vp) vs HEAD with the unlaunched
# split serialiser's code in the object before the CRC kernels (padA)
set -o pipefail
export TMPDIR=/tmp
bash scripts/r06_ab.sh r06ae "c2" "vp padA split1" 3 || exit 1
