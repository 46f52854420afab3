#!/bin/bash
# round 6 session h2: decode A/B (dtail0, dec5), onepass A/B (noprio, win3584,
# CRC rows pass at priority 1 / 2), member serialiser waves per CU (mser8 /
# mser12 dense, msp16 / msp32 sparse); vp = the product's flags as a variant
set -o pipefail
export TMPDIR=/tmp
bash scripts/r06_ab.sh r06h/ab "c5 c5o" "vp dtail0 dec5" 2 || exit 1
bash scripts/r06_ab.sh r06h/ab "c2 c3s_chain c4o_chain c3s" "vp noprio win3584 crcp1 crcp2" 2 || exit 1
bash scripts/r06_ab.sh r06h/ab "c3 c6" "vp mser8 mser12 msp16 msp32" 2 || exit 1
