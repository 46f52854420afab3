#!/bin/bash
# round 6 session k: path-level PMC traffic (every kernel of a step) of C2, C3, C4, c6
set -o pipefail
export TMPDIR=/tmp
bash scripts/profile_round.sh r06p path c2 c3 c4 c6 || exit 1
