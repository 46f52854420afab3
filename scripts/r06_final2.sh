#!/bin/bash
# round 6 final session 2: PMC traffic of each config's dominant kernel(s) and
# of every kernel of a step (path), for the final library build
set -o pipefail
export TMPDIR=/tmp
bash scripts/profile_round.sh r06 pmc || exit 1
bash scripts/profile_round.sh r06 path c2 c3 c4 c6 c2_defq || exit 1
