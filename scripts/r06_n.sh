#!/bin/bash
# round 6 session n: census of member_serialize_kernel at C3
set -o pipefail
export TMPDIR=/tmp
bash scripts/pmc_census.sh gpurun_out/r06n/census c3 "member_serialize" || exit 1
cat gpurun_out/r06n/census/summary.txt
