#!/bin/bash
# round 6 session j: census of onepass16_crc_kernel at C2 (CRCs in the onepass waves)
set -o pipefail
export TMPDIR=/tmp
bash scripts/pmc_census.sh gpurun_out/r06j/census c2 "onepass16" || exit 1
cat gpurun_out/r06j/census/summary.txt
