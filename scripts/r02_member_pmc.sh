#!/bin/bash
# PMC instruction mix of the member kernel at C3 (SQ counters; separate passes)
set -o pipefail
O=gpurun_out/mpmc
mkdir -p $O
bash scripts/pmc_kernel.sh $O/pmc member_chunk_kernel "--config c3 --also none --steps 2 --warmup 1 --no-cpu-baseline" > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc.log; exit 1; }
tail -30 $O/pmc.log
